/*
 * kvr_multi.hip — several GPUs behind one call, included by kvr_api.hip.
 *
 * The store's sorted segment list (engine.rs:51) is dealt round-robin: segment i -> context
 * i mod N.  Segments are independent parse units (framing never crosses files, engine.rs:80-85),
 * so every context replays its shard with kvr_replay on its own host thread and stream, with no
 * collective and no device-to-device traffic; the host gathers the shards.  The merge is exact:
 *   - tuples: a shard's output is in (its segment, offset) order, so the store's order
 *     (engine.rs:55-57 applies records segment by segment) is segment i's run taken from shard
 *     i mod N, for i ascending — an O(n) copy, seg_idx rewritten to the caller's index;
 *   - errors: the store's first error is the minimum (segment, offset) error over the shards
 *     (engine.rs:56 stops at the first one; what other shards found after it is never reached);
 *   - expected CRCs (the caller's manifest in store tuple order) are checked on the merged order.
 * Segments may be host bytes or resident in HBM (KVR_SEGS_ON_DEVICE: segment i on the device of
 * context i mod N, as a sharded store generated or kept in HBM holds them).  The live-index form
 * never reads key bytes on the host side from the segments: every shard exports the key bytes of
 * its per-key last records (kvr_live_keys), and the merge compares those.
 */
#include <thread>

// the last record of each key over t[0, n) (in (segment, offset) order; key i is kp[i], t[i].key_len
// bytes): live[i] = 1 iff t[i] is its key's last record and a SET.  Keys split by tag into one
// partition per thread; each partition keeps an open-addressing table of (tag << 32 | index).
static void fold_last_parallel(const uint8_t *const *kp, const kvr_tuple *t, size_t n, std::vector<uint8_t> &live) {
    live.assign(n, 0);
    if (n == 0) return;
    const uint32_t P = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    auto part = [P](uint32_t tag) { return (uint32_t)(((uint64_t)(tag * 0x9E3779B1u) * P) >> 32); };
    std::vector<std::vector<uint32_t>> idx(P);
    for (size_t i = 0; i < n; ++i) idx[part(t[i].key_tag)].push_back((uint32_t)i);   // each list in order
    std::vector<std::thread> th;
    for (uint32_t p = 0; p < P; ++p) {
        th.emplace_back([&, p]() {
            const std::vector<uint32_t> &L = idx[p];
            if (L.empty()) return;
            uint64_t cap = 16;
            while (cap < 2 * L.size()) cap <<= 1;
            constexpr uint64_t EMPTY = ~0ull;
            std::vector<uint64_t> slot(cap, EMPTY);
            const uint64_t mask = cap - 1;
            for (uint32_t i : L) {
                const kvr_tuple &x = t[i];
                const uint64_t tag = (uint64_t)x.key_tag << 32;
                for (uint64_t h = ((uint64_t)x.key_tag * 0x9E3779B97F4A7C15ull) >> 20;; ++h) {
                    uint64_t &sl = slot[h & mask];
                    if (sl == EMPTY) { sl = tag | i; break; }
                    if ((sl & 0xFFFFFFFF00000000ull) != tag) continue;
                    const kvr_tuple &y = t[(uint32_t)sl];
                    if (y.key_len == x.key_len && memcmp(kp[(uint32_t)sl], kp[i], x.key_len) == 0) {
                        sl = tag | i;   // later record wins (engine.rs:137, :141)
                        break;
                    }
                }
            }
            for (uint64_t sl : slot)
                if (sl != EMPTY && t[(uint32_t)sl].op == 0) live[(uint32_t)sl] = 1;
        });
    }
    for (auto &x : th) x.join();
}

struct kvr_mctx {
    std::vector<kvr_ctx *> c;
    kvr_multi_stats st{};
    // the key bytes of the last kvr_replay_live_multi output, packed in its order (kvr_multi_live_keys)
    std::vector<uint8_t> keys;
    std::vector<uint64_t> koff;
    bool keys_valid = false;
};

extern "C" {

int kvr_mctx_create(const int *devices, int n_devices, kvr_mctx **out) {
    if (!out || n_devices < 1 || !devices) return KVR_EINVAL;
    *out = nullptr;
    kvr_mctx *m = new kvr_mctx();
    for (int i = 0; i < n_devices; ++i) {
        kvr_ctx *c = nullptr;
        const int rc = kvr_ctx_create(devices[i], &c);
        if (rc != KVR_OK) {
            kvr_mctx_destroy(m);
            return rc;
        }
        m->c.push_back(c);
    }
    *out = m;
    return KVR_OK;
}

void kvr_mctx_destroy(kvr_mctx *m) {
    if (!m) return;
    for (kvr_ctx *c : m->c) kvr_ctx_destroy(c);
    delete m;
}

int kvr_mctx_size(const kvr_mctx *m) { return m ? (int)m->c.size() : 0; }

int kvr_last_multi_stats(const kvr_mctx *m, kvr_multi_stats *out) {
    if (!m || !out) return KVR_EINVAL;
    *out = m->st;
    return KVR_OK;
}

static int replay_multi(kvr_mctx *m, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
                        size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err, bool last);

int kvr_replay_multi(kvr_mctx *m, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
                     size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err) {
    return replay_multi(m, segs, n, flags, expected, n_expected, out, cap, n_out, err, false);
}

int kvr_replay_live_multi(kvr_mctx *m, const kvr_segment *segs, size_t n, uint32_t flags, kvr_tuple *out, size_t cap,
                          size_t *n_out, kvr_error *err) {
    return replay_multi(m, segs, n, flags, nullptr, 0, out, cap, n_out, err, true);
}

int kvr_multi_live_keys(const kvr_mctx *m, uint8_t *keys, uint64_t keys_cap, uint64_t *key_off, size_t off_cap,
                        uint64_t *key_bytes) {
    if (!m || !key_bytes || (keys_cap && !keys) || (off_cap && !key_off)) return KVR_EINVAL;
    if (!m->keys_valid) return KVR_EINVAL;
    *key_bytes = m->keys.size();
    if (m->keys.size() > keys_cap || m->koff.size() > off_cap) return KVR_CAPACITY;
    if (!m->keys.empty()) memcpy(keys, m->keys.data(), m->keys.size());
    memcpy(key_off, m->koff.data(), m->koff.size() * sizeof(uint64_t));
    return KVR_OK;
}

}  // extern "C"

// last: each shard reduces its tuples to every key's last record, tombstones included
// (kvr_replay_last: a DEL on one GPU may delete a key another GPU SET); the host
// merges the shards in (segment, offset) order and keeps each key's last record if it is a SET
static int replay_multi(kvr_mctx *m, const kvr_segment *segs, size_t n, uint32_t flags, const uint32_t *expected,
                        size_t n_expected, kvr_tuple *out, size_t cap, size_t *n_out, kvr_error *err, bool last) {
    if (!m || m->c.empty() || (!segs && n) || !n_out || (cap && !out)) return KVR_EINVAL;
    if (flags & ~KVR_SEGS_ON_DEVICE) return KVR_EINVAL;   // host output; segments on the host or on their shard's device
    if (err) memset(err, 0, sizeof(*err));
    *n_out = 0;
    memset(&m->st, 0, sizeof(m->st));
    m->keys_valid = false;
    m->keys.clear();
    m->koff.assign(1, 0);
    const uint32_t sflags = flags & KVR_SEGS_ON_DEVICE;
    for (size_t i = 1; i < n; ++i)
        if (segs[i].seg_id < segs[i - 1].seg_id) return KVR_EINVAL;   // caller sorts (engine.rs:51)
    const size_t N = m->c.size();
    m->st.n_shards = (uint32_t)N;
    if (n == 0) return KVR_OK;
    const auto t0 = std::chrono::steady_clock::now();

    std::vector<std::vector<kvr_segment>> sh(N);
    for (size_t i = 0; i < n; ++i) {
        sh[i % N].push_back(segs[i]);
        m->st.bytes_in += segs[i].len;
    }
    std::vector<std::vector<kvr_tuple>> tv(N);
    std::vector<std::vector<uint8_t>> kb(N);     // last: each shard's exported key bytes ...
    std::vector<std::vector<uint64_t>> ko(N);    // ... and their offsets (kvr_live_keys)
    std::vector<int> rc(N, KVR_OK);
    std::vector<kvr_error> er(N);
    std::vector<size_t> nn(N, 0);
    std::vector<double> dev_ms(N, 0.0);
    std::vector<std::thread> th;
    for (size_t r = 0; r < N; ++r) {
        if (sh[r].empty()) continue;
        th.emplace_back([&, r]() {
            uint64_t bytes = 0;
            for (const kvr_segment &s : sh[r]) bytes += s.len;
            size_t c = (size_t)(bytes / 256) + 4096 + sh[r].size();
            tv[r].resize(c);
            auto run = [&](size_t cc) {
                return last ? kvr_replay_last(m->c[r], sh[r].data(), sh[r].size(), sflags, tv[r].data(), cc, &nn[r], &er[r])
                            : kvr_replay(m->c[r], sh[r].data(), sh[r].size(), sflags, nullptr, 0, tv[r].data(), cc, &nn[r], &er[r]);
            };
            int x = run(c);
            if (x == KVR_CAPACITY) {   // rare: denser than one record per 256 B; replay again into the exact size
                c = nn[r];
                tv[r].resize(c);
                x = run(c);
            }
            if (last && x == KVR_OK) {   // the key bytes of the shard's per-key last records
                uint64_t nb = 0;
                ko[r].assign(nn[r] + 1, 0);
                x = kvr_live_keys(m->c[r], 0, nullptr, 0, ko[r].data(), ko[r].size(), &nb);
                if (x == KVR_CAPACITY || x == KVR_OK) {
                    kb[r].resize(nb + 1);
                    x = kvr_live_keys(m->c[r], 0, kb[r].data(), kb[r].size(), ko[r].data(), ko[r].size(), &nb);
                }
            }
            kvr_stats s;
            kvr_last_stats(m->c[r], &s);
            dev_ms[r] = s.ms_total;
            rc[r] = x;
        });
    }
    for (std::thread &t : th) t.join();
    for (size_t r = 0; r < N; ++r) {
        if (rc[r] < 0) return rc[r];
        m->st.ms_device_max = std::max(m->st.ms_device_max, dev_ms[r]);
    }

    // the store's first error: minimum (segment, offset) over the shards
    bool bad = false;
    kvr_error first{};
    for (size_t r = 0; r < N; ++r) {
        if (rc[r] != KVR_CORRUPTED) continue;
        kvr_error e = er[r];
        e.seg_idx = (uint32_t)(e.seg_idx * N + r);   // local index j of shard r is global j * N + r
        if (!bad || e.seg_idx < first.seg_idx || (e.seg_idx == first.seg_idx && e.rec_off < first.rec_off)) first = e;
        bad = true;
    }
    if (bad) {
        if (err) *err = first;
        m->st.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return KVR_CORRUPTED;
    }

    // merge: segment i's run from shard i mod N, in segment order
    std::vector<size_t> pos(N, 0);
    size_t o = 0;
    uint64_t fails = 0;
    if (last) {   // every shard's key-last records, merged, then the last record of each key overall
        size_t tot = 0;
        for (size_t r = 0; r < N; ++r) tot += nn[r];
        std::vector<kvr_tuple> mt;
        std::vector<const uint8_t *> kp;
        mt.reserve(tot);
        kp.reserve(tot);
        for (size_t i = 0; i < n; ++i) {
            const size_t r = i % N;
            const uint32_t j = (uint32_t)(i / N);
            size_t &p = pos[r];
            while (p < nn[r] && tv[r][p].seg_idx == j) {
                kp.push_back(kb[r].data() + ko[r][p]);
                kvr_tuple x = tv[r][p++];
                x.seg_idx = (uint32_t)i;
                mt.push_back(x);
            }
        }
        std::vector<uint8_t> live;
        fold_last_parallel(kp.data(), mt.data(), mt.size(), live);
        for (size_t i = 0; i < mt.size(); ++i) {
            if (!live[i]) continue;
            if (o < cap) out[o] = mt[i];
            m->keys.insert(m->keys.end(), kp[i], kp[i] + mt[i].key_len);
            m->koff.push_back(m->keys.size());
            ++o;
        }
        m->keys_valid = true;
        *n_out = o;
        m->st.n_records = o;
        m->st.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return o > cap ? KVR_CAPACITY : KVR_OK;
    }
    for (size_t i = 0; i < n; ++i) {
        const size_t r = i % N;
        const uint32_t j = (uint32_t)(i / N);
        const std::vector<kvr_tuple> &t = tv[r];
        size_t &p = pos[r];
        while (p < nn[r] && t[p].seg_idx == j) {
            kvr_tuple x = t[p++];
            x.seg_idx = (uint32_t)i;
            if (expected && o < n_expected && x.op == 0) {
                x.flags |= KVR_TF_VERIFIED;
                if (expected[o] != x.crc32) { x.flags |= KVR_TF_CRC_FAIL; ++fails; }
            }
            if (o < cap) out[o] = x;
            ++o;
        }
    }
    *n_out = o;
    m->st.n_records = o;
    m->st.n_crc_fail = fails;
    m->st.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return o > cap ? KVR_CAPACITY : KVR_OK;
}
