/*
 * kvr_host.cpp — host side of the drop-in (include/kvstore_host.h): discovery, the CPU
 * generator, the last-writer-wins fold and a KVStore mirror whose open() replays on the GPU.
 * Built with g++ into libkvhost.so, linked against libkvreplay.so.
 */
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kvreplay.h"
#include "../../include/kvstore_host.h"
#include "kvr_gen_common.h"

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

uint32_t crc32_update(uint32_t crc, const uint8_t *p, size_t n) {
    if (!crc_ready) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
            crc_table[i] = c;
        }
        crc_ready = true;
    }
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; ++i) c = (c >> 8) ^ crc_table[(c ^ p[i]) & 0xFFu];
    return ~c;
}

bool utf8_valid(const uint8_t *s, size_t n) {   // std::str::from_utf8 acceptance (valid or not)
    size_t i = 0;
    while (i < n) {
        const uint8_t b = s[i];
        if (b < 0x80) { ++i; continue; }
        int w = (b >= 0xC2 && b <= 0xDF) ? 2 : (b >= 0xE0 && b <= 0xEF) ? 3 : (b >= 0xF0 && b <= 0xF4) ? 4 : 0;
        if (!w || i + w > n) return false;
        const uint8_t c1 = s[i + 1];
        bool ok = (c1 & 0xC0) == 0x80;
        if (w == 3) ok = (b == 0xE0) ? (c1 >= 0xA0 && c1 <= 0xBF) : (b == 0xED) ? (c1 >= 0x80 && c1 <= 0x9F) : ok;
        if (w == 4) ok = (b == 0xF0) ? (c1 >= 0x90 && c1 <= 0xBF) : (b == 0xF4) ? (c1 >= 0x80 && c1 <= 0x8F) : ok;
        if (!ok) return false;
        for (int k = 2; k < w; ++k) if ((s[i + k] & 0xC0) != 0x80) return false;
        i += w;
    }
    return true;
}

struct KeyRef {   // key bytes inside a resident segment
    const uint8_t *p;
    uint32_t n;
    uint32_t tag;
};
struct KeyHash {
    size_t operator()(const KeyRef &k) const { return (size_t)k.tag * 0x9E3779B97F4A7C15ull; }
};
struct KeyEq {
    bool operator()(const KeyRef &a, const KeyRef &b) const { return a.n == b.n && memcmp(a.p, b.p, a.n) == 0; }
};

}  // namespace

struct kvs_store {
    std::string dir;
    std::vector<uint64_t> ids;
    std::vector<kvr_segment> segs;               // host bytes of every resident segment
    std::vector<std::pair<void *, uint64_t>> maps;   // kvs_open's mappings: one per segment file
                                                 // (mmap path) or the read arena (pread path)
    std::vector<void *> regs;                    // ranges registered for DMA (kvr_host_register)
    bool pinned = false;                         // every segment byte lies in a registered range
    std::vector<std::vector<uint8_t>> owned;     // segments written by kvs_compact
    // the index (index.rs:5-7 shape): live keys' final SETs and the table over them
    // (kvr_replay_index / kvr_index_find)
    std::vector<kvr_tuple> live;
    std::vector<uint32_t> slots;
    uint64_t total_bytes = 0;
    uint64_t active_id = 0;
    uint32_t open_flags = 0;
    kvs_open_stats ost{};
    void drop_arena() {
        for (void *r : regs) kvr_host_unregister(r);
        regs.clear();
        for (auto &m : maps) munmap(m.first, m.second);
        maps.clear();
        pinned = false;
    }
    ~kvs_store() { drop_arena(); }
};

extern "C" {

int kvh_parse_u64(const char *s, size_t n, uint64_t *out) {
    if (n == 0) return 0;
    size_t i = 0;
    if (s[0] == '+') {   // u64::from_str accepts one leading '+' (not alone)
        if (n == 1) return 0;
        i = 1;
    }
    uint64_t v = 0;
    for (; i < n; ++i) {
        const unsigned d = (unsigned char)s[i] - '0';
        if (d > 9) return 0;
        if (v > (UINT64_MAX - d) / 10) return 0;   // overflow -> Err
        v = v * 10 + d;
    }
    *out = v;
    return 1;
}

int kvh_gen_segment(const kvr_gen_params *p, uint64_t seg_no, uint8_t *buf, uint64_t cap, uint64_t *len_out,
                    uint32_t *expected, uint64_t exp_cap, uint64_t *n_rec_out) {
    if (!p || !len_out) return KVR_EINVAL;
    const uint64_t sbase = kvr_gen_sbase(p->seed, seg_no);
    uint64_t off = 0, i = 0;
    for (;; ++i) {   // size pass
        kvr_gen_rec r;
        kvr_gen_record(p, sbase, i, &r);
        const uint64_t sz = kvr_gen_rec_size(&r);
        if (off + sz > p->seg_bytes) break;
        off += sz;
    }
    *len_out = off;
    if (n_rec_out) *n_rec_out = i;
    if (!buf) return KVR_OK;
    if (off > cap || (expected && i > exp_cap)) return KVR_CAPACITY;
    uint64_t o = 0;
    for (uint64_t k = 0; k < i; ++k) {
        kvr_gen_rec r;
        kvr_gen_record(p, sbase, k, &r);
        uint8_t *q = buf + o;
        q[0] = (uint8_t)r.op;   // engine.rs:169 / :191
        q[1] = (uint8_t)KVR_GEN_KEY_LEN; q[2] = 0; q[3] = 0; q[4] = 0;
        kvr_gen_key(r.key_id, q + 5);
        if (r.op == 0) {
            uint8_t *v = q + 9 + KVR_GEN_KEY_LEN;
            q[5 + KVR_GEN_KEY_LEN] = (uint8_t)r.vlen;
            q[6 + KVR_GEN_KEY_LEN] = (uint8_t)(r.vlen >> 8);
            q[7 + KVR_GEN_KEY_LEN] = (uint8_t)(r.vlen >> 16);
            q[8 + KVR_GEN_KEY_LEN] = (uint8_t)(r.vlen >> 24);
            for (uint64_t j = 0; j < r.vlen; ++j) v[j] = kvr_gen_vbyte(r.vseed, j);
            if (expected) expected[k] = crc32_update(0, v, r.vlen);   // manifest before the fault
            if (r.flip_bit >= 0) v[(uint64_t)r.flip_bit >> 3] ^= (uint8_t)(1u << (r.flip_bit & 7));
        } else if (expected) {
            expected[k] = 0;
        }
        o += kvr_gen_rec_size(&r);
    }
    return KVR_OK;
}

int kvh_discover(const char *dir, uint64_t *ids, size_t cap, char *paths, size_t path_cap, size_t *n_out) {
    if (!dir || !n_out) return KVR_EINVAL;
    DIR *d = opendir(dir);
    if (!d) return KVR_EIO;
    std::vector<std::pair<uint64_t, std::string>> found;
    static const char pre[] = "segment-", suf[] = ".dat";
    while (struct dirent *e = readdir(d)) {
        const char *name = e->d_name;
        const size_t n = strlen(name);
        if (!utf8_valid(reinterpret_cast<const uint8_t *>(name), n)) continue;   // to_str() == None
        if (n < 8 || memcmp(name, pre, 8) != 0) continue;                          // engine.rs:40
        if (n < 4 || memcmp(name + n - 4, suf, 4) != 0) continue;
        if (n < 12) continue;
        uint64_t id;
        if (!kvh_parse_u64(name + 8, n - 12, &id)) continue;                       // engine.rs:43
        std::string full = std::string(dir) + "/" + name;                          // base_dir.join(name)
        found.emplace_back(id, full);
    }
    closedir(d);
    std::stable_sort(found.begin(), found.end(), [](const auto &a, const auto &b) {   // engine.rs:51
        return a.first != b.first ? a.first < b.first : a.second < b.second;
    });
    *n_out = found.size();
    if (found.size() > cap) return KVR_CAPACITY;
    size_t po = 0;
    for (size_t i = 0; i < found.size(); ++i) {
        if (ids) ids[i] = found[i].first;
        if (paths) {
            const size_t L = found[i].second.size() + 1;
            if (po + L > path_cap) return KVR_CAPACITY;
            memcpy(paths + po, found[i].second.c_str(), L);
            po += L;
        }
    }
    return KVR_OK;
}

uint64_t kvh_fold(const kvr_segment *segs, const kvr_tuple *t, size_t n, uint8_t *live, uint64_t *total_bytes) {
    std::unordered_map<KeyRef, size_t, KeyHash, KeyEq> last;
    last.reserve(n / 2 + 16);
    for (size_t i = 0; i < n; ++i) {
        const KeyRef k{segs[t[i].seg_idx].bytes + t[i].rec_off + 5, t[i].key_len, t[i].key_tag};
        auto it = last.find(k);
        if (it == last.end()) last.emplace(k, i);
        else it->second = i;                   // later record wins (engine.rs:137, :141)
    }
    if (live) memset(live, 0, n);
    uint64_t nk = 0, tb = 0;
    for (const auto &kv : last) {
        if (t[kv.second].op == 0) {
            if (live) live[kv.second] = 1;
            ++nk;
            tb += t[kv.second].val_len;
        }
    }
    if (total_bytes) *total_bytes = tb;
    return nk;
}

// Parallel fold: the last writer of a key is its maximal (segment, offset)
// record, so the keys can be split by hash into independent partitions.  Phase 1 counts each
// chunk's tuples per partition, phase 2 scatters the tuple indices partition-major (chunk order
// kept, so each partition stays in (segment, offset) order), phase 3 folds every partition into
// its own open-addressing table (key_tag as the hash, key bytes compared on a tag match).
uint64_t kvh_fold_parallel(const kvr_segment *segs, const kvr_tuple *t, size_t n, uint32_t n_threads,
                           uint8_t *live, uint64_t *total_bytes) {
    if (total_bytes) *total_bytes = 0;
    if (n == 0) return 0;
    if (n_threads == 0) n_threads = std::max(1u, std::thread::hardware_concurrency());
    n_threads = std::min<uint32_t>(n_threads, 256);
    if (n >= 0xFFFFFFFFull || n_threads == 1) return kvh_fold(segs, t, n, live, total_bytes);
    const uint32_t P = n_threads;                       // one partition per thread
    const size_t chunk = (n + P - 1) / P;
    auto part = [P](uint32_t tag) { return (uint32_t)(((uint64_t)(tag * 0x9E3779B1u) * P) >> 32); };
    std::vector<uint64_t> cnt((size_t)P * P, 0);         // cnt[chunk * P + partition]
    std::vector<std::thread> th;
    auto run = [&](auto fn) {
        th.clear();
        for (uint32_t w = 0; w < P; ++w) th.emplace_back(fn, w);
        for (auto &x : th) x.join();
    };
    run([&](uint32_t c) {
        const size_t a = std::min(n, c * chunk), b = std::min(n, a + chunk);
        uint64_t *h = &cnt[(size_t)c * P];
        for (size_t i = a; i < b; ++i) ++h[part(t[i].key_tag)];
    });
    std::vector<uint64_t> pstart(P + 1, 0), cur((size_t)P * P);
    for (uint32_t p = 0; p < P; ++p) {
        uint64_t s = pstart[p];
        for (uint32_t c = 0; c < P; ++c) { cur[(size_t)c * P + p] = s; s += cnt[(size_t)c * P + p]; }
        pstart[p + 1] = s;
    }
    std::vector<uint32_t> idx(n);
    run([&](uint32_t c) {
        const size_t a = std::min(n, c * chunk), b = std::min(n, a + chunk);
        uint64_t *o = &cur[(size_t)c * P];
        for (size_t i = a; i < b; ++i) idx[o[part(t[i].key_tag)]++] = (uint32_t)i;
    });
    if (live) memset(live, 0, n);
    std::vector<uint64_t> nk(P, 0), tb(P, 0);
    run([&](uint32_t p) {
        const uint64_t a = pstart[p], b = pstart[p + 1];
        if (a == b) return;
        uint64_t cap = 16;
        while (cap < 2 * (b - a)) cap <<= 1;
        // slot = key_tag << 32 | tuple index of the key's latest record: probes compare tags in
        // the table and touch the tuple and the key bytes only on a tag match
        constexpr uint64_t EMPTY = ~0ull;
        std::vector<uint64_t> slot(cap, EMPTY);
        const uint64_t mask = cap - 1;
        for (uint64_t j = a; j < b; ++j) {
            const uint32_t i = idx[j];
            const kvr_tuple &x = t[i];
            const uint64_t tag = (uint64_t)x.key_tag << 32;
            for (uint64_t h = ((uint64_t)x.key_tag * 0x9E3779B97F4A7C15ull) >> 20;; ++h) {
                uint64_t &s = slot[h & mask];
                if (s == EMPTY) { s = tag | i; break; }
                if ((s & 0xFFFFFFFF00000000ull) != tag) continue;
                const kvr_tuple &y = t[(uint32_t)s];
                if (y.key_len == x.key_len &&
                    memcmp(segs[y.seg_idx].bytes + y.rec_off + 5, segs[x.seg_idx].bytes + x.rec_off + 5,
                           x.key_len) == 0) {
                    s = tag | i;                      // later record wins (engine.rs:137, :141)
                    break;
                }
            }
        }
        for (uint64_t s : slot) {
            if (s == EMPTY) continue;
            const kvr_tuple &y = t[(uint32_t)s];
            if (y.op != 0) continue;
            if (live) live[(uint32_t)s] = 1;
            ++nk[p];
            tb[p] += y.val_len;
        }
    });
    uint64_t k = 0, bytes = 0;
    for (uint32_t p = 0; p < P; ++p) { k += nk[p]; bytes += tb[p]; }
    if (total_bytes) *total_bytes = bytes;
    return k;
}

}  // extern "C"

namespace {

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// the host-fold path (kvs_open with KVS_OPEN_HOST_FOLD, or when the device index cannot hold the
// store): kvr_replay_stream's batches -> tuples in host memory -> kvh_fold_parallel -> live list
// -> the same table on the host
int index_host_fold(kvs_store *s, kvr_ctx *ctx, uint32_t stream_flags, kvr_error *err) {
    const size_t n = s->segs.size();
    uint64_t total = 0;
    for (const kvr_segment &g : s->segs) total += g.len;
    if (!ctx && total) return KVR_EINVAL;   // records to replay, and no device to replay them on
    std::vector<kvr_tuple> t((size_t)(total / 256) + 16);
    size_t nt = 0;
    kvr_error e{};
    int rc = n && total ? kvr_replay_stream(ctx, s->segs.data(), n, stream_flags, 0, nullptr, 0, t.data(), t.size(), &nt, &e)
               : KVR_OK;
    if (rc == KVR_CAPACITY) {
        t.resize(nt);
        rc = kvr_replay_stream(ctx, s->segs.data(), n, stream_flags, 0, nullptr, 0, t.data(), t.size(), &nt, &e);
    }
    if (rc == KVR_CORRUPTED && err) *err = e;
    if (rc != KVR_OK) return rc;
    std::vector<uint8_t> flag(nt);
    uint64_t tb = 0;
    const uint64_t nk = kvh_fold_parallel(s->segs.data(), t.data(), nt, 0, flag.data(), &tb);
    s->live.clear();
    s->live.reserve(nk);
    for (size_t i = 0; i < nt; ++i)
        if (flag[i]) s->live.push_back(t[i]);
    s->slots.assign(kvr_index_slots(s->live.size()), 0u);
    return kvr_index_build_host(s->live.data(), s->live.size(), s->slots.data(), s->slots.size());
}

// the index from a finished device call: live list + table (KVR_CAPACITY: fetch at full size)
template <class F>
int index_device(kvs_store *s, kvr_ctx *ctx, F call) {
    size_t nl = 0;
    uint64_t ns = 0;
    s->live.resize(std::max<size_t>(16, s->live.capacity()));
    s->slots.resize(std::max<size_t>(16, s->slots.capacity()));
    int rc = call(s->live.data(), s->live.size(), s->slots.data(), s->slots.size(), &nl, &ns);
    if (rc == KVR_CAPACITY) {
        s->live.resize(nl);
        s->slots.resize(ns);
        rc = kvr_index_fetch(ctx, 0, s->live.data(), nl, s->slots.data(), ns);
    }
    if (rc != KVR_OK) return rc;
    s->live.resize(nl);
    s->slots.resize(ns);
    return KVR_OK;
}

void finish_index(kvs_store *s) {
    s->total_bytes = 0;   // stats().total_bytes: live value bytes (engine.rs:253-255)
    for (const kvr_tuple &t : s->live) s->total_bytes += t.val_len;
    s->ost.n_live = s->live.size();
}

// (re)build the index over s->segs (host bytes): the device index, the host fold when the device
// cannot hold the store (KVR_ENOMEM, or KVR_EINVAL at the fold's 2^31-tuple limit)
int build_index(kvs_store *s, kvr_ctx *ctx, uint32_t open_flags, kvr_error *err) {
    s->live.clear();
    s->slots.clear();
    int rc = KVR_ENOMEM;
    if (!(open_flags & KVS_OPEN_HOST_FOLD)) {
        rc = index_device(s, ctx, [&](kvr_tuple *l, size_t lc, uint32_t *sl, uint64_t sc, size_t *nl, uint64_t *ns) {
            return kvr_replay_index(ctx, s->segs.data(), s->segs.size(), 0, l, lc, sl, sc, nl, ns, err);
        });
        s->ost.path = KVS_PATH_DEVICE_INDEX;
    }
    if (rc == KVR_ENOMEM || rc == KVR_EINVAL) {
        rc = index_host_fold(s, ctx, s->pinned ? KVR_HOST_PINNED : 0, err);
        s->ost.path = KVS_PATH_HOST_FOLD;
    }
    if (rc == KVR_OK) finish_index(s);
    return rc;
}

constexpr uint64_t PAGE = 4096;
constexpr uint64_t HUGE_PAGE = 2ull << 20;
constexpr uint64_t PIECE = 8ull << 20;   // pread granule
uint64_t page_up(uint64_t n) { return (n + PAGE - 1) & ~(PAGE - 1); }

// segment readiness shared by the loader threads and the push loop: a segment is ready when all
// its pieces are in (pread) or it is mapped (mmap); len[i] = its bytes (a file shorter than at
// discovery ends at its last byte; one that grew is taken as it was)
struct Loader {
    size_t n;
    std::unique_ptr<std::atomic<uint64_t>[]> left, len;
    std::unique_ptr<std::atomic<uint32_t>[]> group_end;   // pread: a registration group's end
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::thread> th;
    explicit Loader(size_t n_) : n(n_), left(new std::atomic<uint64_t>[n_ + 1]), len(new std::atomic<uint64_t>[n_ + 1]),
                                 group_end(new std::atomic<uint32_t>[n_ + 1]) {
        for (size_t i = 0; i <= n; ++i) { left[i] = 1; len[i] = 0; group_end[i] = (uint32_t)(i + 1); }
    }
    void done_one(size_t i) {
        if (--left[i] == 0) {
            std::lock_guard<std::mutex> g(mu);
            cv.notify_all();
        }
    }
    // the group starting at g0 once all its segments are ready: returns its end
    size_t wait_group(size_t g0) {
        const size_t g1 = group_end[g0];
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] {
            for (size_t i = g0; i < g1; ++i) if (left[i].load()) return false;
            return true;
        });
        return g1;
    }
    void join() { for (auto &t : th) t.join(); th.clear(); }
};

// mmap path: every file mapped read-only and populated from the page cache (no copy; about 1 ms
// for 4 GiB when cached), one file per task over the threads in store order.  Each file is opened,
// mapped and closed at once (a mapping outlives its descriptor), so at most one descriptor per
// thread is open whatever the segment count.  Each mapping is its own registration (a transfer
// must lie inside one).  false: a mapping failed (the pread path takes over; nothing is left
// mapped).  The files must not be truncated while the store is open: a mapped page past a new
// end of file faults (SIGBUS) when touched.
bool load_mmap(kvs_store *s, const std::vector<std::string> &paths, const std::vector<uint64_t> &sizes,
               uint32_t n_threads, Loader &L) {
    const size_t n = L.n;
    std::vector<void *> mp(n, nullptr);
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    for (uint32_t w = 0; w < n_threads && n; ++w) {
        L.th.emplace_back([&]() {
            for (;;) {
                const size_t i = next.fetch_add(1);
                if (i >= n) return;
                if (sizes[i] && !failed) {
                    const int fd = open(paths[i].c_str(), O_RDONLY);
                    void *p = fd < 0 ? MAP_FAILED : mmap(nullptr, sizes[i], PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
                    if (fd >= 0) close(fd);
                    if (p == MAP_FAILED) failed = true;
                    else mp[i] = p;
                }
                L.len[i] = sizes[i];
                L.done_one(i);
            }
        });
    }
    L.join();   // mapping is ~1 ms per GiB when cached: no overlap needed with the pushes
    if (failed) {
        for (size_t i = 0; i < n; ++i) if (mp[i]) munmap(mp[i], sizes[i]);
        for (size_t i = 0; i < n; ++i) { L.left[i] = 1; L.len[i] = 0; }
        return false;
    }
    for (size_t i = 0; i < n; ++i) {
        if (mp[i]) s->maps.emplace_back(mp[i], sizes[i]);
        s->segs[i].bytes = static_cast<const uint8_t *>(mp[i]);
    }
    return true;
}

// pread path: one anonymous arena on 2-MiB pages (page-aligned segment starts), 8-MiB pieces in
// store order over the threads (they fault the arena in parallel); consecutive segments form
// registration groups of >= 256 MiB, each ready when all its pieces are in.  Each piece opens its
// file, reads and closes it (one descriptor per thread at most).  Returns KVR_OK, KVR_ENOMEM when
// the arena cannot be mapped (never an empty store in its place: a later compaction would remove
// the files), or KVR_EIO when a file that opened at discovery no longer does (*io_failed).
int load_pread(kvs_store *s, const std::vector<std::string> &paths, const std::vector<uint64_t> &sizes,
               uint32_t n_threads, Loader &L, std::atomic<bool> *io_failed) {
    const size_t n = L.n;
    std::vector<uint64_t> offs(n);
    uint64_t arena = 0;
    for (size_t i = 0; i < n; ++i) { offs[i] = arena; arena += page_up(sizes[i]); }
    const uint64_t map_len = ((arena + HUGE_PAGE - 1) & ~(HUGE_PAGE - 1)) + HUGE_PAGE;
    void *m = mmap(nullptr, map_len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) {
        for (size_t i = 0; i < n; ++i) { L.len[i] = 0; L.left[i] = 0; }
        return KVR_ENOMEM;
    }
    s->maps.emplace_back(m, map_len);
    uint8_t *base = reinterpret_cast<uint8_t *>((reinterpret_cast<uintptr_t>(m) + HUGE_PAGE - 1) & ~(HUGE_PAGE - 1));
    madvise(base, (arena + HUGE_PAGE - 1) & ~(HUGE_PAGE - 1), MADV_HUGEPAGE);   // 2-MiB faults, fast registration
    for (size_t i = 0; i < n; ++i) s->segs[i].bytes = base + offs[i];
    const uint64_t GROUP = std::max<uint64_t>(256ull << 20, arena / 16);
    for (size_t g0 = 0; g0 < n;) {
        size_t g1 = g0;
        uint64_t gb = 0;
        while (g1 < n && (g1 == g0 || gb < GROUP)) gb += page_up(sizes[g1++]);
        L.group_end[g0] = (uint32_t)g1;
        g0 = g1;
    }
    auto pstart = std::make_shared<std::vector<uint64_t>>(n + 1, 0);
    for (size_t i = 0; i < n; ++i) {
        (*pstart)[i + 1] = (*pstart)[i] + std::max<uint64_t>(1, (sizes[i] + PIECE - 1) / PIECE);
        L.left[i] = (*pstart)[i + 1] - (*pstart)[i];
        L.len[i] = sizes[i];
    }
    auto next = std::make_shared<std::atomic<uint64_t>>(0);
    const uint64_t n_pieces = (*pstart)[n];
    for (uint32_t w = 0; w < n_threads && n; ++w) {
        L.th.emplace_back([&L, &paths, &sizes, base, offs, pstart, next, n_pieces, io_failed]() {
            for (;;) {
                const uint64_t p = next->fetch_add(1);
                if (p >= n_pieces) return;
                const size_t i = (size_t)(std::upper_bound(pstart->begin(), pstart->end(), p) - pstart->begin()) - 1;
                const uint64_t o = (p - (*pstart)[i]) * PIECE;
                const uint64_t want = o < sizes[i] ? std::min(PIECE, sizes[i] - o) : 0;
                uint64_t r = 0;
                const int fd = want ? open(paths[i].c_str(), O_RDONLY) : -1;
                if (want && fd < 0) *io_failed = true;
                while (fd >= 0 && r < want) {   // a short read (EOF, error) ends the segment there (engine.rs:88)
                    const ssize_t k = pread(fd, base + offs[i] + o + r, (size_t)(want - r), (off_t)(o + r));
                    if (k < 0 && errno == EINTR) continue;
                    if (k <= 0) break;
                    r += (uint64_t)k;
                }
                if (fd >= 0) close(fd);
                if (r < want) {
                    uint64_t cur = L.len[i].load();
                    while (o + r < cur && !L.len[i].compare_exchange_weak(cur, o + r)) {}
                }
                L.done_one(i);
            }
        });
    }
    return KVR_OK;
}

// create a directory and its missing parents (std::fs::create_dir_all, engine.rs:26-28)
int mkdir_all(const std::string &dir) {
    struct stat st;
    if (stat(dir.c_str(), &st) == 0) return S_ISDIR(st.st_mode) ? 0 : -1;
    const size_t cut = dir.find_last_of('/');
    if (cut != std::string::npos && cut > 0) {
        const std::string parent = dir.substr(0, cut);
        if (mkdir_all(parent) != 0) return -1;
    }
    if (mkdir(dir.c_str(), 0777) != 0 && errno != EEXIST) return -1;
    return 0;
}

}  // namespace

extern "C" {

static bool is_segment_name(const char *name) {   // compaction.rs:41-43
    const size_t n = strlen(name);
    return n >= 12 && memcmp(name, "segment-", 8) == 0 && memcmp(name + n - 4, ".dat", 4) == 0;
}

static int write_file_sync(const std::string &path, const uint8_t *p, size_t n) {
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return -1;
    size_t o = 0;
    while (o < n) {
        const ssize_t w = write(fd, p + o, n - o);
        if (w < 0) { if (errno == EINTR) continue; close(fd); return -1; }
        o += (size_t)w;
    }
    const int rc = fsync(fd);
    close(fd);
    return rc;
}

int kvs_open_ex(const char *dir, kvr_ctx *ctx, uint32_t flags, kvs_store **out, kvr_error *err, char *msg,
                size_t msg_cap) {
    if (!dir || !out) return KVR_EINVAL;   // (ctx NULL: host only, see kvstore_host.h)
    *out = nullptr;
    if (err) memset(err, 0, sizeof(*err));
    if (msg && msg_cap) msg[0] = 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (mkdir_all(dir) != 0) return KVR_EIO;   // engine.rs:26-28 (create_dir_all)
    size_t n = 0;
    int rc = kvh_discover(dir, nullptr, 0, nullptr, 0, &n);
    if (rc != KVR_OK && rc != KVR_CAPACITY) return rc;
    std::vector<uint64_t> ids(n);
    std::vector<char> pbuf(n * 4200 + 16);
    rc = kvh_discover(dir, ids.data(), n, pbuf.data(), pbuf.size(), &n);
    if (rc != KVR_OK) return rc;
    std::vector<std::string> paths(n);
    size_t po = 0;
    for (size_t i = 0; i < n; ++i) { paths[i] = std::string(pbuf.data() + po); po += paths[i].size() + 1; }

    // engine.rs:55-57 opens segment k only after segments 0 .. k-1 replayed: an unopenable file
    // ends the list, and its error stands only if the segments before it replay cleanly.  Each
    // file is opened, measured and closed here (the loaders open it again), so the descriptors
    // in use never grow with the segment count; running out of descriptors (EMFILE / ENFILE) is a
    // resource failure of this process, not an unopenable segment.
    std::vector<uint64_t> sizes;
    size_t n_ok = n;
    int open_errno = 0;
    for (size_t i = 0; i < n; ++i) {
        const int fd = open(paths[i].c_str(), O_RDONLY);
        if (fd < 0) {
            if (errno == EMFILE || errno == ENFILE) return KVR_EIO;
            n_ok = i; open_errno = errno; break;   // engine.rs:80-82
        }
        struct stat fs;
        const bool dir_like = fstat(fd, &fs) != 0 || S_ISDIR(fs.st_mode);   // read() fails -> EOF (engine.rs:88)
        close(fd);
        sizes.push_back(dir_like ? 0 : (uint64_t)fs.st_size);
    }
    // test knob: segment i's file disappears between discovery and the read (the race that
    // test_open_vanished_segment drives deterministically).  Nothing is deleted: the loader is given a
    // path that does not exist in place of the file's, so its open fails as for a vanished file.
    if (const char *vn = getenv("KVS_TEST_VANISH")) {
        const size_t vi = (size_t)strtoull(vn, nullptr, 10);
        if (vi < n_ok) paths[vi] = std::string("/nonexistent/kvs-test-vanished/") + std::to_string(vi);
    }

    std::unique_ptr<kvs_store> s(new kvs_store());
    s->dir = dir;
    s->open_flags = flags;
    s->ids.assign(ids.begin(), ids.begin() + (ptrdiff_t)n_ok);
    s->ost.n_segments = n_ok;
    s->segs.resize(n_ok);
    for (size_t i = 0; i < n_ok; ++i) s->segs[i] = kvr_segment{ids[i], nullptr, sizes[i]};
    const bool device = ctx && !(flags & KVS_OPEN_HOST_FOLD) && kvr_ingest_begin(ctx, page_up(std::accumulate(
                            sizes.begin(), sizes.end(), (uint64_t)0, [](uint64_t a, uint64_t b) { return a + page_up(b); })), n_ok) == KVR_OK;
    // declared after the store, so destroyed before it: on every return from here on, the copies
    // queued by kvr_ingest_push have finished reading the store's host bytes before those are
    // unregistered and unmapped (an early return, e.g. a file that vanished, leaves them in flight)
    struct IngestGuard {
        kvr_ctx *c;
        bool on;
        ~IngestGuard() { if (on) kvr_ingest_abort(c); }
    } ingest_guard{ctx, device};
    const bool reg = !(flags & KVS_OPEN_NO_PIN);
    const uint32_t n_threads = (uint32_t)std::min<uint64_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    s->ost.read_threads = n_threads;
    Loader L(n_ok);
    const auto tr = std::chrono::steady_clock::now();
    // the segments' host bytes: the files mapped (page cache, no copy) or read into an arena;
    // the loader threads make segment i ready in store order as far as they can, and the push
    // loop below registers and transfers each one as soon as it is
    bool mapped = !(flags & KVS_OPEN_PREAD) && load_mmap(s.get(), paths, sizes, n_threads, L);
    std::atomic<bool> io_failed{false};
    if (!mapped) {
        const int lr = load_pread(s.get(), paths, sizes, n_threads, L, &io_failed);
        if (lr != KVR_OK) return lr;
    }
    s->ost.mode = mapped ? KVS_LOAD_MMAP : KVS_LOAD_PREAD;
    bool all_reg = reg;
    double ms_reg = 0, ms_push = 0;
    int push_rc = KVR_OK;
    for (size_t g0 = 0; g0 < n_ok;) {
        const size_t g1 = L.wait_group(g0);   // [g0, g1): ready, one registration
        for (size_t i = g0; i < g1; ++i) s->segs[i].len = L.len[i];
        const uint8_t *p0 = s->segs[g0].bytes;
        const uint64_t gb = page_up((uint64_t)(s->segs[g1 - 1].bytes + s->segs[g1 - 1].len - p0));
        if (reg && gb && p0) {
            const auto tg = std::chrono::steady_clock::now();
            void *p = const_cast<uint8_t *>(p0);
            if (kvr_host_register(p, gb) == KVR_OK) s->regs.push_back(p);
            else all_reg = false;   // stays pageable: HIP stages the transfers
            ms_reg += ms_since(tg);
        }
        const auto tp = std::chrono::steady_clock::now();
        for (size_t i = g0; i < g1; ++i)
            if (device && push_rc == KVR_OK) push_rc = kvr_ingest_push(ctx, s->segs[i].seg_id, s->segs[i].bytes, s->segs[i].len);
        ms_push += ms_since(tp);
        g0 = g1;
    }
    L.join();
    s->ost.ms_read = ms_since(tr);
    s->ost.ms_register = ms_reg;
    s->ost.ms_push = ms_push;
    s->pinned = all_reg;
    if (io_failed) return KVR_EIO;   // a segment file vanished between discovery and the read
    uint64_t bytes = 0;
    for (const kvr_segment &g : s->segs) bytes += g.len;
    s->ost.bytes = bytes;

    const auto ti = std::chrono::steady_clock::now();
    rc = KVR_ENOMEM;
    if (device && push_rc == KVR_OK) {
        rc = index_device(s.get(), ctx, [&](kvr_tuple *l, size_t lc, uint32_t *sl, uint64_t sc, size_t *nl, uint64_t *ns) {
            return kvr_ingest_index(ctx, 0, l, lc, sl, sc, nl, ns, err);
        });
        s->ost.path = KVS_PATH_DEVICE_INDEX;
    }
    if (rc == KVR_ENOMEM || rc == KVR_EINVAL) {   // HBM too small for the store, or the fold's limits
        rc = index_host_fold(s.get(), ctx, s->pinned ? KVR_HOST_PINNED : 0, err);
        s->ost.path = KVS_PATH_HOST_FOLD;
    }
    s->ost.ms_index = ms_since(ti);
    if (rc == KVR_CORRUPTED) {
        if (msg && err) kvr_format_error(err, paths[err->seg_idx].c_str(), msg, msg_cap);
        return rc;
    }
    if (rc != KVR_OK) return rc;
    if (n_ok < n) {   // every segment before the unopenable one replayed: the open error stands
        if (err) { err->kind = KVR_E_OPEN; err->seg_idx = (uint32_t)n_ok; err->rec_off = 0; err->aux = (uint64_t)open_errno; }
        if (msg && err) kvr_format_error(err, paths[n_ok].c_str(), msg, msg_cap);
        return KVR_CORRUPTED;
    }
    finish_index(s.get());
    // engine.rs:59-68: next id = max + 1, create the (empty) active segment for appends
    s->active_id = (n ? ids[n - 1] : 0) + 1;
    const std::string ap = std::string(dir) + "/segment-" + std::to_string(s->active_id) + ".dat";
    const int fd = open(ap.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd < 0) return KVR_EIO;   // engine.rs:63-67: the create error is StoreError::Io
    close(fd);
    s->ost.ms_total = ms_since(t0);
    *out = s.release();
    return KVR_OK;
}

int kvs_open(const char *dir, kvr_ctx *ctx, kvs_store **out, kvr_error *err, char *msg, size_t msg_cap) {
    return kvs_open_ex(dir, ctx, 0, out, err, msg, msg_cap);
}

int kvs_last_open_stats(const kvs_store *s, kvs_open_stats *out) {
    if (!s || !out) return KVR_EINVAL;
    *out = s->ost;
    return KVR_OK;
}

int kvs_get(const kvs_store *s, const uint8_t *key, size_t klen, const uint8_t **val, size_t *vlen) {
    if (!s) return KVR_EINVAL;
    if (s->live.empty()) return 0;
    const int64_t j = kvr_index_find(s->live.data(), s->slots.data(), s->slots.size(), s->segs.data(), key, klen);
    if (j < 0) return 0;
    const kvr_tuple &t = s->live[(size_t)j];
    if (val) *val = s->segs[t.seg_idx].bytes + t.rec_off + 9 + t.key_len;
    if (vlen) *vlen = t.val_len;
    return 1;
}

int kvs_locate(const kvs_store *s, const uint8_t *key, size_t klen, uint64_t *seg_id, uint64_t *val_off, uint64_t *len) {
    if (!s) return KVR_EINVAL;
    if (s->live.empty()) return 0;
    const int64_t j = kvr_index_find(s->live.data(), s->slots.data(), s->slots.size(), s->segs.data(), key, klen);
    if (j < 0) return 0;
    const kvr_tuple &t = s->live[(size_t)j];
    if (seg_id) *seg_id = s->ids[t.seg_idx];
    if (val_off) *val_off = t.rec_off + 9 + t.key_len;
    if (len) *len = t.val_len;
    return 1;
}

int kvs_stats_get(const kvs_store *s, kvs_stats *out) {
    if (!s || !out) return KVR_EINVAL;
    out->num_keys = s->live.size();
    uint64_t nseg = 0;   // engine.rs:239-250: entries named segment-*.dat, parse or not
    if (DIR *d = opendir(s->dir.c_str())) {
        while (struct dirent *e = readdir(d)) {
            const size_t n = strlen(e->d_name);
            if (n >= 8 && memcmp(e->d_name, "segment-", 8) == 0 && n >= 4 && memcmp(e->d_name + n - 4, ".dat", 4) == 0 &&
                utf8_valid(reinterpret_cast<const uint8_t *>(e->d_name), n))
                ++nseg;
        }
        closedir(d);
    }
    out->num_segments = nseg;
    out->total_bytes = s->total_bytes;
    out->active_segment_id = s->active_id;
    out->oldest_segment_id = 0;   // engine.rs:257
    return KVR_OK;
}

size_t kvs_num_keys(const kvs_store *s) { return s ? s->live.size() : 0; }

int kvs_compact(kvs_store *s, kvr_ctx *ctx, uint64_t seg_target, kvr_error *err) {
    if (!s || !ctx) return KVR_EINVAL;
    if (err) memset(err, 0, sizeof(*err));
    const size_t n = s->segs.size();
    const std::vector<kvr_segment> &segs = s->segs;
    uint64_t bytes_in = 0;
    for (const kvr_segment &g : segs) bytes_in += g.len;
    // 1. the live records, re-framed into new segments, on the GPU
    std::vector<uint8_t> out(std::max<uint64_t>(bytes_in, 1));
    std::vector<uint64_t> ends(seg_target ? bytes_in / seg_target + 2 : 1);
    uint64_t out_len = 0;
    size_t n_new = 0;
    int rc = KVR_OK;
    if (n) {
        rc = kvr_compact(ctx, segs.data(), n, 0, seg_target, out.data(), out.size(), &out_len, ends.data(),
                         ends.size(), &n_new, err);
        if (rc == KVR_CAPACITY) {
            out.resize(out_len);
            ends.resize(n_new);
            rc = kvr_compact(ctx, segs.data(), n, 0, seg_target, out.data(), out.size(), &out_len, ends.data(),
                             ends.size(), &n_new, err);
        }
        if (rc != KVR_OK) return rc;
    }
    // 2. new files first (ids after the active segment), durable before anything is removed
    std::vector<uint64_t> new_ids(n_new);
    std::vector<std::vector<uint8_t>> new_bytes(n_new);
    std::vector<std::string> new_names(n_new);
    uint64_t prev = 0;
    for (size_t j = 0; j < n_new; ++j) {
        new_ids[j] = s->active_id + 1 + j;
        new_names[j] = "segment-" + std::to_string(new_ids[j]) + ".dat";
        new_bytes[j].assign(out.begin() + (ptrdiff_t)prev, out.begin() + (ptrdiff_t)ends[j]);
        if (write_file_sync(s->dir + "/" + new_names[j], new_bytes[j].data(), new_bytes[j].size()) != 0) return KVR_EIO;
        prev = ends[j];
    }
    // 3. every other segment-*.dat goes (compaction.rs:11-23; NotFound is not an error)
    if (DIR *d = opendir(s->dir.c_str())) {
        std::vector<std::string> victims;
        while (struct dirent *e = readdir(d)) {
            if (!is_segment_name(e->d_name)) continue;
            if (std::find(new_names.begin(), new_names.end(), std::string(e->d_name)) != new_names.end()) continue;
            victims.push_back(s->dir + "/" + e->d_name);
        }
        closedir(d);
        for (const auto &v : victims)
            if (unlink(v.c_str()) != 0 && errno != ENOENT) return KVR_EIO;
    } else {
        return KVR_EIO;
    }
    // 4. reset_active_segment (engine.rs:209-229): the next id, an empty file
    s->active_id = s->active_id + n_new + 1;
    const std::string ap = s->dir + "/segment-" + std::to_string(s->active_id) + ".dat";
    const int fd = open(ap.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd < 0) return KVR_EIO;
    close(fd);
    // 5. the store now reads the new files; the index is rebuilt over them (same map).
    // kvr_replay_index leaves kvr_last_compact_stats to this compaction.
    s->ids = new_ids;
    s->owned = std::move(new_bytes);
    s->segs.resize(n_new);
    for (size_t j = 0; j < n_new; ++j) s->segs[j] = kvr_segment{new_ids[j], s->owned[j].data(), s->owned[j].size()};
    s->drop_arena();
    return build_index(s, ctx, s->open_flags, err);
}

void kvs_close(kvs_store *s) { delete s; }

}  // extern "C"
