/*
 * kvr_index.hip — the open-time index on the device, included by kvr_api.hip.
 *
 * KVStore::open (engine.rs:24-76) ends with a HashMap<String, Vec<u8>> (index.rs:5-7 has the
 * shape) holding every live key's final value: replay (engine.rs:55-57), then the fold of
 * engine.rs:137 (insert) / :141 (remove).  Here both run in HBM and only the result crosses
 * PCIe, as two flat arrays:
 *   live[]    each live key's final SET tuple, in (segment, offset) order (kvr_replay_live);
 *   slots[]   an open-addressing table over live[]: slots[h] = 1 + index into live[] (0: free),
 *             home slot kvr_index_hash(key_tag) & (n_slots - 1), linear probing; n_slots =
 *             kvr_index_slots(n_live) (a power of two, >= 2 n_live).
 * A lookup (kvr_index_find) is one CRC-32 of the key and a probe that compares tags first, so the
 * host folds nothing.  The ingest calls stage the store's bytes in HBM as the caller reads the
 * files, so reading, PCIe transfer and (at the end) the replay and fold overlap.
 */

namespace {
// the home slot of a key tag (kvr_index_hash, host and device): the fold table's hash, since
// the index IS the fold table, entry for entry
__host__ __device__ __forceinline__ uint32_t ix_hash(uint32_t h) { return ht_mix(h); }

constexpr uint32_t IX_DEAD = 0xFFFFFFFFu;   // a key whose last record is a DEL: probe on

// slots[h] from fold entry h: free -> 0, a live key -> 1 + its position in the live list, a
// deleted key -> IX_DEAD (keeps the probe sequences of the keys behind it intact).  No atomics:
// the fold already placed every key.
__global__ void k_index_from_fold(const FoldEnt *__restrict__ ent, const uint32_t *__restrict__ fsz,
                                  const uint8_t *__restrict__ flag8, const uint32_t *__restrict__ pos,
                                  uint32_t *__restrict__ slots) {
    const uint64_t n_slots = (uint64_t)fsz[0] + 1;   // the fold table's size on the device; grid-stride
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n_slots; h += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 a = reinterpret_cast<const uint4 *>(&ent[h])[0];
        uint32_t v = 0;
        if (!(a.x == 0xFFFFFFFFu && a.y == 0xFFFFFFFFu)) {
            const uint32_t j = ~a.z;
            v = flag8[j] ? pos[j] + 1u : IX_DEAD;
        }
        slots[h] = v;
    }
}

// key arena: live key i's bytes to keys[off[i] ..) — one thread per key (keys are short; a
// long one loops), 4-B stores where the destination allows
__global__ void k_key_lens(const kvr_tuple *__restrict__ live, uint64_t n, uint64_t *__restrict__ len) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) len[i] = live[i].key_len;
}
__global__ void k_key_copy(const kvr_tuple *__restrict__ live, uint64_t n, const SegDesc *__restrict__ segs,
                           const uint64_t *__restrict__ off, uint8_t *__restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const kvr_tuple t = live[i];
    const uint8_t *src = segs[t.seg_idx].base + t.rec_off + 5;   // [op][klen u32][key] (engine.rs:169-171)
    uint8_t *dst = keys + off[i];
    for (uint32_t b = 0; b < t.key_len; ++b) dst[b] = src[b];
}

uint64_t index_slots(uint64_t n_live) {
    uint64_t s = 16;
    while (s < 2 * n_live) s <<= 1;
    return s;
}

// after compact_front: live flags (a byte per tuple), the dense live list in c->lout (room for every
// tuple) from per-block counts and one workgroup's scan of them (k_dl_*, as kvr_compact's), and
// with index the key table in c->islots (room for the largest table); no host sync — n_live =
// dl_tot[1], read by fold_settle (keep_del: every key's last record instead, tombstones included)
int fold_derive(kvr_ctx *c, size_t nt, bool keep_del, bool index) {
    hipStream_t st = c->stream;
    const uint32_t nb = (uint32_t)((nt + DL_CH - 1) / DL_CH);
    if (c->lout.ensure(nt) || (index && c->islots.ensure(c->fent.n)) || c->dl_cnt.ensure(nb) || c->dl_bytes.ensure(nb) ||
        c->dl_tot.ensure(2))
        return KVR_ENOMEM;
    HIPCHK(live_flags(c, nt, false, keep_del, true));
    hipLaunchKernelGGL(k_dl_count, dim3(nb), dim3(DL_T), 0, st, c->cfl8.p, (const kvr_tuple *)nullptr, c->dl_cnt.p,
                       c->dl_bytes.p);
    hipLaunchKernelGGL(k_dl_scan, dim3(1), dim3(DL_ST), 0, st, c->dl_cnt.p, c->dl_bytes.p, nb, (uint64_t *)nullptr,
                       c->dl_tot.p);
    hipLaunchKernelGGL(k_dl_fill_tup, dim3(nb), dim3(DL_T), 0, st, c->cfl8.p, c->ctup.p, c->dl_cnt.p, c->lout.p, c->cpos.p);
    if (index)
        hipLaunchKernelGGL(k_index_from_fold, dim3(fold_grid(c)), dim3(256), 0, st, c->fent.p, c->fsz.p, c->cfl8.p,
                           c->cpos.p, c->islots.p);
    HIPCHK(hipGetLastError());
    return KVR_OK;
}

// fold_settle + fold_derive again if the deferred fold had to be redone; *total = n_live
int derive_settle(kvr_ctx *c, size_t nt, bool keep_del, bool index, uint64_t *total) {
    uint64_t n_live = 0;
    bool redone = false;
    int rc = fold_settle(c, nt, &redone, &n_live);
    if (rc == KVR_OK && redone) {
        rc = fold_derive(c, nt, keep_del, index);
        if (rc == KVR_OK) rc = fold_settle(c, nt, &redone, &n_live);   // (not pending: reads the totals)
    }
    *total = n_live;
    return rc;
}

int index_copy_out(kvr_ctx *c, uint32_t flags, kvr_tuple *live, size_t live_cap, uint32_t *slots, uint64_t slot_cap) {
    if (c->ix_live > live_cap || c->ix_slots > slot_cap) return KVR_CAPACITY;
    const hipMemcpyKind k = (flags & KVR_OUT_ON_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    hipStream_t st = c->stream;
    if (c->ix_live) HIPCHK(hipMemcpyAsync(live, c->lout.p, c->ix_live * sizeof(kvr_tuple), k, st));
    if (c->ix_slots) HIPCHK(hipMemcpyAsync(slots, c->islots.p, c->ix_slots * 4, k, st));
    HIPCHK(hipStreamSynchronize(st));
    return KVR_OK;
}
}  // namespace

namespace {
int replay_last(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, kvr_tuple *out, size_t cap,
                       size_t *n_out, kvr_error *err, bool keep_del) {
    if (!c || (!segs && n) || !n_out || (cap && !out)) return KVR_EINVAL;
    if (flags & ~(KVR_SEGS_ON_DEVICE | KVR_OUT_ON_DEVICE)) return KVR_EINVAL;
    *n_out = 0;
    c->ix_valid = false;
    HIPCHK(hipSetDevice(c->device));
    size_t nt = 0;
    kvr_compact_stats cs{};
    int rc = compact_front(c, segs, n, flags, err, &nt, false, &cs, true);   // replay + fold (kvr_compact.hip)
    if (rc != KVR_OK) return rc;
    uint64_t total = 0;
    if (nt) {
        rc = fold_derive(c, nt, keep_del, false);
        if (rc == KVR_OK) rc = derive_settle(c, nt, keep_del, false, &total);
        if (rc != KVR_OK) return rc;
    }
    *n_out = total;
    c->ix_live = total;   // kvr_live_keys reads this live list
    c->ix_slots = 0;
    c->ix_valid = true;
    if (total > cap) return KVR_CAPACITY;
    if (total == 0) return KVR_OK;
    const hipMemcpyKind k = (flags & KVR_OUT_ON_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    HIPCHK(hipMemcpyAsync(out, c->lout.p, total * sizeof(kvr_tuple), k, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return KVR_OK;
}
}  // namespace

extern "C" {

int kvr_replay_live(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, kvr_tuple *out, size_t cap,
                    size_t *n_out, kvr_error *err) {
    return replay_last(c, segs, n, flags, out, cap, n_out, err, false);
}

int kvr_replay_last(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, kvr_tuple *out, size_t cap,
                    size_t *n_out, kvr_error *err) {
    return replay_last(c, segs, n, flags, out, cap, n_out, err, true);
}

uint64_t kvr_index_slots(uint64_t n_live) { return index_slots(n_live); }

uint32_t kvr_index_hash(uint32_t key_tag) { return ix_hash(key_tag); }

int kvr_replay_index(kvr_ctx *c, const kvr_segment *segs, size_t n, uint32_t flags, kvr_tuple *live, size_t live_cap,
                     uint32_t *slots, uint64_t slot_cap, size_t *n_live, uint64_t *n_slots, kvr_error *err) {
    if (!c || (!segs && n) || !n_live || !n_slots || (live_cap && !live) || (slot_cap && !slots)) return KVR_EINVAL;
    if (flags & ~(KVR_SEGS_ON_DEVICE | KVR_OUT_ON_DEVICE)) return KVR_EINVAL;
    *n_live = 0;
    *n_slots = 0;
    c->ix_valid = false;
    c->ix_live = c->ix_slots = 0;
    HIPCHK(hipSetDevice(c->device));
    memset(&c->istats, 0, sizeof(c->istats));
    const auto t0 = std::chrono::steady_clock::now();
    size_t nt = 0;
    kvr_compact_stats cs{};
    int rc = compact_front(c, segs, n, flags, err, &nt, false, &cs, true);   // deferred fold rounds
    c->istats.bytes_in = cs.bytes_in;
    c->istats.n_tuples = nt;
    c->istats.ms_replay = cs.ms_replay;
    if (rc != KVR_OK) return rc;
    uint64_t total = 0;
    hipStream_t st = c->stream;
    if (nt) {
        // the live list and the key table are launched behind the fold; one sync for all of it
        rc = fold_derive(c, nt, false, true);
        if (rc != KVR_OK) return rc;
        HIPCHK(hipEventRecord(c->ev[4], st));
        rc = derive_settle(c, nt, false, true, &total);
        if (rc != KVR_OK) return rc;
        c->istats.ms_fold = ev_ms(c->ev[0], c->ev[4]);   // fold rounds .. index table
    } else {
        if (c->islots.ensure(16)) return KVR_ENOMEM;
        HIPCHK(hipMemsetAsync(c->islots.p, 0, 16 * 4, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    const uint64_t ns = nt ? c->fold_slots : 16;
    c->ix_live = total;
    c->ix_slots = ns;
    c->ix_valid = true;
    c->istats.n_live = total;
    c->istats.n_slots = ns;
    c->istats.fold_rounds = c->fold_rounds;
    c->istats.fold_slots = c->fold_slots;
    c->istats.fold_est = c->fold_est;
    c->istats.fold_redo = c->fold_redo;
    *n_live = total;
    *n_slots = ns;
    rc = index_copy_out(c, flags, live, live_cap, slots, slot_cap);
    c->istats.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int kvr_index_fetch(kvr_ctx *c, uint32_t flags, kvr_tuple *live, size_t live_cap, uint32_t *slots, uint64_t slot_cap) {
    if (!c || !c->ix_valid || (live_cap && !live) || (slot_cap && !slots)) return KVR_EINVAL;
    if (flags & ~KVR_OUT_ON_DEVICE) return KVR_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    return index_copy_out(c, flags, live, live_cap, slots, slot_cap);
}

int kvr_live_keys(kvr_ctx *c, uint32_t flags, uint8_t *keys, uint64_t keys_cap, uint64_t *key_off, size_t off_cap,
                  uint64_t *key_bytes) {
    if (!c || !key_bytes || (keys_cap && !keys) || (off_cap && !key_off)) return KVR_EINVAL;
    if (flags & ~KVR_OUT_ON_DEVICE) return KVR_EINVAL;
    if (!c->ix_valid) return KVR_EINVAL;   // no live list (or a later call replaced it: every replay clears it)
    HIPCHK(hipSetDevice(c->device));
    const uint64_t n = c->ix_live;
    hipStream_t st = c->stream;
    *key_bytes = 0;
    if (c->koff.ensure(n + 1)) return KVR_ENOMEM;
    if (n) {
        const uint32_t g = (uint32_t)((n + 255) / 256);
        if (c->klen.ensure(n + 1)) return KVR_ENOMEM;
        hipLaunchKernelGGL(k_key_lens, dim3(g), dim3(256), 0, st, c->lout.p, n, c->klen.p);
        HIPCHK(hipMemsetAsync(c->klen.p + n, 0, 8, st));
        size_t tb = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, c->klen.p, c->koff.p, (int)(n + 1), st));
        if (c->ctmp.n < tb && c->ctmp.ensure(tb)) return KVR_ENOMEM;
        tb = c->ctmp.n;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->ctmp.p, tb, c->klen.p, c->koff.p, (int)(n + 1), st));
        HIPCHK(hipMemcpyAsync(key_bytes, c->koff.p + n, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (c->kbuf.ensure(*key_bytes + 1)) return KVR_ENOMEM;
        hipLaunchKernelGGL(k_key_copy, dim3(g), dim3(256), 0, st, c->lout.p, n, c->segs.p, c->koff.p, c->kbuf.p);
        HIPCHK(hipGetLastError());
    } else {
        HIPCHK(hipMemsetAsync(c->koff.p, 0, 8, st));
    }
    if (*key_bytes > keys_cap || n + 1 > off_cap) {
        HIPCHK(hipStreamSynchronize(st));
        return KVR_CAPACITY;
    }
    const hipMemcpyKind k = (flags & KVR_OUT_ON_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (*key_bytes) HIPCHK(hipMemcpyAsync(keys, c->kbuf.p, *key_bytes, k, st));
    HIPCHK(hipMemcpyAsync(key_off, c->koff.p, (n + 1) * 8, k, st));
    HIPCHK(hipStreamSynchronize(st));
    return KVR_OK;
}

int kvr_last_index_stats(const kvr_ctx *c, kvr_index_stats *out) {
    if (!c || !out) return KVR_EINVAL;
    *out = c->istats;
    return KVR_OK;
}

int kvr_ingest_begin(kvr_ctx *c, uint64_t total_bytes, size_t n_segs) {
    if (!c) return KVR_EINVAL;
    c->ix_valid = false;
    c->ing_off = 0;
    c->ing_segs.clear();
    HIPCHK(hipSetDevice(c->device));
    if (c->copy) HIPCHK(hipStreamSynchronize(c->copy));   // no copy of an earlier ingest in flight
    const char *lim = getenv("KVR_INGEST_LIMIT");         // test knob: a smaller HBM budget
    if (lim && total_bytes > strtoull(lim, nullptr, 10)) return KVR_ENOMEM;
    if (c->ing.ensure(total_bytes + 256 * ((uint64_t)n_segs + 1))) return KVR_ENOMEM;
    c->ing_segs.reserve(n_segs);
    if (!c->copy) {
        HIPCHK(hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
        for (auto &e : c->ev_copy) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    return KVR_OK;
}

int kvr_ingest_push(kvr_ctx *c, uint64_t seg_id, const uint8_t *bytes, uint64_t len) {
    if (!c || (len && !bytes) || !c->copy) return KVR_EINVAL;
    if (!c->ing_segs.empty() && seg_id < c->ing_segs.back().seg_id) return KVR_EINVAL;   // engine.rs:51 order
    const uint64_t padded = (len + 255) & ~255ull;
    if (c->ing_off + padded > c->ing.n) return KVR_CAPACITY;
    uint8_t *d = c->ing.p + c->ing_off;
    if (len) HIPCHK(hipMemcpyAsync(d, bytes, len, hipMemcpyHostToDevice, c->copy));
    c->ing_segs.push_back(kvr_segment{seg_id, d, len});
    c->ing_off += padded;
    return KVR_OK;
}

int kvr_ingest_abort(kvr_ctx *c) {
    if (!c) return KVR_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    if (c->copy) HIPCHK(hipStreamSynchronize(c->copy));   // every queued DMA has read its host bytes
    c->ing_segs.clear();
    c->ing_off = 0;
    return KVR_OK;
}

int kvr_ingest_index(kvr_ctx *c, uint32_t flags, kvr_tuple *live, size_t live_cap, uint32_t *slots, uint64_t slot_cap,
                     size_t *n_live, uint64_t *n_slots, kvr_error *err) {
    if (!c || !c->copy) return KVR_EINVAL;
    if (flags & ~KVR_OUT_ON_DEVICE) return KVR_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    // the replay waits for the last transfer on the device, not on the host
    HIPCHK(hipEventRecord(c->ev_copy[0], c->copy));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_copy[0], 0));
    return kvr_replay_index(c, c->ing_segs.data(), c->ing_segs.size(), KVR_SEGS_ON_DEVICE | flags, live, live_cap,
                            slots, slot_cap, n_live, n_slots, err);
}

int64_t kvr_index_find(const kvr_tuple *live, const uint32_t *slots, uint64_t n_slots, const kvr_segment *segs,
                       const uint8_t *key, size_t klen) {
    if (!live || !slots || !segs || n_slots == 0 || (n_slots & (n_slots - 1)) || (klen && !key)) return -1;
    const uint32_t tag = kvr_crc32(0, key, klen);
    const uint64_t mask = n_slots - 1;
    for (uint64_t h = ix_hash(tag) & mask, probe = 0; probe < n_slots; ++probe, h = (h + 1) & mask) {
        const uint32_t v = slots[h];
        if (v == 0) return -1;
        if (v == IX_DEAD) continue;
        const kvr_tuple &t = live[v - 1];
        if (t.key_tag == tag && t.key_len == klen &&
            (klen == 0 || memcmp(segs[t.seg_idx].bytes + t.rec_off + 5, key, klen) == 0))
            return (int64_t)(v - 1);
    }
    return -1;
}

int kvr_index_build_host(const kvr_tuple *live, size_t n_live, uint32_t *slots, uint64_t n_slots) {
    if ((n_live && !live) || !slots || n_slots <= n_live || (n_slots & (n_slots - 1)) || n_live >= 0xFFFFFFFFull)
        return KVR_EINVAL;
    memset(slots, 0, n_slots * 4);
    const uint64_t mask = n_slots - 1;
    for (size_t j = 0; j < n_live; ++j) {
        uint64_t h = ix_hash(live[j].key_tag) & mask;
        while (slots[h]) h = (h + 1) & mask;
        slots[h] = (uint32_t)j + 1u;
    }
    return KVR_OK;
}

int kvr_host_alloc(uint64_t bytes, void **out) {
    if (!out) return KVR_EINVAL;
    *out = nullptr;
    if (hipHostMalloc(out, bytes ? bytes : 1) != hipSuccess) {
        *out = nullptr;
        return KVR_ENOMEM;
    }
    return KVR_OK;
}

void kvr_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int kvr_host_register(void *p, uint64_t bytes) {
    if (!p || !bytes) return KVR_EINVAL;
    return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? KVR_OK : KVR_EHIP;
}

void kvr_host_unregister(void *p) {
    if (p) (void)hipHostUnregister(p);
}

}  // extern "C"
