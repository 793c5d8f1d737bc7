/*
 * kvr_kernels.hip — the support kernels around k_replay (kvr_replay_kernel.hip), gfx950.
 *
 *   k_link     one workgroup: verify every stripe's speculated entry against its predecessor's
 *              exit, pick the first error in (segment, offset) order (engine.rs:55-56) and
 *              list the stripes that must be re-walked from their true entry.
 *   k_compact_s
 *              one workgroup per stripe: the gather of the pool into the dense output in
 *              (segment, offset) order, with per-record CRC verification.
 *   k_gen_fill / k_gen_manifest
 *              device side of the synthetic generator (kvr_gen_common.h).
 */
#include "kvr_device.h"
#include "kvr_gen_common.h"

namespace kvr {

// ---------------------------------------------------------------------------------------
// k_link — one workgroup of 1024 threads.
// ---------------------------------------------------------------------------------------
constexpr int LT = 1024;

__device__ __forceinline__ uint64_t stripe_hi(const StripeDesc &d, const SegDesc &g, uint32_t tile) {
    const int64_t h = (int64_t)d.t_end * tile - (int64_t)g.d0;
    return (uint64_t)h > g.len ? g.len : (uint64_t)h;
}

__device__ __forceinline__ uint64_t stripe_lo(const StripeDesc &d, const SegDesc &g, uint32_t tile) {
    const int64_t l = (int64_t)d.t_begin * tile - (int64_t)g.d0;
    return l < 0 ? 0ull : (uint64_t)l;
}

// segments whose first-problem stripes k_link keeps in LDS (more: in the global arrays)
constexpr uint32_t LINK_LSEG = 4096;

__global__ __launch_bounds__(LT) void k_link(const SegDesc *__restrict__ segs, uint32_t n_segs,
                                             const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                             StripeRes *__restrict__ sres, RedoEnt *__restrict__ redo,
                                             uint32_t redo_cap, LinkResult *res, uint32_t *seg_bad_g,
                                             uint32_t *seg_err_g, uint32_t tile, uint64_t *__restrict__ soff,
                                             Counters *ctr, LinkResult *hres, Counters *hctr) {
    __shared__ int32_t wm[LT / 64];
    __shared__ uint64_t wx[LT / 64];
    __shared__ unsigned long long wsum[LT / 64];
    __shared__ uint32_t first_problem, nredo;
    __shared__ uint32_t l_bad[LINK_LSEG], l_err[LINK_LSEG];
    // per segment: its first inconsistent stripe and its first error stripe (LDS for the usual
    // segment counts; flat pointers, so the atomics below serve both)
    uint32_t *const seg_bad = n_segs <= LINK_LSEG ? l_bad : seg_bad_g;
    uint32_t *const seg_err = n_segs <= LINK_LSEG ? l_err : seg_err_g;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (uint32_t g = tid; g < n_segs; g += LT) { seg_bad[g] = ~0u; seg_err[g] = ~0u; }
    if (tid == 0) { first_problem = ~0u; nredo = 0; }
    const uint32_t per = (n_stripes + LT - 1) / LT;
    const uint32_t b = tid * per, e = min(b + per, n_stripes);
    // this thread's chunk: its last stripe with a record start (and that stripe's exit), and its
    // stripes' records (the output offsets k_compact_s writes from); exclusive scans over the
    // chunks, a "latest" and a sum, by wave shuffles and then the 16 wave totals, so no stripe
    // result is read twice and none after the scan
    // (up to KL stripes per thread, the common case: their results and descriptors are loaded
    // once, all together, and kept in registers for the passes below)
    constexpr int KL = 4;
    const bool cached = per <= (uint32_t)KL;
    uint64_t c_entry[KL], c_exit[KL];
    uint32_t c_kind[KL], c_count[KL], c_seg[KL], c_tb[KL], c_te[KL], c_first[KL];
    if (cached) {
#pragma unroll
        for (int i = 0; i < KL; ++i) {
            const uint32_t s = b + i;
            c_entry[i] = NONE; c_exit[i] = NONE; c_kind[i] = 0; c_count[i] = 0; c_seg[i] = 0; c_tb[i] = 0; c_te[i] = 0;
            c_first[i] = 0;
            if (s < e) {
                c_entry[i] = sres[s].entry; c_exit[i] = sres[s].exit; c_kind[i] = sres[s].err_kind;
                c_count[i] = sres[s].count;
                const StripeDesc d = stripes[s];
                c_seg[i] = d.seg; c_tb[i] = d.t_begin; c_te[i] = d.t_end; c_first[i] = d.pad;
            }
        }
    }
    int32_t m = -1;
    uint64_t mx = NONE;   // the exit of stripe m
    unsigned long long mine = 0;
    if (cached) {
#pragma unroll
        for (int i = 0; i < KL; ++i) {
            if (b + i < e && c_entry[i] != NONE) { m = (int32_t)(b + i); mx = c_exit[i]; }
            mine += c_count[i];
        }
    } else {
        for (uint32_t s = b; s < e; ++s) {
            const StripeRes r = sres[s];
            if (r.entry != NONE) { m = (int32_t)s; mx = r.exit; }
            mine += r.count;
        }
    }
    int32_t im = m;
    uint64_t ix = mx;
    unsigned long long is = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t om = __shfl_up(im, d, 64);
        const uint64_t ox = __shfl_up(ix, d, 64);
        const unsigned long long os = __shfl_up(is, d, 64);
        if (lane >= d) {
            if (om > im) { im = om; ix = ox; }
            is += os;
        }
    }
    if (lane == 63) { wm[wv] = im; wx[wv] = ix; wsum[wv] = is; }
    __syncthreads();
    int32_t pm = -1;
    uint64_t px = NONE;
    unsigned long long ps = 0, all_recs = 0;
    for (int i = 0; i < LT / 64; ++i) {
        if (i < wv) {
            if (wm[i] > pm) { pm = wm[i]; px = wx[i]; }
            ps += wsum[i];
        }
        all_recs += wsum[i];
    }
    const int32_t xm = __shfl_up(im, 1, 64);
    const uint64_t xx = __shfl_up(ix, 1, 64);
    const unsigned long long xs = __shfl_up(is, 1, 64);
    int32_t run0 = pm;                       // the last stripe with records before the chunk ...
    uint64_t xrun0 = px;                     // ... and its exit
    if (lane && xm > pm) { run0 = xm; xrun0 = xx; }
    if (soff) {
        unsigned long long at = (lane ? xs : 0ull) + ps;
        if (cached) {
#pragma unroll
            for (int i = 0; i < KL; ++i) if (b + i < e) { soff[b + i] = at; at += c_count[i]; }
        } else {
            for (uint32_t s = b; s < e; ++s) { soff[s] = at; at += sres[s].count; }
        }
    }

    // pass 1: consistency of every stripe with its predecessor's exit
    int32_t run = run0;
    if (cached) {
        uint64_t xrun = run0 >= 0 ? xrun0 : NONE;   // the exit of stripe `run`
#pragma unroll
        for (int i = 0; i < KL; ++i) {
            const uint32_t s = b + i;
            if (s >= e) break;
            StripeDesc d;
            d.seg = c_seg[i]; d.t_begin = c_tb[i]; d.t_end = c_te[i]; d.pad = 0;
            const bool first = c_first[i] != 0u;    // (the host marks a segment's first stripe)
            bool bad = false, after_err = false;
            if (!first) {
                const uint64_t xp = run >= 0 ? xrun : NONE;
                if (xp == ERRP) after_err = true;
                else if (c_entry[i] == NONE) bad = xp < stripe_hi(d, segs[d.seg], tile);   // (a pass-through stripe)
                else bad = (c_entry[i] != xp);
            }
            if (bad && !after_err) atomicMin(&seg_bad[d.seg], s);
            if (c_kind[i] != 0 && !after_err && !bad) atomicMin(&seg_err[d.seg], s);
            if (c_entry[i] != NONE) { run = (int32_t)s; xrun = c_exit[i]; }
        }
    } else
    for (uint32_t s = b; s < e; ++s) {
        const StripeRes r = sres[s];
        const StripeDesc d = stripes[s];
        const SegDesc g = segs[d.seg];
        const bool first = (s == g.stripe0);
        bool bad = false, after_err = false;
        if (!first) {
            const uint64_t xp = run >= 0 ? sres[run].exit : NONE;
            if (xp == ERRP) after_err = true;
            else if (r.entry == NONE) bad = xp < stripe_hi(d, g, tile);
            else bad = (r.entry != xp);
        }
        if (bad && !after_err) atomicMin(&seg_bad[d.seg], s);
        if (r.err_kind != 0 && !after_err && !bad) atomicMin(&seg_err[d.seg], s);
        if (r.entry != NONE) run = (int32_t)s;
    }
    __syncthreads();
    // A segment whose first inconsistent stripe precedes its first error stripe is unresolved;
    // one whose error comes first has its true first error.  Segments are independent chains.
    for (uint32_t g = tid; g < n_segs; g += LT) {
        const uint32_t bb = __hip_atomic_load(&seg_bad[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t ee = __hip_atomic_load(&seg_err[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ee != ~0u && ee < bb) atomicMin(&first_problem, g);     // first segment with a resolved error
    }
    __syncthreads();
    const uint32_t fe = first_problem;       // segments after it are never reached (engine.rs:56 `?`)
    __syncthreads();
    if (tid == 0) first_problem = ~0u;
    __syncthreads();
    for (uint32_t g = tid; g < n_segs && g < fe; g += LT) {
        const uint32_t bb = __hip_atomic_load(&seg_bad[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (bb != ~0u) atomicMin(&first_problem, g);                // first unresolved segment
    }
    __syncthreads();
    const uint32_t fu = first_problem;
    const bool unresolved = fu != ~0u;
    // pass 2: re-walk list, in every segment before the first resolved error.  A stripe whose
    // entry disagrees with the chain so far is inconsistent (owned bit 1, every stripe's bits are
    // rewritten here); it is listed (bit 0) only when its predecessor is consistent, so its entry
    // is the predecessor's exit.  Its re-walk walks on into the inconsistent stripes after it
    // (k_replay, redo pass), so a run of wrong speculations is one pass, not one per stripe.
    if (unresolved) {
        // (two sweeps: the first flags the inconsistent stripes, the second lists the first of each
        // run; the flags of a neighbouring chunk are read only after the barrier)
        for (int sweep = 0; sweep < 2; ++sweep) {
            run = run0;
            for (uint32_t s = b; s < e; ++s) {
                const StripeRes r = sres[s];
                const StripeDesc d = stripes[s];
                const SegDesc g = segs[d.seg];
                uint32_t own = 0;
                if (d.seg < fe && s != g.stripe0) {
                    const uint64_t xp = run >= 0 ? sres[run].exit : NONE;
                    bool bad = false;
                    if (xp != ERRP) {
                        if (r.entry == NONE) bad = xp < stripe_hi(d, g, tile);
                        else bad = (r.entry != xp);
                    }
                    own = bad ? 2u : 0u;
                    if (sweep == 1 && bad) {
                        const uint32_t se = __hip_atomic_load(&seg_err[d.seg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const bool prev_bad =
                            (__hip_atomic_load(&sres[s - 1].owned, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2u) != 0u;
                        // a predecessor exit short of this stripe lands in a pass-through stripe in
                        // between, which is inconsistent too and listed or walked first
                        if (!prev_bad && s < se && xp >= stripe_lo(d, g, tile)) {
                            own = 3u;
                            const uint32_t i = atomicAdd(&nredo, 1u);
                            if (i < redo_cap) { redo[i].stripe = s; redo[i].pad = 0; redo[i].entry = xp; }
                        }
                    }
                }
                // (sweep 1 changes bit 0 only: a neighbour reading bit 1 sees the same either way)
                __hip_atomic_store(&sres[s].owned, own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (r.entry != NONE) run = (int32_t)s;
            }
            __syncthreads();
        }
    }
    __syncthreads();
    if (tid == 0) {
        LinkResult L;
        L.first_problem_seg = unresolved ? fu : fe;
        L.n_redo = nredo < redo_cap ? nredo : redo_cap;
        L.passes = res->passes + 1;
        L.err_kind = 0; L.err_seg = 0; L.err_pos = 0; L.err_aux = 0;
        if (unresolved) {
            L.status = 3;
        } else if (fe == ~0u) {
            L.status = 0;
            if (soff) ctr->total_tuples = all_recs;
        } else {
            const StripeRes r = sres[__hip_atomic_load(&seg_err[fe], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)];
            L.status = 1;
            L.err_kind = r.err_kind;
            L.err_seg = fe;
            L.err_pos = r.err_pos;
            L.err_aux = r.err_aux;
        }
        *res = L;
        if (hres) {   // the host's pinned mirror (fine-grained), written straight: no copy on the stream
            *hres = L;
            const uint32_t ov = ctr->overflow;
            hctr->pool_cursor = ctr->pool_cursor;
            hctr->overflow = ov;
            hctr->piece_done = ctr->piece_done;
            hctr->total_tuples = (L.status == 0 && soff) ? all_recs : ctr->total_tuples;
            hctr->crc_fail = 0;   // (k_compact_s adds its failures here)
            if (L.status == 0 && ov == 0u) {   // a clean pass: the block is cleared for the next call
                res->passes = 0;
                ctr->pool_cursor = 0;
                ctr->total_tuples = 0;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// The ordered gather pool -> out.
// ---------------------------------------------------------------------------------------
constexpr int CT = 256;           // threads per compaction block
constexpr int CB = CT;            // tiles per chunk of k_compact_s

// One workgroup per stripe (the stripe's output offset from k_link, so no separate scan of the
// tile counts): the stripe's tiles in chunks of CB, each chunk's tile offsets scanned in LDS.
// Thread k2 moves half k2 & 1 of tuple k2 >> 1 as one 16-B load and store, so a wave's loads and
// stores are 1 KiB contiguous; the second half holds val_len, crc32, key_tag, op and flags, so
// its thread also does the expected-CRC check, and moves the key prefix when the call keeps one
// (kpool -> kout, the fold's keys) and writes (key tag, key length) beside it (ktk).
//
// Linked mode (scnt != null, the replay pipeline's common case: no k_link before it).  Each
// workgroup links its own stripe: its speculated entry must be the exit of the last earlier stripe
// of the segment with a record start (a stripe without one must be crossed by that exit), and it
// must hold no error.  Its output offset is the sum of the earlier stripes' counts (scnt, dense,
// written by k_replay).  A stripe that fails either test sets hctr->unlinked and moves nothing;
// the host then runs k_link and this kernel in its plain mode, which rewrite every output slot.
// Workgroup 0 mirrors the pool counters to the host and clears the other link + counters block
// (lc_next, the next call's), the last workgroup writes the total.
__device__ __forceinline__ bool stripe_links(const SegDesc *__restrict__ segs, const StripeDesc *__restrict__ stripes,
                                             const StripeRes *__restrict__ sres, uint32_t s, uint32_t tile) {
    const StripeRes r = sres[s];
    const StripeDesc d = stripes[s];
    if (r.err_kind != 0u) return false;
    if (d.pad) return true;                 // the segment's first stripe: its entry is offset 0
    uint32_t j = s - 1;                     // (the segment's first stripe always has a record start)
    while (sres[j].entry == NONE && !stripes[j].pad) --j;
    const StripeRes p = sres[j];
    if (p.entry == NONE || p.exit == ERRP || p.exit == NONE) return false;
    if (r.entry == NONE) return p.exit >= stripe_hi(d, segs[d.seg], tile);   // a pass-through stripe
    return r.entry == p.exit;
}

__global__ __launch_bounds__(CT) void k_compact_s(const SegDesc *__restrict__ segs, const StripeDesc *__restrict__ stripes,
                                                  const StripeRes *__restrict__ sres,
                                                  const uint64_t *__restrict__ soff, const TileRes *__restrict__ tres,
                                                  const kvr_tuple *__restrict__ pool, uint64_t pool_cap,
                                                  kvr_tuple *__restrict__ out, uint64_t out_cap,
                                                  const uint32_t *__restrict__ expected, uint64_t n_expected,
                                                  Counters *ctr, const LinkResult *__restrict__ link,
                                                  const uint4 *__restrict__ kpool, uint4 *__restrict__ kout,
                                                  uint32_t *__restrict__ ktk, Counters *hctr,
                                                  const uint32_t *__restrict__ scnt, uint32_t n_stripes, uint32_t tile,
                                                  uint4 *__restrict__ lc_next, const PieceRun *__restrict__ prun,
                                                  const uint2 *__restrict__ pcrc) {
    __shared__ uint64_t off[CB + 1];
    __shared__ uint64_t part[CT];
    __shared__ uint32_t s_ok;
    uint64_t o_lk = 0;                      // linked mode: this stripe's output offset
    if (scnt) {
        const uint32_t ov = ctr->overflow;
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) { hctr->pool_cursor = ctr->pool_cursor; hctr->overflow = ov; hctr->piece_done = ctr->piece_done; }
            if (threadIdx.x < LC_BLOCK / 16) lc_next[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
        }
        if (ov) return;
        const uint32_t s = blockIdx.x;
        if (threadIdx.x == 0) s_ok = stripe_links(segs, stripes, sres, s, tile) ? 1u : 0u;
        // (16-B loads, four counts each, unrolled: one or two round trips at 4096 stripes instead
        // of one per 256 counts)
        unsigned long long a = 0;
        const uint32_t s4 = s >> 2;
        const uint4 *const sc4 = reinterpret_cast<const uint4 *>(scnt);
#pragma unroll 4
        for (uint32_t i = threadIdx.x; i < s4; i += CT) {
            const uint4 v = sc4[i];
            a += (unsigned long long)v.x + v.y + v.z + v.w;
        }
        for (uint32_t i = (s4 << 2) + threadIdx.x; i < s; i += CT) a += scnt[i];
        for (int d = 32; d >= 1; d >>= 1) a += __shfl_xor(a, d, 64);
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
        __syncthreads();
        for (int i = 0; i < CT / 64; ++i) o_lk += part[i];
        if (!s_ok) {
            if (threadIdx.x == 0) atomicOr_system(&hctr->unlinked, 1u);
            return;
        }
        if (s + 1 == n_stripes && threadIdx.x == 0) hctr->total_tuples = o_lk + scnt[s];
        __syncthreads();   // (part is rewritten below)
    } else if (link->status != 0 || ctr->overflow) {
        return;
    }
    const uint64_t o_base = scnt ? o_lk : soff[blockIdx.x];
    uint32_t fails = 0;
    // the tuple of output slot o from pool slot src: half k2 & 1 per thread, the manifest check
    // on the second half (a SET: op in byte 0 of w), the key prefix beside it
    // (the stripe's records k_piece left in run form: the tuple from the run and pcrc)
    const PieceRun pr = prun ? prun[blockIdx.x] : PieceRun{0ull, 0u, 0u, 0u, 0u, 0u, 0u};
    auto move = [&](uint64_t src, uint64_t o, uint32_t half) {
        if (src >= pool_cap) return;
        uint4 v;
        const uint64_t q = src - pr.first;
        if (q < pr.n) {
            if (half) {
                const uint2 c = pcrc[src];
                v = make_uint4(pr.vu, c.x, c.y, 0u);
            } else {
                const uint64_t ro = pr.Pe + q * pr.L;
                v = make_uint4((uint32_t)ro, (uint32_t)(ro >> 32), pr.seg, pr.ku);
            }
        } else {
            v = reinterpret_cast<const uint4 *>(pool + src)[half];
        }
        if (half && expected && o < n_expected && (v.w & 255u) == 0u) {
            v.w |= KVR_TF_VERIFIED << 8;
            if (expected[o] != v.y) { v.w |= KVR_TF_CRC_FAIL << 8; ++fails; }
        }
        if (o < out_cap) {
            reinterpret_cast<uint4 *>(out + o)[half] = v;
            if (half && kout) kout[o] = kpool[src];
            // (key tag, key length) for the fold's estimate and partition: each half has one of them,
            // so a wave's stores are 256 B contiguous
            if (ktk) ktk[2 * o + (half ^ 1u)] = half ? v.z : v.w;
        }
    };
    // the CRC failures go to the host's pinned mirror (a system-scope atomic, only for a wave
    // that found any), or to the device counters
    auto finish = [&]() {
        for (int d = 32; d >= 1; d >>= 1) fails += __shfl_xor(fails, d, 64);
        if ((threadIdx.x & 63) == 0 && fails) {
            if (hctr) atomicAdd_system(&hctr->crc_fail, (unsigned long long)fails);
            else atomicAdd(&ctr->crc_fail, (unsigned long long)fails);
        }
    };
    const uint64_t run = sres[blockIdx.x].pool_run;
    if (run != NONE) {   // the stripe's tuples are one run of the pool: a straight copy
        const uint64_t n = sres[blockIdx.x].count, o0 = o_base;
        if (n && pr.n == n && run == pr.first) {
            // every record of the stripe in run form (k_piece ran it to its end): a thread builds
            // whole tuples from the run and pcrc, with the manifest check
            // (RF records a thread per round, their loads issued before any store: one round trip a round)
            constexpr int RF = 4;
            const uint64_t lim = o0 + n <= out_cap ? n : (out_cap > o0 ? out_cap - o0 : 0ull);
            for (uint64_t k0 = threadIdx.x; k0 < lim; k0 += (uint64_t)CT * RF) {
                uint2 c[RF];
                uint32_t e[RF];
#pragma unroll
                for (int i = 0; i < RF; ++i) {
                    const uint64_t k = k0 + (uint64_t)i * CT, o = o0 + k;
                    c[i] = k < lim ? pcrc[run + k] : make_uint2(0u, 0u);
                    e[i] = k < lim && expected && o < n_expected ? expected[o] : 0u;
                }
#pragma unroll
                for (int i = 0; i < RF; ++i) {
                    const uint64_t k = k0 + (uint64_t)i * CT, o = o0 + k;
                    if (k >= lim) break;
                    const uint64_t ro = pr.Pe + k * pr.L;
                    uint32_t fw = 0;
                    if (expected && o < n_expected) {
                        fw = KVR_TF_VERIFIED << 8;
                        if (e[i] != c[i].x) { fw |= KVR_TF_CRC_FAIL << 8; ++fails; }
                    }
                    uint4 *const dst = reinterpret_cast<uint4 *>(out + o);
                    dst[0] = make_uint4((uint32_t)ro, (uint32_t)(ro >> 32), pr.seg, pr.ku);
                    dst[1] = make_uint4(pr.vu, c[i].x, c[i].y, fw);
                    if (kout) kout[o] = kpool[run + k];
                    if (ktk) { ktk[2 * o] = c[i].y; ktk[2 * o + 1] = pr.ku; }
                }
            }
            finish();
            return;
        }
        for (uint64_t k2 = threadIdx.x; k2 < 2 * n; k2 += CT) move(run + (k2 >> 1), o0 + (k2 >> 1), (uint32_t)k2 & 1u);
        finish();
        return;
    }
    const StripeDesc sd = stripes[blockIdx.x];
    const uint32_t tile0 = segs[sd.seg].tile0;
    const uint32_t t_end = tile0 + sd.t_end;
    uint64_t carry = o_base;
    for (uint32_t tb = tile0 + sd.t_begin; tb < t_end; tb += CB) {
        const uint32_t nt = min((uint32_t)CB, t_end - tb);
        const uint32_t t = tb + threadIdx.x;
        const uint64_t cnt = threadIdx.x < nt ? tres[t].count : 0u;
        part[threadIdx.x] = cnt;
        __syncthreads();
        for (int d = 1; d < CT; d <<= 1) {
            const uint64_t o = threadIdx.x >= (uint32_t)d ? part[threadIdx.x - d] : 0ull;
            __syncthreads();
            part[threadIdx.x] += o;
            __syncthreads();
        }
        off[threadIdx.x] = carry + part[threadIdx.x] - cnt;
        const uint64_t ctotal = part[CT - 1];
        __syncthreads();
        const uint64_t b0 = carry;
        for (uint64_t k2 = threadIdx.x; k2 < 2 * ctotal; k2 += CT) {
            const uint64_t k = k2 >> 1;
            const uint32_t half = (uint32_t)k2 & 1u;
            uint32_t lo_i = 0, hi_i = nt - 1;       // last tile i with off[i] - b0 <= k
            while (lo_i < hi_i) {
                const uint32_t mid = (lo_i + hi_i + 1) >> 1;
                if (off[mid] - b0 <= k) lo_i = mid; else hi_i = mid - 1;
            }
            const uint64_t o = b0 + k;
            const TileRes &tr = tres[tb + lo_i];
            const uint64_t r = o - off[lo_i];
            const uint64_t src = r < tr.count1 ? tr.pool_off + r : tr.pool_off2 + (r - tr.count1);
            move(src, o, half);
        }
        carry += ctotal;
        __syncthreads();   // (off and part are rewritten by the next chunk)
    }
    finish();
}

// ---------------------------------------------------------------------------------------
// Synthetic generator, device side.  Layout (record offsets + params) comes from the host.
// ---------------------------------------------------------------------------------------
struct GenRecDev {
    uint64_t off;
    uint64_t key_id;
    uint64_t vseed;
    int64_t  flip_bit;
    uint32_t op, vlen;
};

__global__ void k_gen_fill(const GenRecDev *__restrict__ recs, uint64_t n_rec, uint8_t *__restrict__ buf) {
    for (uint64_t r = blockIdx.x; r < n_rec; r += gridDim.x) {
        const GenRecDev g = recs[r];
        uint8_t *p = buf + g.off;
        if (threadIdx.x == 0) {
            p[0] = (uint8_t)g.op;
            p[1] = (uint8_t)KVR_GEN_KEY_LEN; p[2] = 0; p[3] = 0; p[4] = 0;
            uint8_t key[KVR_GEN_KEY_LEN];
            kvr_gen_key(g.key_id, key);
            for (uint32_t i = 0; i < KVR_GEN_KEY_LEN; ++i) p[5 + i] = key[i];
            if (g.op == 0) {
                uint8_t *q = p + 5 + KVR_GEN_KEY_LEN;
                q[0] = (uint8_t)g.vlen; q[1] = (uint8_t)(g.vlen >> 8);
                q[2] = (uint8_t)(g.vlen >> 16); q[3] = (uint8_t)(g.vlen >> 24);
            }
        }
        if (g.op == 0) {
            uint8_t *v = p + 9 + KVR_GEN_KEY_LEN;
            const uint64_t fb = g.flip_bit >= 0 ? (uint64_t)g.flip_bit >> 3 : ~0ull;
            const uint8_t fm = g.flip_bit >= 0 ? (uint8_t)(1u << (g.flip_bit & 7)) : 0;
            for (uint64_t j8 = threadIdx.x; j8 * 8 < g.vlen; j8 += blockDim.x) {
                const uint64_t w = kvr_mix64(g.vseed + j8);
                for (int b = 0; b < 8; ++b) {
                    const uint64_t j = j8 * 8 + b;
                    if (j < g.vlen) v[j] = (uint8_t)(w >> (8 * b)) ^ (j == fb ? fm : (uint8_t)0);
                }
            }
        }
    }
}

__global__ void k_gen_manifest(const GenRecDev *__restrict__ recs, uint64_t n_rec,
                               const uint32_t *__restrict__ g_crc, uint32_t *__restrict__ expected) {
    __shared__ uint32_t T[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = g_crc[i];
    __syncthreads();
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_rec;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const GenRecDev g = recs[r];
        if (g.op != 0) { expected[r] = 0; continue; }
        uint32_t c = ~0u;
        for (uint64_t j8 = 0; j8 * 8 < g.vlen; ++j8) {
            const uint64_t w = kvr_mix64(g.vseed + j8);
            const uint32_t nb = (g.vlen - j8 * 8) < 8 ? (uint32_t)(g.vlen - j8 * 8) : 8u;
            for (uint32_t b = 0; b < nb; ++b) c = (c >> 8) ^ T[(c ^ (uint32_t)(w >> (8 * b))) & 0xFFu];
        }
        expected[r] = ~c;
    }
}

}  // namespace kvr
