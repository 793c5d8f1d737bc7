/*
 * kvr_compact.hip — the live-record rewrite (BASELINE config 4).
 *
 * What the reference's compaction is meant to do (README.md:283-287: "collect all live keys,
 * write to new segments, delete old segments"); its compaction.rs:9-29 only deletes the files
 * (SURVEY R3).  Parity target: a reference replay (engine.rs:79-154) of the new segments
 * reproduces the pre-compaction map (tests/store_integration.rs:22-31, now across a reopen).
 *
 * Input: the replay tuples of the store (kvr_replay, in (segment, offset) order) and the
 * segment bytes in HBM.  Device pipeline, one stream:
 *   k_fold_claim    every tuple into an open-addressing table of 32-B entries keyed by its
 *                   key bytes (key_tag = CRC-32 of the key as the hash): an atomicCAS of
 *                   (tag << 32 | tuple) claims an empty entry for a key's first tuple, whose
 *                   length and first 16 key bytes the claimer copies into the entry; a tuple
 *                   that meets its own tag stops there (tentatively)
 *   k_fold_verify   every tuple checks its key against the entry it stopped at (length and the
 *                   16-B prefix from the entry itself, the rest of a longer key from the
 *                   representative's bytes) and, when equal, keeps the key's LAST tuple index by
 *                   atomicMin of ~index — the last-writer-wins fold of engine.rs:137 / :141 as
 *                   an associative max.  Both kernels walk the tuples latest first: the claimer
 *                   (which stores its own index as best) is then usually the key's last tuple,
 *                   and a tuple below the best already stored skips its atomic (device-scope
 *                   atomics execute at the memory side, about 20 G/s chip-wide).  A tag collision between two keys sends the tuple to the
 *                   next round, which resumes its probe one entry further (rounds until no tuple
 *                   is left; distinct keys sharing a CRC-32 are a few hundred per million keys)
 *   k_fold_part / k_fold_lds   (the default first round, below) the same fold per 2048-entry
 *                   range of the table in one workgroup's LDS; the claim and verify kernels then
 *                   only take the few tuples whose probe leaves their range
 *   k_live_ent      per claimed entry: its key's last tuple is live iff it is a SET: flag, size
 *                   9 + k + v
 *   (scan)          exclusive sums of sizes (output offsets) and live flags (dense index)
 *   k_scatter       dense live list (source address, output offset)
 *   k_gather_r      one wave per live record: the record's bytes copied verbatim (the framing of
 *                   engine.rs:169-173 is the record's own), its 16-B aligned output body as 16 B
 *                   per lane, the unaligned head and tail bytes one per lane
 *   k_cuts          new-segment boundaries: a segment starts at the first live record whose
 *                   output offset is >= k * seg_target
 * Bytes moved (the roofline): live bytes read + live bytes written + 32 B per
 * tuple of the fold; HBM-bound.
 */
#ifndef KVR_COMPACT_HIP
#define KVR_COMPACT_HIP

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kvr_device.h"

namespace kvr {

constexpr uint32_t HT_EMPTY = 0xFFFFFFFFu;
constexpr int CT_GATHER = 256;       // threads per gather workgroup (4 records at a time)

__host__ __device__ __forceinline__ uint32_t ht_mix(uint32_t h) {   // the key_tag is a CRC: spread it
    h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
    return h;
}

__device__ __forceinline__ const uint8_t *key_ptr(const SegDesc *segs, const kvr_tuple &t) {
    return segs[t.seg_idx].base + t.rec_off + 5;   // [op][klen u32][key] (engine.rs:169-171)
}

// n bytes at pa and pb equal: 16-byte chunks of independent (predicated) loads, so a compare costs
// one memory round trip per 16 bytes instead of one per byte
__device__ bool bytes_eq(const uint8_t *pa, const uint8_t *pb, uint32_t n) {
    for (uint32_t i = 0; i < n; i += 16) {
        const uint32_t m = n - i < 16u ? n - i : 16u;
        uint32_t diff = 0;
#pragma unroll
        for (uint32_t q = 0; q < 16; ++q) {
            const uint32_t x = q < m ? pa[i + q] : 0u, y = q < m ? pb[i + q] : 0u;
            diff |= x ^ y;
        }
        if (diff) return false;
    }
    return true;
}

// key bytes equal (the tags and lengths are compared first)
__device__ bool key_eq(const SegDesc *segs, const kvr_tuple &a, const kvr_tuple &b) {
    if (a.key_tag != b.key_tag || a.key_len != b.key_len) return false;
    return bytes_eq(key_ptr(segs, a), key_ptr(segs, b), a.key_len);
}

// the fold table: one 32-B entry per slot, at least 2 n slots (a power of two)
struct __align__(32) FoldEnt {
    unsigned long long tagrep;   // (key_tag << 32) | representative tuple; FE_EMPTY: free
    uint32_t best;               // ~(the key's last tuple index); every claimed entry has one
    uint32_t klen;               // the representative's key length
    uint32_t key[4];             // its first 16 key bytes, zero padded
};
static_assert(sizeof(FoldEnt) == 32, "fold entry");
constexpr unsigned long long FE_EMPTY = ~0ull;   // the table is memset to 0xFF


// bytes [0, min(klen, 16)) of the key of tuple t, zero padded.  Aligned dword loads: a dword is
// read only if it starts before the segment's end, so it holds a segment byte and cannot cross
// into an unmapped page, whatever padding the caller's buffer has.  (Two aligned 16-B loads
// measured slower: 401 vs 333 us for k_fold_verify on cfg2.)
__device__ __forceinline__ void key_prefix16(const SegDesc &g, const kvr_tuple &t, uint32_t w[4]) {
#ifdef KVR_FOLD_NOKEY   // timing diagnostic only (build.py variant foldnokey): no key reads, wrong results
    w[0] = w[1] = w[2] = w[3] = t.key_tag;
    return;
#endif
    const uintptr_t p = reinterpret_cast<uintptr_t>(g.base) + t.rec_off + 5;
    const uintptr_t end = reinterpret_cast<uintptr_t>(g.base) + g.len;
    const uintptr_t pa = p & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)(p & 3u);
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
        d[k] = pa + 4u * k < end ? *reinterpret_cast<const uint32_t *>(pa + 4u * k) : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t x = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
        const int valid = (int)t.key_len - 4 * j;   // bytes of this dword inside the key
        w[j] = valid >= 4 ? x : valid <= 0 ? 0u : (x & ((1u << (8 * valid)) - 1u));
    }
}

// distinct-key estimate that sizes the fold table (HyperLogLog, 2^14 registers over the key
// tags): each workgroup keeps registers in LDS and writes them out; k_hll_merge takes the max
// over the workgroups.  A smaller table stays in the caches (the 256-MiB table for cfg2's 4 M
// tuples holds 1 M keys).
constexpr int HLL_P = 14, HLL_M = 1 << HLL_P, HLL_T = 1024;   // (1024 threads, two workgroups per CU: 81 -> 54 us on cfg4)
__device__ __forceinline__ uint32_t hll_mix(uint32_t h) {   // independent of ht_mix's bits
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return h;
}
// (tk: (key tag, key length) per tuple, written by k_compact_s beside the key prefixes; else the tuples')
__global__ void __launch_bounds__(HLL_T) k_hll(const kvr_tuple *__restrict__ tup, const uint2 *__restrict__ tk,
                                               uint64_t n, uint8_t *__restrict__ part) {
    __shared__ uint32_t reg[HLL_M];
    for (int j = threadIdx.x; j < HLL_M; j += HLL_T) reg[j] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * HLL_T + threadIdx.x; i < n; i += (uint64_t)gridDim.x * HLL_T) {
        const uint32_t x = hll_mix(tk ? tk[i].x : tup[i].key_tag);
        const uint32_t rank = (uint32_t)__clz((x << HLL_P) | (1u << (HLL_P - 1))) + 1u;
        atomicMax(&reg[x >> (32 - HLL_P)], rank);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < HLL_M; j += HLL_T) part[(uint64_t)blockIdx.x * HLL_M + j] = (uint8_t)reg[j];
}
// byte-wise max of two words of four registers each
__device__ __forceinline__ uint32_t max4u8(uint32_t a, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 32; k += 8) r |= max((a >> k) & 255u, (b >> k) & 255u) << k;
    return r;
}

// thread (g, s) takes register group g (16 registers, one 16-B load per partition) over
// partitions s, s + HLL_MR, ...; 4 groups per workgroup, so HLL_M / 64 workgroups share the
// partitions; an LDS tree folds the HLL_MR rows
constexpr int HLL_MERGE_T = 256, HLL_MG = 4, HLL_MR = HLL_MERGE_T / HLL_MG;
__global__ void __launch_bounds__(HLL_MERGE_T) k_hll_merge(const uint8_t *__restrict__ part, uint32_t n_parts,
                                                           uint8_t *__restrict__ out) {
    __shared__ uint4 acc[HLL_MR][HLL_MG];
    const uint32_t gl = threadIdx.x % HLL_MG, sl = threadIdx.x / HLL_MG;
    const uint32_t g = blockIdx.x * HLL_MG + gl;   // register group: registers 16 g .. 16 g + 15
    uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll 4
    for (uint32_t b = sl; b < n_parts; b += HLL_MR) {
        const uint4 v = reinterpret_cast<const uint4 *>(part + (uint64_t)b * HLL_M)[g];
        m = make_uint4(max4u8(m.x, v.x), max4u8(m.y, v.y), max4u8(m.z, v.z), max4u8(m.w, v.w));
    }
    acc[sl][gl] = m;
    __syncthreads();
    for (uint32_t d = HLL_MR / 2; d > 0; d >>= 1) {
        if (sl < d) {
            const uint4 v = acc[sl + d][gl], a = acc[sl][gl];
            acc[sl][gl] = make_uint4(max4u8(a.x, v.x), max4u8(a.y, v.y), max4u8(a.z, v.z), max4u8(a.w, v.w));
        }
        __syncthreads();
    }
    if (sl == 0) reinterpret_cast<uint4 *>(out)[g] = acc[0][gl];
}

// the fold table's size on the device, so no host round trip sits between the estimate and the
// claims: fsz[0] = entries - 1 (a power of two minus one), fsz[2..3] = the estimate (uint64).
// The same arithmetic as the host's hll_estimate (kvr_api.hip), summed in a different order.
constexpr int HLL_SIZE_T = 1024;   // 16 registers per thread, one 16-B load each
static_assert(HLL_M == 16 * HLL_SIZE_T, "k_hll_size: one 16-B word of registers per thread");
__global__ void __launch_bounds__(HLL_SIZE_T) k_hll_size(const uint8_t *__restrict__ reg, uint64_t full_slots,
                                                         uint32_t *__restrict__ fsz) {
    __shared__ double ss[HLL_SIZE_T];
    __shared__ uint32_t sz[HLL_SIZE_T];
    double sum = 0;
    uint32_t zeros = 0;
    {
        const uint4 q = reinterpret_cast<const uint4 *>(reg)[threadIdx.x];
        const uint32_t wds[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t r = (wds[i >> 2] >> (8 * (i & 3))) & 255u;
            sum += ldexp(1.0, -(int)r);
            zeros += r == 0u;
        }
    }
    ss[threadIdx.x] = sum;
    sz[threadIdx.x] = zeros;
    __syncthreads();
    for (int d = HLL_SIZE_T / 2; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) { ss[threadIdx.x] += ss[threadIdx.x + d]; sz[threadIdx.x] += sz[threadIdx.x + d]; }
        __syncthreads();
    }
    if (threadIdx.x) return;
    const double m = HLL_M, alpha = 0.7213 / (1.0 + 1.079 / m);
    double e = alpha * m * m / ss[0];
    if (e <= 2.5 * m && sz[0]) e = m * log(m / sz[0]);
    const double two32 = 4294967296.0;
    if (e > two32 / 30.0) e = e < two32 ? -two32 * log(1.0 - e / two32) : two32;
    uint64_t want = 16;
    while ((double)want < 1.6 * e + 1024.0) want <<= 1;
    const uint64_t slots = want < full_slots ? want : full_slots;
    fsz[0] = (uint32_t)(slots - 1);
    *reinterpret_cast<uint64_t *>(fsz + 2) = (uint64_t)e;
}
__global__ void k_fold_setsize(uint32_t *__restrict__ fsz, uint32_t mask) {
    fsz[0] = mask;
    *reinterpret_cast<uint64_t *>(fsz + 2) = 0;
}
// free entries (all ones) for the table size on the device; grid-stride
__global__ void k_fent_clear(FoldEnt *__restrict__ ent, const uint32_t *__restrict__ fsz) {
    const uint32_t mask = fsz[0];
    const uint4 ff = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h <= mask; h += (uint64_t)gridDim.x * blockDim.x) {
        reinterpret_cast<uint4 *>(&ent[h])[0] = ff;
        reinterpret_cast<uint4 *>(&ent[h])[1] = ff;
    }
}

// one probe round: tuple i (all tuples in round 0, list[] afterwards) walks from its start entry
// (the tag's home slot in round 0, slot[i] afterwards) to the first entry that is free (claimed
// here) or holds its tag (verified by k_fold_verify)
// (n_dev: a later round launched before the host knows its size reads it here; n caps it at the
// grid, and the host checks afterwards that no round was larger)
// (kd: the tuples' key prefixes, which k_replay wrote when the call asked for them: one sequential
// 16-B read instead of reading the key in the segment bytes at random; null: from the segments)
template <bool PRE>
__global__ void k_fold_claim(const kvr_tuple *__restrict__ tup, uint64_t n, const uint32_t *__restrict__ n_dev,
                             const uint32_t *__restrict__ list, const SegDesc *__restrict__ segs,
                             FoldEnt *__restrict__ ent, const uint32_t *__restrict__ fsz,
                             uint32_t *__restrict__ slot, uint32_t *__restrict__ full, const uint4 *__restrict__ kd) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n_dev && *n_dev < n) n = *n_dev;
    if (g >= n) return;
    const uint32_t mask = fsz[0];
    // latest tuples first (workgroups start in index order): a key's claimer is then usually its
    // last tuple, which k_fold_verify exploits
    const uint32_t i = list ? list[n - 1 - g] : (uint32_t)(n - 1 - g);
    const kvr_tuple t = tup[i];
    uint32_t h = list ? slot[i] : (ht_mix(t.key_tag) & mask);
    const unsigned long long mine = ((unsigned long long)t.key_tag << 32) | i;
    uint32_t w[4];   // PRE: the key prefix, loaded alongside the probe (only a claimer stores it)
    if (PRE && !kd) key_prefix16(segs[t.seg_idx], t, w);
    for (uint32_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
        unsigned long long v = __hip_atomic_load(&ent[h].tagrep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v == FE_EMPTY) {
            v = atomicCAS(&ent[h].tagrep, FE_EMPTY, mine);
            if (v == FE_EMPTY) {   // claimed: this tuple represents its key in entry h
                if (kd) {
                    const uint4 q = kd[i];
                    w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
                } else if (!PRE) {
                    key_prefix16(segs[t.seg_idx], t, w);
                }
                ent[h].best = ~i;   // nobody else writes best during the claims
                ent[h].klen = t.key_len;
                *reinterpret_cast<uint4 *>(ent[h].key) = make_uint4(w[0], w[1], w[2], w[3]);
                slot[i] = h;
                return;
            }
        }
        if ((uint32_t)(v >> 32) == t.key_tag) {
            slot[i] = h;
            return;
        }
    }
    slot[i] = HT_EMPTY;   // the table is full (the distinct-key estimate was low): the host
    atomicAdd(full, 1u);  // folds again with a table of 2 n entries
}

// same key as the entry's representative: keep the last index; else on to the next round
__global__ void k_fold_verify(const kvr_tuple *__restrict__ tup, uint64_t n, const uint32_t *__restrict__ n_dev,
                              const uint32_t *__restrict__ list, const SegDesc *__restrict__ segs,
                              FoldEnt *__restrict__ ent, const uint32_t *__restrict__ fsz,
                              uint32_t *__restrict__ slot, uint32_t *__restrict__ next, uint32_t *__restrict__ n_next,
                              const uint4 *__restrict__ kd) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n_dev && *n_dev < n) n = *n_dev;
    if (g >= n) return;
    const uint32_t mask = fsz[0];
    const uint32_t i = list ? list[n - 1 - g] : (uint32_t)(n - 1 - g);   // latest first
    const uint32_t h = slot[i];
    if (h == HT_EMPTY) return;
    const uint4 a = reinterpret_cast<const uint4 *>(&ent[h])[0];
    const uint32_t rep = a.x;
    if (rep == i) return;   // the claimer stored its own index as best
    bool same = false;
    {
        const kvr_tuple t = tup[i];
        if (a.w == t.key_len) {
            const uint4 k = reinterpret_cast<const uint4 *>(&ent[h])[1];
            uint32_t w[4];
            if (kd) {
                const uint4 q = kd[i];
                w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
            } else {
                key_prefix16(segs[t.seg_idx], t, w);
            }
            same = ((w[0] ^ k.x) | (w[1] ^ k.y) | (w[2] ^ k.z) | (w[3] ^ k.w)) == 0u;
            if (same && t.key_len > 16u)
                same = bytes_eq(key_ptr(segs, tup[rep]) + 16, key_ptr(segs, t) + 16, t.key_len - 16u);
        }
    }
    if (same) {
        // best only grows (as an index): a tuple below the best seen needs no atomic.  Latest
        // first, a key's later tuples are usually done before its earlier ones run, so most
        // tuples skip the (memory-side) atomic.
        if (~a.z < i) atomicMin(&ent[h].best, ~i);
    } else {   // another key with this tag holds entry h: probe on from h + 1 next round
        next[atomicAdd(n_next, 1u)] = i;
        slot[i] = (h + 1) & mask;
    }
}

// ---- the partitioned fold: the table's ranges folded in LDS ----
// Bucket b is the table's slot range [b S, (b + 1) S) (S = FP_S, or the whole table when it is
// smaller).  k_fold_part takes FP_CH tuples per workgroup and writes their records (index, tag,
// length, 16-B key prefix) into the workgroup's own FP_CH-record region, grouped by bucket (whole
// cache lines, no atomics outside LDS), with the region's bucket offsets beside it.  k_fold_lds
// folds one bucket per workgroup in an LDS copy of its range, gathering the bucket's runs from
// every region, with the global claim's probe order (linear from the home slot, first free entry
// or the key's own), and writes the range out, free entries included (no clear).  The random
// traffic of the claims and checks stays in LDS: HBM sees the tuples once, the records twice and
// the table once.  A tuple whose probe runs off the end of its range goes to the global rounds
// (k_fold_claim / k_fold_verify over a list), which go on probing in the table from where it
// stopped: every entry it passed is taken, so the linear-probing invariant holds.
#ifndef KVR_FP_PER
#define KVR_FP_PER 8   // tuples per thread of k_fold_part (build knob)
#endif
// (FP_WMAX: k_fold_lds keeps two words per region in LDS; 1984 lets two 1024-thread workgroups
// share a CU's 160 KiB)
constexpr uint32_t FP_S = 2048, FP_T = 1024, FP_PER = KVR_FP_PER, FP_CH = FP_T * FP_PER, FP_PMAX = 16384,
                   FP_WMAX = 1984;
static_assert(FP_CH <= 8192 && FP_PMAX <= 1u << 19, "k_fold_part packs bucket and rank in 32 bits");
struct __align__(16) FPRec {
    uint32_t i, tag, klen, pad;
    uint4 key;   // the first 16 key bytes, zero padded
};
static_assert(sizeof(FPRec) == 32, "partition record");
struct FPGeom {
    uint32_t mask, s, shift, p;
};
// the partition geometry of the table size on the device (k_hll_size / k_fold_setsize): P ranges
// of S = min(slots, s_lim) entries (s_lim: FP_S, or a smaller power of two as a test knob)
__device__ __forceinline__ FPGeom fp_geom(const uint32_t *fsz, uint32_t s_lim) {
    FPGeom g;
    g.mask = fsz[0];
    const uint64_t slots = (uint64_t)g.mask + 1;
    g.s = slots < s_lim ? (uint32_t)slots : s_lim;
    g.shift = (uint32_t)__builtin_ctz(g.s);
    g.p = (uint32_t)(slots >> g.shift);
    return g;
}

// exclusive prefix sum of a[0, n) in LDS, in place, by the whole block (FP_T threads, each a
// contiguous run of ceil(n / FP_T) entries; wave scans by shuffles, then the FP_T / 64 wave
// totals); returns the sum
__device__ uint32_t block_excl_scan(uint32_t *a, uint32_t n, uint32_t *wsum) {
    const uint32_t t = threadIdx.x, lane = t & 63u, per = (n + FP_T - 1) / FP_T;
    const uint32_t lo = t * per < n ? t * per : n, hi = lo + per < n ? lo + per : n;
    uint32_t s = 0;
    for (uint32_t j = lo; j < hi; ++j) s += a[j];
    uint32_t x = s;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63u) wsum[t >> 6] = x;
    __syncthreads();
    if (t < 64u) {
        uint32_t w = t < FP_T / 64 ? wsum[t] : 0u;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(w, d, 64);
            if (lane >= d) w += y;
        }
        if (t < FP_T / 64) wsum[t] = w;
    }
    __syncthreads();
    uint32_t before = x - s + ((t >> 6) ? wsum[(t >> 6) - 1] : 0u);
    const uint32_t total = wsum[FP_T / 64 - 1];
    for (uint32_t j = lo; j < hi; ++j) {
        const uint32_t v = a[j];
        a[j] = before;
        before += v;
    }
    __syncthreads();
    return total;
}

// workgroup w: tuples [w FP_CH, (w + 1) FP_CH) -> records rec[w FP_CH ..), grouped by bucket;
// woff[w (P + 1) + b] = the first record of bucket b in the region (b = P: the region's count).
// An LDS histogram gives each tuple its rank in its bucket, its prefix sum the buckets' offsets.
__global__ void __launch_bounds__(FP_T, 8) k_fold_part(const kvr_tuple *__restrict__ tup, uint64_t n,
                                                       const SegDesc *__restrict__ segs, const uint4 *__restrict__ kd,
                                                       const uint2 *__restrict__ tk,
                                                       const uint32_t *__restrict__ fsz, uint32_t s_lim,
                                                       FPRec *__restrict__ rec, uint32_t *__restrict__ woff) {
    __shared__ uint32_t hist[FP_PMAX + 1];
    __shared__ uint32_t wsum[FP_T / 64];
    const FPGeom G = fp_geom(fsz, s_lim);
    for (uint32_t j = threadIdx.x; j <= G.p; j += FP_T) hist[j] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * FP_CH + threadIdx.x;
    // bk: bucket << 13 | rank in the region's share of it
    uint32_t bk[FP_PER], tag[FP_PER], kl[FP_PER];
#pragma unroll
    for (int u = 0; u < FP_PER; ++u) {
        const uint64_t i = base + (uint64_t)u * FP_T;
        if (i < n) {
            if (tk) {   // (8 B a tuple instead of the tuple's 32)
                const uint2 q = tk[i];
                tag[u] = q.x;
                kl[u] = q.y;
            } else {
                tag[u] = tup[i].key_tag;
                kl[u] = tup[i].key_len;
            }
            const uint32_t b = (ht_mix(tag[u]) & G.mask) >> G.shift;
            bk[u] = b << 13 | atomicAdd(&hist[b], 1u);
        }
    }
    __syncthreads();
    block_excl_scan(hist, G.p + 1, wsum);
    uint32_t *wo = woff + (uint64_t)blockIdx.x * (G.p + 1);
    for (uint32_t j = threadIdx.x; j <= G.p; j += FP_T) wo[j] = hist[j];
    FPRec *rg = rec + (uint64_t)blockIdx.x * FP_CH;
#pragma unroll
    for (int u = 0; u < FP_PER; ++u) {
        const uint64_t i = base + (uint64_t)u * FP_T;
        if (i >= n) continue;
        FPRec r;
        r.i = (uint32_t)i;
        r.tag = tag[u];
        r.klen = kl[u];
        r.pad = 0;
        if (kd) {
            r.key = kd[i];
        } else {
            const kvr_tuple t = tup[i];
            uint32_t w[4];
            key_prefix16(segs[t.seg_idx], t, w);
            r.key = make_uint4(w[0], w[1], w[2], w[3]);
        }
        rg[hist[bk[u] >> 13] + (bk[u] & 8191u)] = r;
    }
}

// bytes 16 .. klen of two keys equal (the rare long-key check, out of line: its unrolled loads
// would otherwise hold registers through k_fold_lds)
__device__ __attribute__((noinline)) bool key_tail_eq(const SegDesc *segs, const kvr_tuple *tup, uint32_t a,
                                                      uint32_t b, uint32_t klen) {
    return bytes_eq(key_ptr(segs, tup[a]) + 16, key_ptr(segs, tup[b]) + 16, klen - 16u);
}

// append v to list (count *n) from the active lanes of a wave: one atomic per wave
__device__ __forceinline__ void list_push(uint32_t *__restrict__ list, uint32_t *__restrict__ n, uint32_t v) {
    const uint64_t m = __ballot(1);
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(n, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = v;
}

// one workgroup per bucket: the range's entries in LDS; the bucket's records (its run in each of
// the nwg regions, located by a prefix sum over the runs' lengths and a binary search), each thread
// its own records, latest first, with no barrier between them.  A probe step claims a free entry
// (64-bit LDS CAS; the claimer writes the key length and prefix, then publishes its index as the
// entry's best), stops at an entry with the tuple's tag, or moves on.  A tuple that stopped waits
// for the entry to be published (its claimer has done the CAS and writes on without waiting, and
// a claimer of the same wave finishes its writes in the same probe step, before any lane of the
// wave waits), compares its key, and keeps the larger index (an atomicMax only when it is larger:
// latest first, a hot key's later tuples skip it), or probes on.  slot_all: every tuple's entry
// to slot[] (is_last, the sharded compaction); the overflow tuples' restart entries always.
// A bucket folds its latest cap records in LDS (cap_lim, or 4 times the mean bucket, at least
// 16 Ki); a longer bucket (a hot key's) leaves its earlier records to k_fold_hot, which the whole
// device runs: it gets the bucket (hb: bucket, count) and its run arrays (hw), fewer than P / 4
// buckets (cap >= 4 n / P).
#ifndef KVR_FP_U
#define KVR_FP_U 2   // records per thread and step of k_fold_lds (build knob; 4 spills)
#endif
constexpr uint32_t FP_U = KVR_FP_U;
constexpr uint32_t FP_UNPUB = 0xFFFFFFFFu;   // s_best of a claimed entry not yet published (indices < 2^31)
__global__ void __launch_bounds__(FP_T, 8) k_fold_lds(const kvr_tuple *__restrict__ tup, const SegDesc *__restrict__ segs,
                                                      const uint32_t *__restrict__ fsz, uint32_t s_lim,
                                                      const FPRec *__restrict__ rec, const uint32_t *__restrict__ woff,
                                                      uint32_t nwg, FoldEnt *__restrict__ ent, uint32_t *__restrict__ ovl,
                                                      uint32_t *__restrict__ ovn, uint32_t *__restrict__ slot,
                                                      uint32_t slot_all, uint64_t n, uint32_t cap_lim,
                                                      uint32_t *__restrict__ hb, uint32_t *__restrict__ hw,
                                                      uint32_t *__restrict__ hn, uint32_t hot_cap) {
    __shared__ unsigned long long s_tr[FP_S];
    __shared__ uint32_t s_best[FP_S], s_klen[FP_S];
    __shared__ uint4 s_key[FP_S];
    __shared__ uint32_t wsc[FP_WMAX + 1];   // the bucket's first record in run w (prefix sum)
    __shared__ uint32_t wrb[FP_WMAX];       // run w's first record in rec[]
    __shared__ uint32_t wsum[FP_T / 64];
    const FPGeom G = fp_geom(fsz, s_lim);
    const uint32_t b = blockIdx.x;
    if (b >= G.p) return;
    for (uint32_t j = threadIdx.x; j < G.s; j += FP_T) {
        s_tr[j] = FE_EMPTY;
        s_best[j] = FP_UNPUB;
    }
    const uint64_t stride = (uint64_t)G.p + 1;
    for (uint32_t w = threadIdx.x; w <= nwg; w += FP_T) {
        uint32_t len = 0;
        if (w < nwg) {
            const uint32_t o0 = woff[w * stride + b];
            len = woff[w * stride + b + 1] - o0;
            wrb[w] = w * FP_CH + o0;
        }
        wsc[w] = len;
    }
    __syncthreads();
    const uint32_t cnt = block_excl_scan(wsc, nwg + 1, wsum);
    const uint32_t first = b << G.shift;
    const uint64_t mean4 = 4 * (n / G.p);
    const uint32_t cap = cap_lim ? cap_lim : (uint32_t)(mean4 > 16384 ? (mean4 < 0x7FFFFFFF ? mean4 : 0x7FFFFFFF) : 16384);
    uint32_t n_lds = cnt;   // the bucket's latest records, k in [cnt - n_lds, cnt), fold here
    if (cnt > cap) {   // a hot bucket: its records [0, cnt - cap) to k_fold_hot, with the run arrays
        __shared__ uint32_t s_j;
        if (threadIdx.x == 0) {
            s_j = atomicAdd(hn, 1u);
            if (s_j < hot_cap) {
                hb[2 * s_j] = b;
                hb[2 * s_j + 1] = cnt - cap;
            }
        }
        __syncthreads();
        if (s_j < hot_cap) {   // (else, beyond the room for hot buckets: all of it here)
            uint32_t *dst = hw + (uint64_t)s_j * 2 * (nwg + 1);
            for (uint32_t w = threadIdx.x; w <= nwg; w += FP_T) {
                dst[w] = wsc[w];
                if (w < nwg) dst[nwg + 1 + w] = wrb[w];
            }
            n_lds = cap;
        }
    }
    // record k of the bucket: the last run starting at or before k, by binary search
    auto locate = [&](uint32_t k) -> FPRec {
        uint32_t lo = 0, hi = nwg - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (wsc[mid] <= k) lo = mid;
            else hi = mid - 1;
        }
        return rec[wrb[lo] + (k - wsc[lo])];
    };
    // FP_U records per thread and step, their loads issued together (a hot key's bucket is long)
    for (uint32_t q0 = threadIdx.x; q0 < n_lds; q0 += FP_T * FP_U) {
      FPRec rr[FP_U];
#pragma unroll
      for (uint32_t u = 0; u < FP_U; ++u)
        if (q0 + u * FP_T < n_lds) rr[u] = locate(cnt - 1 - (q0 + u * FP_T));
#pragma unroll
      for (uint32_t u = 0; u < FP_U; ++u) {
        if (q0 + u * FP_T >= n_lds) break;
        const FPRec &r = rr[u];
        uint32_t h = ht_mix(r.tag) & G.mask & (G.s - 1);
        const unsigned long long mine = ((unsigned long long)r.tag << 32) | r.i;
        uint32_t restart = HT_EMPTY;   // set: on to the global rounds from this entry
        for (;;) {
            // probe: claim (fill, then publish) or stop at the tuple's tag.  The wave leaves this
            // loop only when all its lanes have, so a claimer of the same wave has published
            // before any lane of the wave waits below.
            bool match = false;
            unsigned long long v;
            for (;;) {
                v = __hip_atomic_load(&s_tr[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (v == FE_EMPTY) {
                    v = atomicCAS(&s_tr[h], FE_EMPTY, mine);
                    if (v == FE_EMPTY) {   // this tuple represents its key in entry h
                        s_klen[h] = r.klen;
                        s_key[h] = r.key;
                        __hip_atomic_store(&s_best[h], r.i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        break;
                    }
                }
                if ((uint32_t)(v >> 32) == r.tag) { match = true; break; }
                if (++h == G.s) { restart = (first + G.s) & G.mask; break; }   // on into the next range
            }
            if (!match) break;
            uint32_t best, spins = 0;
            while ((best = __hip_atomic_load(&s_best[h], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) == FP_UNPUB &&
                   ++spins < (1u << 20)) {
            }
            if (best == FP_UNPUB) {   // (a bound on the wait, never reached in practice: the global
                restart = first + h;   // rounds take the tuple from this entry)
                break;
            }
            const uint4 e = s_key[h];
            bool same = s_klen[h] == r.klen &&
                        ((e.x ^ r.key.x) | (e.y ^ r.key.y) | (e.z ^ r.key.z) | (e.w ^ r.key.w)) == 0u;
            if (same && r.klen > 16u) same = key_tail_eq(segs, tup, (uint32_t)v, r.i, r.klen);
            if (same) {
                if (best < r.i) atomicMax(&s_best[h], r.i);   // the fold's last writer: the largest index
                break;
            }
            if (++h == G.s) {   // another key with this tag: probe on
                restart = (first + G.s) & G.mask;
                break;
            }
        }
        if (restart != HT_EMPTY) {
            list_push(ovl, ovn, r.i);
            slot[r.i] = restart;
        } else if (slot_all) {
            slot[r.i] = first + h;
        }
      }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < G.s; j += FP_T) {
        const unsigned long long v = s_tr[j];
        uint4 a, q;
        if (v == FE_EMPTY) {
            a = make_uint4(~0u, ~0u, ~0u, ~0u);
            q = a;
        } else {
            a = make_uint4((uint32_t)v, (uint32_t)(v >> 32), ~s_best[j], s_klen[j]);
            q = s_key[j];
        }
        reinterpret_cast<uint4 *>(&ent[first + j])[0] = a;
        reinterpret_cast<uint4 *>(&ent[first + j])[1] = q;
    }
}

// the hot buckets' earlier records (k_fold_lds: buckets longer than their LDS cap), over the
// whole device, bucket after bucket: each record looks its key up in the table the ranges wrote,
// with plain loads (a hot entry stays in every L2); a key already there with a later tuple as its
// best needs nothing more.  Any other tuple goes to the global rounds from its home entry.
__global__ void k_fold_hot(const kvr_tuple *__restrict__ tup, const SegDesc *__restrict__ segs,
                           const uint32_t *__restrict__ fsz, const FPRec *__restrict__ rec, uint32_t nwg,
                           const FoldEnt *__restrict__ ent, const uint32_t *__restrict__ hb,
                           const uint32_t *__restrict__ hw, const uint32_t *__restrict__ hn, uint32_t *__restrict__ ovl,
                           uint32_t *__restrict__ ovn, uint32_t *__restrict__ slot, uint32_t slot_all,
                           uint32_t hot_cap) {
    const uint32_t nh = *hn < hot_cap ? *hn : hot_cap, mask = fsz[0];
    for (uint32_t j = 0; j < nh; ++j) {
        const uint32_t m = hb[2 * j + 1];
        const uint32_t *wsc = hw + (uint64_t)j * 2 * (nwg + 1), *wrb = wsc + nwg + 1;
        for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < m; k += gridDim.x * blockDim.x) {
            uint32_t lo = 0, hi = nwg - 1;   // the last run starting at or before k
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (wsc[mid] <= k) lo = mid;
                else hi = mid - 1;
            }
            const FPRec r = rec[wrb[lo] + (k - wsc[lo])];
            const uint32_t home = ht_mix(r.tag) & mask;
            uint32_t h = home;
            bool done = false;
            for (uint32_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
                const uint4 a = reinterpret_cast<const uint4 *>(&ent[h])[0];
                if (a.x == 0xFFFFFFFFu && a.y == 0xFFFFFFFFu) break;   // free: the key is not in the table
                if (a.y != r.tag || a.w != r.klen) continue;
                const uint4 q = reinterpret_cast<const uint4 *>(&ent[h])[1];
                bool same = ((r.key.x ^ q.x) | (r.key.y ^ q.y) | (r.key.z ^ q.z) | (r.key.w ^ q.w)) == 0u;
                if (same && r.klen > 16u) same = key_tail_eq(segs, tup, a.x, r.i, r.klen);
                if (same) {
                    done = ~a.z > r.i;   // a later tuple of the key is its best already
                    break;
                }
            }
            if (done) {
                if (slot_all) slot[r.i] = h;
            } else {
                list_push(ovl, ovn, r.i);
                slot[r.i] = home;
            }
        }
    }
}

__device__ __forceinline__ bool is_last(const FoldEnt *ent, const uint32_t *slot, uint64_t i) {
    const uint32_t s = slot[i];
    return s != HT_EMPTY && ~ent[s].best == (uint32_t)i;
}

// live flags and output sizes, from the table's side: one thread per entry; a claimed entry's
// last tuple is live iff it is a SET (flag and size must be zero beforehand).  Reads the table once (the
// claimed entries' last tuples at random) instead of every tuple and its entry.
// (keep_del: every key's last record, a DEL included — the per-GPU reduction of a sharded store,
// whose tombstones may delete a key another GPU SET)
// (grid-stride over the table size on the device)
// (flag8: one byte a tuple instead, for the dense list above; size and flag are then null)
__global__ void k_live_ent(const FoldEnt *__restrict__ ent, const uint32_t *__restrict__ fsz,
                           const kvr_tuple *__restrict__ tup, uint64_t *__restrict__ size,
                           uint32_t *__restrict__ flag, uint8_t *__restrict__ flag8, uint32_t keep_del) {
    const uint64_t n_slots = (uint64_t)fsz[0] + 1;
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n_slots; h += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 a = reinterpret_cast<const uint4 *>(&ent[h])[0];
        if (a.x == 0xFFFFFFFFu && a.y == 0xFFFFFFFFu) continue;   // free
        const uint32_t j = ~a.z;
        const kvr_tuple t = tup[j];
        if (t.op != 0 && !keep_del) continue;
        if (flag8) {
            flag8[j] = 1u;
            continue;
        }
        if (!flag) {   // packed (kvr_compact): size << 24 | 1, one scan gives offsets and positions
            size[j] = (9ull + t.key_len + t.val_len) << 24 | 1ull;
            continue;
        }
        flag[j] = 1u;
        if (size) size[j] = 9ull + t.key_len + t.val_len;   // SET framing, engine.rs:169-173
    }
}

// ---- the dense live list from byte flags (kvr_compact; round 4) ----------------------------------
// k_live_ent marks each live tuple with a byte (flag8; 0.5 M of cfg4's 8 M tuples), then: per block of
// DL_CH tuples its live count and bytes (k_dl_count, 16 flags a thread as one 16-B load, the tuple
// read only when live), one workgroup scans the blocks (k_dl_scan), and each block writes its live
// records' sources and output offsets (k_dl_fill).  No per-tuple size array, no scan over every
// tuple: the flags are nt bytes, against 8 B a tuple for the packed scan this replaces.
constexpr int DL_T = 256, DL_PER = 16, DL_CH = DL_T * DL_PER;   // tuples per block: 4096
__device__ __forceinline__ uint64_t rec_size(const kvr_tuple &t) { return 9ull + t.key_len + t.val_len; }   // engine.rs:169-173
#ifndef KVR_DL_BATCH   // 1: the dense-list kernels load their live tuples four at a time (A/B knob, round 5)
#define KVR_DL_BATCH 1
#endif
// the thread's 16 flags as a bit mask (bit k: tuple i0 + k is live)
__device__ __forceinline__ uint32_t dl_bits(const uint4 f) {
    const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
    uint32_t b = 0;
#pragma unroll
    for (int k = 0; k < DL_PER; ++k) b |= ((fw[k >> 2] >> (8 * (k & 3))) & 255u) ? 1u << k : 0u;
    return b;
}
// the next four live tuples of the mask (-1: none), taken off it
__device__ __forceinline__ void dl_next4(uint32_t &bits, int (&kk)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        kk[q] = bits ? __builtin_ctz(bits) : -1;
        bits &= bits ? bits - 1u : 0u;
    }
}
// (flags of the thread's 16 tuples: flag8 holds nt bytes rounded up to DL_CH, zero past nt)
__device__ __forceinline__ uint4 dl_flags(const uint8_t *flag8, uint64_t i0) {
    return *reinterpret_cast<const uint4 *>(flag8 + i0);
}
// the thread's live count and bytes over its 16 tuples (tup null: the count alone)
__device__ __forceinline__ void dl_sums(const uint4 f, const kvr_tuple *tup, uint64_t i0, uint32_t &c, uint64_t &by) {
#if KVR_DL_BATCH
    uint32_t bits = dl_bits(f);
    c = (uint32_t)__builtin_popcount(bits);
    by = 0;
    if (!tup) return;
    while (bits) {   // (the live tuples' lengths four at a time, their loads issued together)
        int kk[4];
        dl_next4(bits, kk);
        uint32_t kl[4], vl[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const kvr_tuple *t = tup + i0 + (uint64_t)(kk[q] >= 0 ? kk[q] : kk[0]);
            kl[q] = t->key_len;
            vl[q] = t->val_len;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) by += kk[q] >= 0 ? 9ull + kl[q] + vl[q] : 0ull;   // engine.rs:169-173
    }
    return;
#endif
    const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
    c = 0;
    by = 0;
#pragma unroll
    for (int k = 0; k < DL_PER; ++k) {
        if ((fw[k >> 2] >> (8 * (k & 3))) & 255u) {
            ++c;
            if (tup) by += rec_size(tup[i0 + k]);
        }
    }
}
// block-wide exclusive prefix of (count, bytes) over DL_T threads; returns the block's totals
__device__ __forceinline__ void dl_block_scan(uint32_t &c, uint64_t &by, uint32_t &tc, uint64_t &tby) {
    __shared__ uint32_t wc[DL_T / 64];
    __shared__ uint64_t wb[DL_T / 64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t xc = c;
    uint64_t xb = by;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t yc = __shfl_up(xc, d, 64);
        const uint64_t yb = __shfl_up(xb, d, 64);
        if (lane >= d) { xc += yc; xb += yb; }
    }
    if (lane == 63u) { wc[w] = xc; wb[w] = xb; }
    __syncthreads();
    uint32_t pc = 0;
    uint64_t pb = 0;
    tc = 0;
    tby = 0;
#pragma unroll
    for (uint32_t k = 0; k < DL_T / 64; ++k) {
        if (k < w) { pc += wc[k]; pb += wb[k]; }
        tc += wc[k];
        tby += wb[k];
    }
    c = pc + xc - c;
    by = pb + xb - by;
}
__global__ void __launch_bounds__(DL_T) k_dl_count(const uint8_t *__restrict__ flag8, const kvr_tuple *__restrict__ tup,
                                                   uint32_t *__restrict__ bcnt, uint64_t *__restrict__ bbytes) {
    const uint64_t i0 = (uint64_t)blockIdx.x * DL_CH + (uint64_t)threadIdx.x * DL_PER;
    uint32_t c;
    uint64_t by;
    dl_sums(dl_flags(flag8, i0), tup, i0, c, by);
    uint32_t tc;
    uint64_t tby;
    dl_block_scan(c, by, tc, tby);
    if (threadIdx.x == 0) { bcnt[blockIdx.x] = tc; bbytes[blockIdx.x] = tby; }
}
// one workgroup: the blocks' exclusive prefixes in place, 1024 blocks a pass; the totals to
// totals[0] (bytes), totals[1] (live records) and the dense offsets' end sentinel l_off[live]
constexpr int DL_ST = 1024;
__global__ void __launch_bounds__(DL_ST) k_dl_scan(uint32_t *__restrict__ bcnt, uint64_t *__restrict__ bbytes, uint32_t nb,
                                                   uint64_t *__restrict__ l_off, uint64_t *__restrict__ totals) {
    __shared__ uint32_t wc[DL_ST / 64];
    __shared__ uint64_t wb[DL_ST / 64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t carry_c = 0;
    uint64_t carry_b = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += DL_ST) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t c = b < nb ? bcnt[b] : 0u;
        const uint64_t by = b < nb ? bbytes[b] : 0ull;
        uint32_t xc = c;
        uint64_t xb = by;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t yc = __shfl_up(xc, d, 64);
            const uint64_t yb = __shfl_up(xb, d, 64);
            if (lane >= d) { xc += yc; xb += yb; }
        }
        if (lane == 63u) { wc[w] = xc; wb[w] = xb; }
        __syncthreads();
        uint32_t pc = carry_c, tc = 0;
        uint64_t pb = carry_b, tb = 0;
        for (uint32_t k = 0; k < DL_ST / 64; ++k) {
            if (k < w) { pc += wc[k]; pb += wb[k]; }
            tc += wc[k];
            tb += wb[k];
        }
        if (b < nb) { bcnt[b] = pc + xc - c; bbytes[b] = pb + xb - by; }
        carry_c += tc;
        carry_b += tb;
        __syncthreads();   // (wc / wb are rewritten by the next pass)
    }
    if (threadIdx.x == 0) {
        totals[0] = carry_b;
        totals[1] = carry_c;
        if (l_off) l_off[carry_c] = carry_b;
    }
}
__global__ void __launch_bounds__(DL_T) k_dl_fill(const uint8_t *__restrict__ flag8, const kvr_tuple *__restrict__ tup,
                                                  const SegDesc *__restrict__ segs, const uint32_t *__restrict__ bcnt,
                                                  const uint64_t *__restrict__ bbytes, uint64_t *__restrict__ l_src,
                                                  uint64_t *__restrict__ l_off) {
    const uint64_t i0 = (uint64_t)blockIdx.x * DL_CH + (uint64_t)threadIdx.x * DL_PER;
    const uint4 f = dl_flags(flag8, i0);
    uint32_t c;
    uint64_t by;
    dl_sums(f, tup, i0, c, by);
    uint32_t tc;
    uint64_t tby;
    dl_block_scan(c, by, tc, tby);
    if (tc == 0) return;
    uint64_t d = (uint64_t)bcnt[blockIdx.x] + c, o = bbytes[blockIdx.x] + by;
#if KVR_DL_BATCH
    uint32_t bits = dl_bits(f);
    while (bits) {   // (four live tuples at a time, their loads issued together ahead of the branches)
        int kk[4];
        dl_next4(bits, kk);
        kvr_tuple t[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = tup[i0 + (uint64_t)(kk[q] >= 0 ? kk[q] : kk[0])];
        asm volatile("" ::"v"(t[0].rec_off), "v"(t[0].seg_idx), "v"(t[0].key_len), "v"(t[0].val_len),
                     "v"(t[1].rec_off), "v"(t[1].seg_idx), "v"(t[1].key_len), "v"(t[1].val_len),
                     "v"(t[2].rec_off), "v"(t[2].seg_idx), "v"(t[2].key_len), "v"(t[2].val_len),
                     "v"(t[3].rec_off), "v"(t[3].seg_idx), "v"(t[3].key_len), "v"(t[3].val_len));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (kk[q] < 0) break;
            l_src[d] = reinterpret_cast<uint64_t>(segs[t[q].seg_idx].base + t[q].rec_off);
            l_off[d] = o;
            ++d;
            o += rec_size(t[q]);
        }
    }
    return;
#endif
    const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int k = 0; k < DL_PER; ++k) {
        if ((fw[k >> 2] >> (8 * (k & 3))) & 255u) {
            const kvr_tuple t = tup[i0 + k];
            l_src[d] = reinterpret_cast<uint64_t>(segs[t.seg_idx].base + t.rec_off);
            l_off[d] = o;
            ++d;
            o += rec_size(t);
        }
    }
}

// the same dense list for the index (fold_derive): the live tuples themselves, and each live
// tuple's place in the list (pos, read by k_index_from_fold at the live tuples only)
__global__ void __launch_bounds__(DL_T) k_dl_fill_tup(const uint8_t *__restrict__ flag8, const kvr_tuple *__restrict__ tup,
                                                      const uint32_t *__restrict__ bcnt, kvr_tuple *__restrict__ out,
                                                      uint32_t *__restrict__ pos) {
    const uint64_t i0 = (uint64_t)blockIdx.x * DL_CH + (uint64_t)threadIdx.x * DL_PER;
    const uint4 f = dl_flags(flag8, i0);
    uint32_t c;
    uint64_t by;
    dl_sums(f, nullptr, i0, c, by);
    uint32_t tc;
    uint64_t tby;
    dl_block_scan(c, by, tc, tby);
    if (tc == 0) return;
    uint32_t d = bcnt[blockIdx.x] + c;
#if KVR_DL_BATCH
    uint32_t bits = dl_bits(f);
    while (bits) {   // (four live tuples at a time, their loads issued together ahead of the branches)
        int kk[4];
        dl_next4(bits, kk);
        u32x4 t[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(tup + i0 + (uint64_t)(kk[q] >= 0 ? kk[q] : kk[0]));
            t[q][0] = src[0];
            t[q][1] = src[1];
        }
        asm volatile("" ::"v"(t[0][0]), "v"(t[0][1]), "v"(t[1][0]), "v"(t[1][1]), "v"(t[2][0]), "v"(t[2][1]),
                     "v"(t[3][0]), "v"(t[3][1]));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (kk[q] < 0) break;
            u32x4 *dst = reinterpret_cast<u32x4 *>(out + d);
            dst[0] = t[q][0];
            dst[1] = t[q][1];
            pos[i0 + kk[q]] = d;
            ++d;
        }
    }
    return;
#endif
    const uint32_t fw[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int k = 0; k < DL_PER; ++k) {
        if ((fw[k >> 2] >> (8 * (k & 3))) & 255u) {
            out[d] = tup[i0 + k];
            pos[i0 + k] = d;
            ++d;
        }
    }
}

// totals: live bytes, live records, and the end sentinel of the dense offsets
__global__ void k_ctotals(const uint64_t *__restrict__ size, const uint64_t *__restrict__ off,
                          const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos, uint64_t n,
                          uint64_t *__restrict__ l_off, uint64_t *__restrict__ totals) {
    if (threadIdx.x || blockIdx.x) return;
    const uint64_t bytes = n ? off[n - 1] + size[n - 1] : 0;
    const uint64_t live = n ? (uint64_t)pos[n - 1] + flag[n - 1] : 0;
    l_off[live] = bytes;
    totals[0] = bytes;
    totals[1] = live;
}

// dense live list
__global__ void k_scatter(const kvr_tuple *__restrict__ tup, uint64_t n, const SegDesc *__restrict__ segs,
                          const uint64_t *__restrict__ size, const uint64_t *__restrict__ off,
                          const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                          uint64_t *__restrict__ l_src, uint64_t *__restrict__ l_off) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const kvr_tuple t = tup[i];
    const uint32_t j = pos[i];
    l_src[j] = reinterpret_cast<uint64_t>(segs[t.seg_idx].base + t.rec_off);
    l_off[j] = off[i];
}

// one wave per live record (grid-stride over records): the record's source and
// output range come straight from the dense live list (two dependent loads instead of the block
// search's four); the output's 16-B aligned body moves as 16 B per lane (five source dwords
// funnel-shifted), the unaligned head and tail bytes one per lane.  A long record loops 4 KiB at
// a time with all its loads issued first.
__global__ void __launch_bounds__(CT_GATHER) k_gather_r(const uint64_t *__restrict__ l_src, const uint64_t *__restrict__ l_off,
                                                        const uint64_t *__restrict__ totals, uint8_t *__restrict__ out,
                                                        uint64_t cap) {
    const int lane = threadIdx.x & 63;
    const uint64_t total = totals[0];
    const uint64_t n_live = totals[1];
    const uint64_t lim = total < cap ? total : cap;
    const uint64_t waves = (uint64_t)gridDim.x * (CT_GATHER / 64);
    const uint64_t w0 = (uint64_t)blockIdx.x * (CT_GATHER / 64) + (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t j = w0; j < n_live; j += waves) {
        const uint64_t src = l_src[j], s0 = l_off[j];
        uint64_t s1 = l_off[j + 1];
        if (s0 >= lim) continue;
        s1 = s1 < lim ? s1 : lim;
        const uint8_t *sp = reinterpret_cast<const uint8_t *>(src);
        const uint64_t oa = reinterpret_cast<uint64_t>(out);
        // body [a0, a1): output offsets whose absolute address is 16-B aligned
        uint64_t a0 = ((oa + s0 + 15) & ~15ull) - oa, a1 = ((oa + s1) & ~15ull) - oa;
        if (a0 >= a1) { a0 = s1; a1 = s1; }   // no whole 16-B word: all bytes go one by one
        // head [s0, a0) and tail [a1, s1): fewer than 16 bytes each, or the whole record when it
        // has no body (then fewer than 32)
        {
            const uint64_t nh = a0 - s0, nt = s1 - a1;
            if ((uint64_t)lane < nh) out[s0 + lane] = sp[lane];
            if ((uint64_t)lane < nt) out[a1 + lane] = sp[a1 - s0 + lane];
        }
        for (uint64_t xb = a0; xb < a1; xb += 4 * 1024) {
            uint32_t d[4][5];
            uint32_t sh[4];
            bool on[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t x = xb + (uint64_t)u * 1024 + 16u * (uint32_t)lane;
                on[u] = x < a1;
                const uint64_t sa = src + (on[u] ? x - s0 : 0);
                const uint32_t *b = reinterpret_cast<const uint32_t *>(sa & ~3ull);
                sh[u] = (uint32_t)sa & 3u;
                if (on[u]) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) d[u][q] = b[q];
                    d[u][4] = sh[u] ? b[4] : 0u;   // b[4] holds byte sa + 15 when sh != 0
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (!on[u]) continue;
                const uint64_t x = xb + (uint64_t)u * 1024 + 16u * (uint32_t)lane;
                uint4 v;
                v.x = __builtin_amdgcn_alignbyte(d[u][1], d[u][0], sh[u]);
                v.y = __builtin_amdgcn_alignbyte(d[u][2], d[u][1], sh[u]);
                v.z = __builtin_amdgcn_alignbyte(d[u][3], d[u][2], sh[u]);
                v.w = __builtin_amdgcn_alignbyte(d[u][4], d[u][3], sh[u]);
                *reinterpret_cast<uint4 *>(out + x) = v;
            }
        }
    }
}

// cut k (k = 1 .. (total - 1) / target): the output offset of the first live record at or after
// k * target (grid-stride; the count comes from the device totals, cuts has room for it)
__global__ void k_cuts(const uint64_t *__restrict__ l_off, const uint64_t *__restrict__ totals, uint64_t target,
                       uint64_t *__restrict__ cuts) {
    const uint64_t total = totals[0];
    const uint64_t n_cuts = total > target ? (total - 1) / target : 0;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_cuts; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t want = (k + 1) * target;
        uint64_t lo = 0, hi = totals[1];   // lower_bound over l_off[0, n_live)
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (l_off[mid] < want) lo = mid + 1;
            else hi = mid;
        }
        cuts[k] = l_off[lo];   // l_off[n_live] = total
    }
}


// ---------------------------------------------------------------------------------------
// sharded compaction (kvr_compact_stage / _resolve / _finish): the global last-writer fold of a
// store whose segments are dealt over several GPUs.  A candidate is a key's LOCAL last record;
// it goes to owner rank hash(key) mod n_ranks, which keeps the candidate with the largest
// global position (global segment index, offset) per key and answers with one flag each.
// ---------------------------------------------------------------------------------------
constexpr uint32_t NO_OWNER = 0xFFFFFFFFu;
constexpr uint64_t CPOS_SHIFT = 40;   // global position = (global segment index << 40) | rec_off

__device__ __forceinline__ uint32_t owner_of(uint32_t key_tag, uint32_t n_ranks) {
    return (ht_mix(key_tag) >> 7) % n_ranks;   // other bits than the table slot's
}

__global__ void k_cand(const kvr_tuple *__restrict__ tup, uint64_t n, const FoldEnt *__restrict__ ent,
                       const uint32_t *__restrict__ slot, uint32_t n_ranks, uint32_t *__restrict__ cown) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    cown[i] = is_last(ent, slot, i) ? owner_of(tup[i].key_tag, n_ranks) : NO_OWNER;
}

// per owner o: (1 << 40) | padded key bytes for its candidates (one exclusive scan gives both
// the header index and the key offset inside the owner's group)
__global__ void k_cand_val(const kvr_tuple *__restrict__ tup, uint64_t n, const uint32_t *__restrict__ cown, uint32_t o,
                           uint64_t *__restrict__ val) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    val[i] = cown[i] == o ? ((1ull << CPOS_SHIFT) | ((tup[i].key_len + 3ull) & ~3ull)) : 0ull;
}

// gstart[o] / gstart[N + 1 + o]: first header / first key byte of owner o's group
__global__ void k_cand_total(const uint64_t *__restrict__ scan, const uint64_t *__restrict__ val, uint64_t n, uint32_t o,
                             uint32_t n_ranks, uint64_t *__restrict__ gstart) {
    if (threadIdx.x || blockIdx.x) return;
    const uint64_t t = n ? scan[n - 1] + val[n - 1] : 0;
    const uint64_t mask = (1ull << CPOS_SHIFT) - 1;
    gstart[o + 1] = gstart[o] + (t >> CPOS_SHIFT);
    gstart[n_ranks + 1 + o + 1] = gstart[n_ranks + 1 + o] + (t & mask);
}

__global__ void k_cand_place(const kvr_tuple *__restrict__ tup, uint64_t n, const SegDesc *__restrict__ segs,
                             const uint32_t *__restrict__ gidx, const uint32_t *__restrict__ cown, uint32_t o,
                             uint32_t n_ranks, const uint64_t *__restrict__ scan, const uint64_t *__restrict__ gstart,
                             kvr_cand *__restrict__ hdr, uint8_t *__restrict__ keys, uint32_t *__restrict__ send_idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || cown[i] != o) return;
    const kvr_tuple t = tup[i];
    const uint64_t mask = (1ull << CPOS_SHIFT) - 1;
    const uint64_t h = gstart[o] + (scan[i] >> CPOS_SHIFT), koff = scan[i] & mask;
    kvr_cand c;
    c.pos = ((uint64_t)gidx[t.seg_idx] << CPOS_SHIFT) | t.rec_off;
    c.key_len = t.key_len;
    c.key_tag = t.key_tag;
    c.key_off = (uint32_t)koff;
    c.pad = 0;
    hdr[h] = c;
    const uint8_t *k = key_ptr(segs, t);
    uint8_t *d = keys + gstart[n_ranks + 1 + o] + koff;
    for (uint32_t b = 0; b < t.key_len; ++b) d[b] = k[b];
    send_idx[i] = (uint32_t)h;
}

// owner side: the candidates received from every rank (headers and keys in sender order)
__device__ __forceinline__ const uint8_t *cand_key(const kvr_cand &c, uint64_t i, const uint8_t *keys,
                                                   const uint64_t *hstart, const uint64_t *kbase, uint32_t n_ranks) {
    uint32_t s = 0;
    while (s + 1 < n_ranks && i >= hstart[s + 1]) ++s;   // the sender (a few ranks: linear)
    return keys + kbase[s] + c.key_off;
}

__global__ void k_res_insert(const kvr_cand *__restrict__ hdr, uint64_t m, const uint8_t *__restrict__ keys,
                             const uint64_t *__restrict__ hstart, const uint64_t *__restrict__ kbase, uint32_t n_ranks,
                             uint32_t *__restrict__ rep, unsigned long long *__restrict__ best, uint32_t mask,
                             uint32_t *__restrict__ slot) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const kvr_cand c = hdr[i];
    const uint8_t *k = cand_key(c, i, keys, hstart, kbase, n_ranks);
    uint32_t h = ht_mix(c.key_tag) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
        uint32_t r = __hip_atomic_load(&rep[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (r == HT_EMPTY) {
            r = atomicCAS(&rep[h], HT_EMPTY, (uint32_t)i);
            if (r == HT_EMPTY) r = (uint32_t)i;
        }
        bool same = r == (uint32_t)i;
        if (!same) {
            const kvr_cand o = hdr[r];
            if (o.key_tag == c.key_tag && o.key_len == c.key_len)
                same = bytes_eq(cand_key(o, r, keys, hstart, kbase, n_ranks), k, c.key_len);
        }
        if (same) {
            atomicMax(&best[h], (unsigned long long)c.pos);
            slot[i] = h;
            return;
        }
    }
    slot[i] = HT_EMPTY;
}

__global__ void k_res_flag(const kvr_cand *__restrict__ hdr, uint64_t m, const unsigned long long *__restrict__ best,
                           const uint32_t *__restrict__ slot, uint8_t *__restrict__ win) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t s = slot[i];
    win[i] = (s != HT_EMPTY && best[s] == (unsigned long long)hdr[i].pos) ? 1 : 0;
}

// this rank's live records after the exchange: a SET that is its key's local last AND the
// key's global last (its candidate won at the owner)
__global__ void k_live_global(const kvr_tuple *__restrict__ tup, uint64_t n, const FoldEnt *__restrict__ ent,
                              const uint32_t *__restrict__ slot, const uint32_t *__restrict__ send_idx,
                              const uint8_t *__restrict__ win, uint64_t *__restrict__ size, uint32_t *__restrict__ flag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const kvr_tuple t = tup[i];
    const bool cand = is_last(ent, slot, i);
    const bool live = t.op == 0 && cand && win[send_idx[i]] != 0;
    size[i] = live ? 9ull + t.key_len + t.val_len : 0ull;
    flag[i] = live ? 1u : 0u;
}

}  // namespace kvr

#endif
