/*
 * kvr_replay8.hip — k_replay8 (V8), the hot path (gfx950): the same walk as k_replay (V7,
 * kvr_replay_kernel.hip) with the same outputs (StripeRes, TileRes, pool tuples), reorganised
 * around what bounds V7 on MI355X: the CU's single scalar unit (870 of V7's 1188 SALU per tile
 * go to the header hops) and a tile load that is never in flight while the wave computes.
 *
 * One WAVE replays one stripe of 8-KiB tiles (src/store/engine.rs:79-154 semantics: first error
 * in record order, last-writer-free tuples; CRC-32/ISO-HDLC = crc32fast::hash, storage.rs:27).
 * Per tile:
 *   top   the landing registers (this tile, loaded during the previous tile) are written to the
 *         wave's LDS slot, and the NEXT tile's loads are issued into them at once: they stay in
 *         flight for the whole tile.  Stores of the previous tile's bookkeeping are issued
 *         before that prefetch, so the next top's vmcnt(0) waits only for it.
 *   F     framing hops, exact from the tile entry.  Headers come from a 256-B window: one LDS
 *         read per lane (lane k: dword wb + 4k), fields taken with v_readlane.  A window serves
 *         every header inside it (many small records per LDS round trip).
 *   R     records, one lane per record: key CRC and UTF-8 check, short values, read from LDS
 *         (V7 re-read them from L2, 0.88 GB of extra HBM traffic per cfg2 launch).
 *   C     long values: each lane CRCs its 128-B unit (read back from LDS) as two chains with a
 *         snapshot where a value ends and a restart where one starts; a segmented Kogge-Stone
 *         scan over the wave (wave_shr:1 DPP, then ds_bpermute for d = 2..32; constant
 *         multipliers x^(8*128*d), six nibble tables)
 *         gives the register at every unit boundary; the lane holding a value's end finishes it.
 *
 * LDS (160 KiB, 12 waves): 64 KiB of tables + 12 x 8 KiB tile slots.
 *   Row b (256 B) of the table area: dwords [0,16) table 1 (a byte then a zero byte) x16
 *   replicas, [16,32) table 0 (one byte) x16 replicas, [32,64) a hole.  In one ds_read_b32 the
 *   lanes 0-15 of a 32-lane half look table 1 up while lanes 16-31 look table 0 up (the next read
 *   swaps them), so a half's 32 lookups hit 32 distinct banks; the address is one v_perm_b32.
 *   The holes hold the nibble tables of "multiply by a constant" (KT: x^(8*128*2^j), j<6; KQ:
 *   x^(8*4q), q<=32) and IX (0xFFFFFFFF * x^(8j)).
 *   A tile slot stores lane l's 16-B granule i at granule i ^ (l & 7) of its row (conflict-free
 *   ds_write_b128).
 */
#include "kvr_device.h"
#include <type_traits>

namespace kvr {
namespace v8 {

#ifndef KVR8_RT
#define KVR8_RT 768
#endif
constexpr int RT = KVR8_RT;               // 12 waves: 12 x 8-KiB slots + 64 KiB tables = 160 KiB
constexpr int WPB = RT / 64;
constexpr int UW = SC / 4;                // dwords of a lane's unit
constexpr int SC_LOG = 7;
constexpr uint32_t N32 = 0xFFFFFFFFu;
constexpr uint32_t POOL_CHUNK = 2048;
constexpr uint32_t TILE_RECS = TILE / 5 + 1;
static_assert(POOL_CHUNK >= TILE_RECS, "the rest of a tile's records fits in one fresh chunk");
constexpr int32_t FAR = 1 << 30;
constexpr int KEYW = 6;                   // key words of the record fast path (<= 24 B)
constexpr int VALW = SMALL / 4;
constexpr int NKT = 6;                    // scan multipliers x^(8*SC*2^j), j < NKT
constexpr int HIX = 4 * (NKT + NQ);       // first hole row of IX
static_assert(HIX + (NIX + 31) / 32 <= 256, "nibble tables and IX fit in the holes");

struct __align__(16) Smem {
    uint32_t T[256 * 64];                 // CRC rows + holes (64 KiB)
    uint32_t tiles[WPB][TILE / 4];        // one 8-KiB tile slot per wave
};
static_assert(sizeof(Smem) <= 163840, "LDS");

#ifndef KVR_ABLATE
#define KVR_ABLATE 0
#endif

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// a copy the compiler cannot prove wave-uniform: what is computed from it stays in VGPRs (VALU)
__device__ __forceinline__ int32_t vdiv(int32_t x) {
    int32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) | __builtin_amdgcn_readlane((uint32_t)v, l);
}
template <int CTRL, int ROWS = 0xF, bool BC = true>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, BC);
}

// ---------------------------------------------------------------------------------------
// CRC primitives on the paired slice-by-2 rows
// ---------------------------------------------------------------------------------------
constexpr uint32_t SEL_T1_B0 = 0x0C0C0401u;   // address byte 1 = x byte 0, byte 0 = L byte 1 (table 1)
constexpr uint32_t SEL_T0_B1 = 0x0C0C0500u;   // address byte 1 = x byte 1, byte 0 = L byte 0 (table 0)
constexpr uint32_t SEL_T0_B0 = 0x0C0C0400u;   // one byte: x byte 0 in table 0
struct Crc {
    const uint8_t *t;   // S.T
    uint32_t L;         // byte 0: 4 (16 + (lane & 15)) (table-0 replica), byte 1: 4 (lane & 15) (table-1 replica)
    uint32_t s1, s2;    // this lane's selectors for the two lookups of a 2-byte step
};
__device__ __forceinline__ uint32_t tget(const Crc &k, uint32_t x, uint32_t sel) {
    return *reinterpret_cast<const uint32_t *>(k.t + __builtin_amdgcn_perm(x, k.L, sel));
}
__device__ __forceinline__ uint32_t crc2(const Crc &k, uint32_t x) {
    uint32_t a = tget(k, x, k.s1), b = tget(k, x, k.s2);
    asm("" : "+v"(a), "+v"(b));
    return (x >> 16) ^ a ^ b;
}
__device__ __forceinline__ uint32_t crc4(uint32_t c, uint32_t w, const Crc &k) { return crc2(k, crc2(k, c ^ w)); }
__device__ __forceinline__ void crc2x2(const Crc &k, uint32_t &xa, uint32_t &xb) {
    uint32_t a0 = tget(k, xa, k.s1), a1 = tget(k, xa, k.s2);
    uint32_t b0 = tget(k, xb, k.s1), b1 = tget(k, xb, k.s2);
    asm("" : "+v"(a0), "+v"(a1), "+v"(b0), "+v"(b1));
    xa = (xa >> 16) ^ a0 ^ a1;
    xb = (xb >> 16) ^ b0 ^ b1;
}
__device__ __forceinline__ void crc4x2(uint32_t &ca, uint32_t wa, uint32_t &cb, uint32_t wb, const Crc &k) {
    uint32_t xa = ca ^ wa, xb = cb ^ wb;
    crc2x2(k, xa, xb);
    crc2x2(k, xa, xb);
    ca = xa;
    cb = xb;
}
__device__ __forceinline__ uint32_t crc1(uint32_t c, uint32_t b, const Crc &k) {
    const uint32_t x = c ^ b;
    return (x >> 8) ^ tget(k, x, SEL_T0_B0);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t xor8(uint32_t *t) {
    asm("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]));
    return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}
// nibble table c in the holes: entry (i, n) at dword (4c + (i >> 1)) * 64 + 32 + 16 (i & 1) + n
__device__ __forceinline__ const uint32_t *ntab(const uint32_t *T, int c) { return T + 4 * c * 64 + 32; }
// v times the constant of nibble table K
__device__ __forceinline__ uint32_t kmul(uint32_t v, const uint32_t *K) {
    uint32_t pl[2] = {v & 0x0F0F0F0Fu, (v >> 4) & 0x0F0F0F0Fu};
    asm("" : "+v"(pl[0]), "+v"(pl[1]));
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = K[(i >> 1) * 64 + (i & 1) * 16 + ((pl[i & 1] >> (8 * (i >> 1))) & 255u)];
    return xor8(t);
}
__device__ __forceinline__ uint32_t ixv(const uint32_t *T, int j) { return T[(HIX + (j >> 5)) * 64 + 32 + (j & 31)]; }

// ---------------------------------------------------------------------------------------
// the wave's tile slot: tile byte o -> LDS byte (granule i of unit l at granule i ^ (l & 7))
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t swz(uint32_t o) { return o ^ ((o >> 3) & 0x70u); }
__device__ __forceinline__ uint32_t lds32(const uint8_t *tl, uint32_t o) {   // o 4-aligned, o < TILE
    return *reinterpret_cast<const uint32_t *>(tl + swz(o));
}

// raw CRC register (from ~0) over the n <= 4 NW bytes at tile offset o, from the slot
// ((o & ~3) + 4 (NW + 1) <= TILE); *bad = the 0x80 bits of those bytes
template <int NW>
__device__ __forceinline__ uint32_t crc_span_lds(const uint8_t *tl, const Crc &K, int o, uint32_t n, uint32_t nw,
                                                 uint32_t *bad) {
    const int a = o & ~3;
    const uint32_t sh = (uint32_t)o & 3u;
    uint32_t r[NW + 1];
#pragma unroll
    for (int i = 0; i <= NW; ++i) r[i] = (uint32_t)i <= nw ? lds32(tl, (uint32_t)(a + 4 * i)) : 0u;
    uint32_t c = ~0u, tail = 0, bd = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if ((uint32_t)i < nw) {
            const uint32_t kw = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
            const uint32_t m = n > 4u * i ? n - 4u * i : 0u;
            const uint32_t msk = m >= 4u ? ~0u : ((1u << (8 * m)) - 1u);
            bd |= kw & msk & 0x80808080u;
            const uint32_t cn = crc4(c, kw, K);
            c = m >= 4u ? cn : c;
            tail = (m > 0u && m < 4u) ? kw : tail;
        }
    }
    for (uint32_t b = 0; b < (n & 3u); ++b) c = crc1(c, (tail >> (8 * b)) & 255u, K);
    *bad = bd;
    return c;
}

// the same over global memory (V7's TileSeg reads), for spans that leave the tile
template <int NW>
__device__ __forceinline__ uint32_t crc_span_g(const TileSeg &ts, const Crc &K, int o, uint32_t n, uint32_t nw,
                                               uint32_t *bad) {
    const int a = o & ~3;
    const uint32_t sh = (uint32_t)o & 3u;
    uint32_t r[NW + 1];
#pragma unroll
    for (int i = 0; i <= NW; ++i) r[i] = (uint32_t)i <= nw ? ts.w32a(a + 4 * i) : 0u;
    uint32_t c = ~0u, tail = 0, bd = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if ((uint32_t)i < nw) {
            const uint32_t kw = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
            const uint32_t m = n > 4u * i ? n - 4u * i : 0u;
            const uint32_t msk = m >= 4u ? ~0u : ((1u << (8 * m)) - 1u);
            bd |= kw & msk & 0x80808080u;
            const uint32_t cn = crc4(c, kw, K);
            c = m >= 4u ? cn : c;
            tail = (m > 0u && m < 4u) ? kw : tail;
        }
    }
    for (uint32_t b = 0; b < (n & 3u); ++b) c = crc1(c, (tail >> (8 * b)) & 255u, K);
    *bad = bd;
    return c;
}

// CRC register update over segment bytes [o, o + n) through global memory (general path)
__device__ inline uint32_t crc_long(const TileSeg &ts, uint32_t c, int64_t o, uint64_t n, const Crc &K) {
    const int64_t e = o + (int64_t)n;
    #pragma unroll 1
    while (o < e && ((o & 3) || o < 0 || o + 8 > ts.lim)) {
        c = crc1(c, ts.b8(o), K);
        ++o;
    }
    #pragma unroll 1
    while (o + 4 <= e && o + 8 <= ts.lim) { c = crc4(c, ts.w32a((int)o), K); o += 4; }
    #pragma unroll 1
    while (o < e) { c = crc1(c, ts.b8(o), K); ++o; }
    return c;
}

struct RecRes {
    uint32_t err, kind;
    uint64_t aux;
};

// the record at tile offset o with every engine.rs check, in engine.rs order (V7 do_record)
__device__ inline RecRes do_record(const TileSeg &ts, const Crc &K, int64_t o, uint32_t j, uint64_t slot, uint32_t seg,
                                   kvr_tuple *pool, uint64_t pool_cap) {
    RecRes ro;
    ro.err = N32; ro.kind = 0; ro.aux = 0;
    const int64_t rem = (int64_t)ts.len - ts.lo;
    const uint32_t op = ts.b8(o);
    if (rem - o < 5) { ro.err = j; ro.kind = KVR_E_KEY_LEN; return ro; }                  // engine.rs:96
    const uint64_t klen = ts.u32(o + 1);
    const int64_t kb = o + 5;
    if ((uint64_t)(rem - kb) < klen) { ro.err = j; ro.kind = KVR_E_KEY; return ro; }      // engine.rs:107
    uint64_t vu = 0;
    uint32_t el = 0;
    if (!utf8_check(ts, kb, klen, &vu, &el)) {                                          // engine.rs:114
        ro.err = j; ro.kind = KVR_E_UTF8; ro.aux = vu | ((uint64_t)el << 32); return ro;
    }
    if (op > 1u) { ro.err = j; ro.kind = KVR_E_OPCODE; ro.aux = op; return ro; }          // engine.rs:143
    kvr_tuple t;
    t.rec_off = (uint64_t)(ts.lo + o);
    t.seg_idx = seg;
    t.key_len = (uint32_t)klen;
    t.key_tag = ~crc_long(ts, ~0u, kb, klen, K);
    t.op = (uint8_t)op;
    t.flags = 0;
    t.reserved = 0;
    t.crc32 = 0;
    t.val_len = 0;
    if (op == 0u) {
        const int64_t q = kb + (int64_t)klen;
        if (rem - q < 4) { ro.err = j; ro.kind = KVR_E_VAL_LEN; return ro; }              // engine.rs:121
        const uint64_t vlen = ts.u32(q);
        if ((uint64_t)(rem - q - 4) < vlen) { ro.err = j; ro.kind = KVR_E_VAL; return ro; }   // engine.rs:130
        t.val_len = (uint32_t)vlen;
        if (vlen <= (uint64_t)SMALL) t.crc32 = ~crc_long(ts, ~0u, q + 4, vlen, K);
    }
    if (slot < pool_cap) pool[slot] = t;
    return ro;
}

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(RT) void k_replay8(const SegDesc *__restrict__ segs,
                                                const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                                StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                                kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                                Tables tb, const RedoEnt *__restrict__ redo,
                                                const LinkResult *__restrict__ link, int redo_mode,
                                                uint32_t pool_chunk) {
    __shared__ Smem S;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 256 * 32; i += RT) {
        const int b = i >> 5, d = i & 31;
        S.T[b * 64 + d] = tb.crc8[(d < 16 ? 256 : 0) + b];
    }
    for (int i = tid; i < (NKT + NQ) * 128; i += RT) {
        const int c = i >> 7, ii = (i >> 4) & 7, n = i & 15;
        const int set = c < NKT ? c : KSET_Q + (c - NKT);
        S.T[(4 * c + (ii >> 1)) * 64 + 32 + 16 * (ii & 1) + n] = tb.kmul[(set * 8 + ii) * 16 + n];
    }
    for (int j = tid; j < NIX; j += RT) S.T[(HIX + (j >> 5)) * 64 + 32 + (j & 31)] = tb.initx[j];
    __syncthreads();   // the only workgroup barrier

    const uint32_t r16 = (uint32_t)(lane & 15);
    const bool h16 = (lane & 16) != 0;
    const Crc K{reinterpret_cast<const uint8_t *>(S.T), (4u * (16u + r16)) | ((4u * r16) << 8),
                h16 ? SEL_T0_B1 : SEL_T1_B0, h16 ? SEL_T1_B0 : SEL_T0_B1};
    const uint32_t *T = S.T;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint8_t *const tl = reinterpret_cast<uint8_t *>(S.tiles[wv]);
    const uint32_t gw = blockIdx.x * WPB + (uint32_t)wv;
    uint32_t si;
    uint64_t forced = NONE;
    if (redo_mode) {
        if (gw >= link->n_redo || link->status != 3) return;
        si = redo[gw].stripe;
        forced = redo[gw].entry;
    } else {
        if (gw >= n_stripes) return;
        si = gw;
    }
    const StripeDesc sd = stripes[si];
    const SegDesc sg = segs[sd.seg];
    const uint64_t len = sg.len;
    const int64_t d0 = sg.d0;
    const int64_t shi_i = (int64_t)sd.t_end * TILE - d0;
    const uint64_t s_hi = (uint64_t)shi_i > len ? len : (uint64_t)shi_i;
    const uint8_t *abase = sg.base - d0;

    uint64_t entry = redo_mode ? forced : ((sd.t_begin == 0) ? 0ull : NONE);
    bool search = entry == NONE;
    uint64_t stripe_entry = (entry != NONE && entry >= s_hi) ? NONE : entry;
    int stop = (entry != NONE && entry >= s_hi) ? 2 : 0;
    if (entry != NONE && (int64_t)entry < (int64_t)sd.t_begin * TILE - d0) {   // bug trap: k_link never does this
        stop = 2;
        stripe_entry = NONE;
        if (lane == 0) atomicOr(&ctr->overflow, 4u);
    }
    uint64_t err_pos = NONE, err_aux = 0;
    uint32_t err_kind = 0, total = 0;
    uint64_t chunk_base = 0, chunk_left = 0;
    uint32_t carry = 0, c_state = 0;
    uint64_t c_vb = 0, c_ve = 0, c_slot = 0;
    // deferred stores of the previous tile (issued before the next prefetch): its TileRes and
    // the crc32 of the long value ending in this lane's unit
    bool p_tres = false;
    TileRes p_tr{};
    uint32_t p_tile = 0;
    uint64_t p_ms = NONE;
    uint32_t p_crc = 0;

    uint32_t w[UW];        // landing registers: the next tile, in flight while this one is processed
    bool loaded = false;
    uint32_t k = sd.t_begin;
    if (!stop && k < sd.t_end && k < sg.n_tiles) {
        load_unit(abase, d0, len, k, lane, w);
        loaded = true;
    }
    for (;; ++k) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // the previous tile's deferred stores
        if (p_tres && lane == 0) tres[sg.tile0 + p_tile] = p_tr;
        if (p_ms != NONE && p_ms < pool_cap) pool[p_ms].crc32 = p_crc;
        p_tres = false;
        p_ms = NONE;
        const bool in_stripe = k < sd.t_end;
        if (stop || (!in_stripe && !carry) || k >= sg.n_tiles) break;
        if (!loaded) {
            load_unit(abase, d0, len, k, lane, w);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // the tile into the wave's slot, then the next tile's loads into the landing registers
#pragma unroll
        for (int i = 0; i < UW / 4; ++i) {
            const u32x4 v = {w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
            *reinterpret_cast<u32x4 *>(tl + 128 * lane + 16 * (i ^ (lane & 7))) = v;
        }
        loaded = false;
        if (k + 1 < sd.t_end && k + 1 < sg.n_tiles) {
            load_unit(abase, d0, len, k + 1, lane, w);
            loaded = true;
        }
        if (KVR_ABLATE & 64) {
            uint32_t x = lds32(tl, 4u * (uint32_t)lane);
            if (x == 0x9E3779B9u && lane == 0) atomicOr(&ctr->overflow, 8u);
            carry = 0;
            continue;
        }

        const int64_t lo = (int64_t)k * TILE - d0;      // segment position of tile byte 0
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        const int64_t rem = (int64_t)len - lo;
        const int64_t vlo_r = (int64_t)vlo - lo, vhi_r = (int64_t)vhi - lo;
        const TileSeg ts = tile_seg(abase, sg.base, d0, len, k);
        const int us = lane * SC, ue = us + SC;

        // ---- stripe entry: the first plausible record start (V7's SWAR filter + plausible()) --
        if (in_stripe && search) {
            uint32_t u[UW];
#pragma unroll
            for (int i = 0; i < UW / 4; ++i) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(tl + 128 * lane + 16 * (i ^ (lane & 7)));
                u[4 * i] = v.x; u[4 * i + 1] = v.y; u[4 * i + 2] = v.z; u[4 * i + 3] = v.w;
            }
            const int o0 = us > (int)vlo_r ? us : (int)vlo_r, o1 = ue < (int)vhi_r ? ue : (int)vhi_r;
            const int32_t rc = rem > 0x7FFFFFFFll ? 0x7FFFFFFF : (int32_t)rem;
            const uint32_t addT = (0x7Fu - ((uint32_t)rc >> 24)) * 0x01010101u;
            uint32_t cm[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < UW; ++i) {
                const uint32_t y = u[i] & 0xFEFEFEFEu;
                uint32_t z = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
                if (i + 1 < UW) {
                    const uint32_t x = u[i + 1];
                    z &= ~((((x & 0x7F7F7F7Fu) + addT) | x));
                }
                cm[i >> 3] |= z >> (7 - (i & 7));
            }
            int cand = -1;
            uint32_t m0 = cm[0], m1 = cm[1], m2 = cm[2], m3 = cm[3];
#pragma unroll 1
            for (;;) {
                const uint64_t fnd = __ballot(cand >= 0);
                if (fnd != 0ull && lane > (int)__builtin_ctzll(fnd)) { m0 = m1 = m2 = m3 = 0u; }
                if (__ballot((m0 | m1 | m2 | m3) != 0u) == 0ull) break;
                if ((m0 | m1 | m2 | m3) != 0u) {
                    const int q = m0 ? 0 : m1 ? 1 : m2 ? 2 : 3;
                    const uint32_t mb = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
                    const uint32_t nb = mb & (mb - 1u);
                    m0 = q == 0 ? nb : m0; m1 = q == 1 ? nb : m1; m2 = q == 2 ? nb : m2; m3 = q == 3 ? nb : m3;
                    const int t = __builtin_ctz(mb);
                    const int o = us + 32 * q + 4 * (t & 7) + (t >> 3);
                    if (o >= o0 && o < o1 && (cand < 0 || o < cand) && plausible(ts, o)) cand = o;
                }
            }
            const uint64_t fnd = __ballot(cand >= 0);
            const uint64_t mn = fnd == 0ull ? NONE : (uint64_t)(lo + (int64_t)rl32((uint32_t)cand, (int)__builtin_ctzll(fnd)));
            if (mn != NONE) { entry = mn; search = false; stripe_entry = mn; }
        }
        const bool walk = in_stripe && !search && entry < vhi;
        uint64_t tile_exit = entry;
        bool vx = false;
        int32_t a_off = -1;
        bool vx_carry = false;
        int32_t m = 0;
        uint64_t m_ref = 0;
        bool m_abs = false;
        bool any_long = false;
        bool out = false;
        uint64_t out_ve = 0, out_ref = 0;
        bool out_abs = false;
        auto consider = [&](int32_t vb, uint64_t ve_abs, uint64_t ref, bool is_abs, bool from_carry) {
            const int64_t v64 = (int64_t)ve_abs - lo;
            const int32_t ver = v64 > FAR ? FAR : (int32_t)v64;
            if (vb < ue && ver > ue) { vx = true; a_off = vb >= us ? vb - us : -1; vx_carry = from_carry; }
            if (vb < us && ver > us && ver <= ue) { m = ver - us; m_ref = ref; m_abs = is_abs; }
            if (ver > TILE) { out = true; out_ve = ve_abs; out_ref = ref; out_abs = is_abs; }
            any_long = true;
        };
        uint32_t n_carry = 0;
        uint64_t n_vb = 0, n_ve = 0, n_ref = 0;
        bool n_abs = true;
        if (carry == 1u) consider(-FAR, c_ve, c_slot, true, true);
        if (carry == 2u) {
            if ((int64_t)c_vb - lo < TILE) consider((int32_t)((int64_t)c_vb - lo), c_ve, c_slot, true, false);
            else { n_carry = 2; n_vb = c_vb; n_ve = c_ve; n_ref = c_slot; }
        }
        uint64_t b1 = 0, b2 = 0;
        uint32_t c1 = N32;
        uint32_t nrec = 0, err_rec = N32;
        if (walk) {
            const bool huge = rem > 0x7FFFFFFFll;
            int64_t p = (int64_t)entry - lo;
            bool broke = false;
            // the header window: lane k holds the dword at tile offset wb + 4k (wb uniform)
            int32_t wb = -(1 << 20);
            uint32_t win = 0;
            auto wload = [&](int32_t o) {
                wb = o & ~3;
                const int32_t a = wb + 4 * lane;
                win = lds32(tl, (uint32_t)(a < TILE ? a : TILE - 4));
            };
            auto wu64 = [&](int32_t o) -> uint64_t {   // the 8 bytes from tile offset o, wb <= o <= wb + 240
                const int32_t d = o - wb;
                const int l = d >> 2;
                const uint32_t lo32 = rl32(win, l), hi32 = rl32(win, l + 1);
                return ((((uint64_t)hi32) << 32) | lo32) >> (8u * (uint32_t)(d & 3));
            };
            if (KVR_ABLATE & 4) p = vhi_r;
#pragma unroll 1
            while (p < vhi_r && !broke && err_rec == N32) {
                uint32_t nb = 0, kmx = 0;
                int32_t myrec = -1;
                uint32_t my_op = 0, my_klen = 0, my_vlen = 0;
                // Fast hops (segments < 2 GiB past the tile): the hop state lives in VGPRs (the
                // same value in every lane, hidden from uniformity analysis by vdiv) so the walk
                // issues on the SIMD's VALU instead of the CU's single scalar unit, and the body
                // is branch free: header and vlen straight from the slot, every engine.rs bound
                // as a compare.  The first record that is not simple (header or vlen leaving the
                // tile, a bound or opcode violation) ends the fast run; the exact scalar hop below
                // takes it, errors included.
                auto fast32 = [&](int32_t q0) -> int32_t {
                    // loop-carried state as 32-bit integers: a bool carried through a divergent
                    // loop becomes an SGPR lane mask merged with exec on every iteration (SALU)
                    int32_t q = vdiv(q0);
                    uint32_t n = (uint32_t)vdiv((int32_t)nb), kx = (uint32_t)vdiv((int32_t)kmx);
                    uint32_t fany = 0, fo_e2 = 0, fo_ref = N32;      // fo_ref != N32: a value runs past the tile
                    int32_t la = -2;                                 // >= -1: a fast record set (vx, a_off)
                    int32_t lm = 0;                                  // != 0: a fast record set (m, m_ref)
                    uint32_t lmr = 0;
                    const uint32_t rem32 = (uint32_t)rem, vhi32 = (uint32_t)vhi_r;
#pragma unroll 1
                    for (;;) {
                        const uint32_t uq = (uint32_t)q;
                        if (!(uq < vhi32 && n < 64u && uq + 8u <= (uint32_t)TILE)) break;
                        const uint32_t a = uq & ~3u;
                        const uint32_t x0 = lds32(tl, a), x1 = lds32(tl, a + 4u);
                        const uint32_t op = __builtin_amdgcn_alignbyte(x1, x0, uq & 3u) & 255u;
                        const uint32_t klen = (uint32_t)((((uint64_t)x1 << 32) | x0) >> (8u * ((uq & 3u) + 1u)));
                        const uint32_t rq = rem32 - uq;
                        const uint32_t e = uq + 5u + klen;               // (meaningful when ok1)
                        const uint32_t set = op == 0u ? 1u : 0u;
                        const uint32_t vin = (e + 8u <= (uint32_t)TILE && e >= uq) ? 1u : 0u;
                        const uint32_t ea = (vin ? e : 0u) & ~3u;
                        const uint32_t y0 = lds32(tl, ea), y1 = lds32(tl, ea + 4u);
                        const uint32_t vlen = __builtin_amdgcn_alignbyte(y1, y0, e & 3u);
                        const uint32_t re = rem32 - e;
                        const uint32_t ok1 = (op <= 1u && rq >= 5u && klen <= rq - 5u) ? 1u : 0u;
                        const uint32_t ok2 = (vin && re >= 4u && vlen <= re - 4u) ? 1u : 0u;
                        if ((ok1 & (ok2 | (set ^ 1u))) == 0u) break;
                        const uint32_t vb = e + 4u, e2 = vb + vlen;
                        const bool me = lane == (int)n;
                        myrec = me ? q : myrec;
                        my_op = me ? op : my_op;
                        my_klen = me ? klen : my_klen;
                        my_vlen = me ? vlen : my_vlen;
                        kx = klen > kx ? klen : kx;
                        // a value longer than SMALL that crosses a unit boundary (consider(), with
                        // vb inside the tile)
                        const uint32_t lv = set & (vlen > (uint32_t)SMALL ? 1u : 0u) & ((vb >> SC_LOG) != ((e2 - 1u) >> SC_LOG) ? 1u : 0u);
                        const uint32_t idx = nrec + n;
                        const int32_t vbi = (int32_t)vb, e2i = (int32_t)e2;
                        la = (lv && vbi < ue && e2i > ue) ? (vbi >= us ? vbi - us : -1) : la;
                        const bool mm = lv && vbi < us && e2i > us && e2i <= ue;
                        lm = mm ? e2i - us : lm;
                        lmr = mm ? idx : lmr;
                        fany |= lv;
                        const bool o = lv && e2 > (uint32_t)TILE;
                        fo_e2 = o ? e2 : fo_e2;
                        fo_ref = o ? idx : fo_ref;
                        ++n;
                        q = (int32_t)(set ? e2 : e);
                    }
                    if (la >= -1) { vx = true; a_off = la; vx_carry = false; }
                    if (lm != 0) { m = lm; m_ref = lmr; m_abs = false; }
                    nb = uni32(n);
                    kmx = uni32(kx);
                    if (uni32(fany)) any_long = true;
                    const uint32_t fr = uni32(fo_ref);
                    if (fr != N32) {
                        out = true; out_ve = (uint64_t)(lo + (int64_t)uni32(fo_e2)); out_ref = fr; out_abs = false;
                    }
                    return (int32_t)uni32((uint32_t)q);
                };
                auto hops = [&](auto q) -> decltype(q) {
                    using Ty = decltype(q);
                    using U = std::make_unsigned_t<Ty>;
                    const Ty remT = (Ty)rem, vhiT = (Ty)vhi_r;
#pragma unroll 1
                    while (q < vhiT && nb < 64u) {
                        if constexpr (std::is_same_v<Ty, int32_t>) {
                            if (!(KVR_ABLATE & 32)) {
                                q = fast32(q);
                                if (!(q < vhiT && nb < 64u)) break;
                            }
                        }
                        uint32_t op, klen;
                        if (q + 8 <= TILE) {
                            const int32_t qi = (int32_t)q;
                            if (qi < wb || qi > wb + 240) wload(qi);
                            const uint64_t x = wu64(qi);
                            op = (uint32_t)x & 255u;
                            klen = (uint32_t)(x >> 8);
                        } else {
                            op = uni32(ts.b8(q));
                            klen = remT - q >= 5 ? uni32(ts.u32(q + 1)) : 0u;
                        }
                        const bool me = lane == (int)nb;
                        myrec = me ? (int32_t)q : myrec;
                        my_op = me ? op : my_op;
                        my_klen = me ? klen : my_klen;
                        ++nb;
                        if (op > 1u || remT - q < 5 || (U)klen > (U)(remT - q - 5)) { broke = true; break; }
                        kmx = klen > kmx ? klen : kmx;
                        const Ty e = q + 5 + (Ty)klen;
                        if (op == 1u) { q = e; continue; }
                        if (remT - e < 4) { broke = true; break; }
                        uint32_t vlen;
                        if (e + 8 <= TILE) {
                            const int32_t ei = (int32_t)e;
                            if (ei > wb + 240) wload(ei);
                            vlen = (uint32_t)wu64(ei);
                        } else {
                            vlen = uni32(ts.u32(e));
                        }
                        my_vlen = lane == (int)nb - 1 ? vlen : my_vlen;
                        const Ty vb = e + 4;
                        if ((U)vlen > (U)(remT - vb)) { broke = true; break; }
                        const Ty e2 = vb + (Ty)vlen;
                        if (vlen > (uint32_t)SMALL && (vb >> SC_LOG) != ((e2 - 1) >> SC_LOG)) {
                            const uint64_t idx = nrec + nb - 1;
                            if (KVR_ABLATE & 32) any_long = true;
                            else if (vb < TILE) consider((int32_t)vb, (uint64_t)(lo + e2), idx, false, false);
                            else { n_carry = 2; n_vb = (uint64_t)(lo + vb); n_ve = (uint64_t)(lo + e2); n_ref = idx; n_abs = false; }
                        }
                        q = e2;
                    }
                    return q;
                };
                if (huge) p = hops((int64_t)p);
                else p = hops((int32_t)p);
                if (nb > chunk_left) {
                    const uint64_t cm = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
                    unsigned long long bb = 0;
                    if (lane == 0) {
                        bb = atomicAdd(&ctr->pool_cursor, (unsigned long long)cm);
                        if (bb + cm > pool_cap) atomicOr(&ctr->overflow, 1u);
                    }
                    chunk_base = uni64(bb);
                    chunk_left = cm;
                    if (nrec) { b2 = chunk_base; c1 = nrec; }
                }
                if (nrec == 0) b1 = chunk_base;
                const uint64_t slot = chunk_base + (uint64_t)lane;
                chunk_base += nb;
                chunk_left -= nb;
                uint32_t rerr = N32, rkind = 0;
                uint64_t raux = 0;
                const uint32_t j = nrec + (uint32_t)lane;
                if (!(KVR_ABLATE & 1) && myrec >= 0) {
                    if (broke && lane == (int)nb - 1) {
                        const RecRes r = do_record(ts, K, myrec, j, slot, sd.seg, pool, pool_cap);
                        rerr = r.err; rkind = r.kind; raux = r.aux;
                        if (r.err == N32) { rerr = j; rkind = KVR_E_VAL; }
                    } else {
                        const uint32_t kc = kmx > 4u * KEYW ? 4u * KEYW : kmx;
                        const uint32_t nw = (kc + 3u) >> 2;
                        const int kb = myrec + 5;
                        const uint32_t klen = my_klen;
                        uint32_t c = ~0u, bad = 0x80u;
                        if (klen <= 4u * KEYW) {
                            if ((kb & ~3) + 4 * (KEYW + 1) <= TILE) c = crc_span_lds<KEYW>(tl, K, kb, klen, nw, &bad);
                            else if (kb + 4 * KEYW + 8 <= ts.lim) c = crc_span_g<KEYW>(ts, K, kb, klen, nw, &bad);
                        }
                        if (bad != 0u) {
                            uint64_t vu = 0;
                            uint32_t el = 0;
                            if (!utf8_check(ts, kb, klen, &vu, &el)) {   // engine.rs:114
                                rerr = j; rkind = KVR_E_UTF8; raux = vu | ((uint64_t)el << 32);
                            } else {
                                c = crc_long(ts, ~0u, kb, klen, K);
                            }
                        }
                        if (rerr == N32) {
                            kvr_tuple t;
                            t.rec_off = (uint64_t)(lo + myrec);
                            t.seg_idx = sd.seg;
                            t.key_len = klen;
                            t.val_len = 0;
                            t.crc32 = 0;
                            t.key_tag = ~c;
                            t.op = (uint8_t)my_op;
                            t.flags = 0;
                            t.reserved = 0;
                            if (my_op == 0u) {
                                t.val_len = my_vlen;
                                const int vb = kb + (int)klen + 4;
                                uint32_t vbad;
                                if (my_vlen <= (uint32_t)SMALL) {
                                    if ((vb & ~3) + 4 * (VALW + 1) <= TILE)
                                        t.crc32 = ~crc_span_lds<VALW>(tl, K, vb, my_vlen, (uint32_t)VALW, &vbad);
                                    else if (vb + 4 * VALW + 8 <= ts.lim)
                                        t.crc32 = ~crc_span_g<VALW>(ts, K, vb, my_vlen, (uint32_t)VALW, &vbad);
                                    else t.crc32 = ~crc_long(ts, ~0u, vb, my_vlen, K);
                                } else if ((vb >> SC_LOG) == ((vb + (int)my_vlen - 1) >> SC_LOG)) {   // inside one unit
                                    if ((vb & ~3) + 4 * (UW + 1) <= TILE)
                                        t.crc32 = ~crc_span_lds<UW>(tl, K, vb, my_vlen, (uint32_t)UW, &vbad);
                                    else t.crc32 = ~crc_long(ts, ~0u, vb, my_vlen, K);
                                }
                            }
                            if (slot < pool_cap) pool[slot] = t;
                        }
                    }
                }
                if (__ballot(rerr != N32)) {
                    uint32_t er = rerr;
#pragma unroll
                    for (int dd = 32; dd >= 1; dd >>= 1) {
                        const uint32_t o = __shfl_xor(er, dd, 64);
                        er = o < er ? o : er;
                    }
                    err_rec = uni32(er);
                    const int el = (int)(err_rec - nrec);
                    err_kind = rl32(rkind, el);
                    err_aux = rl64(raux, el);
                    err_pos = (uint64_t)(lo + (int64_t)(int32_t)rl32((uint32_t)myrec, el));
                }
                nrec = err_rec != N32 ? err_rec : nrec + nb;
            }
            tile_exit = broke ? ERRP : (uint64_t)(lo + p);
        }
        if (c1 == N32) c1 = nrec;
        auto slot_of = [&](uint64_t ref, bool is_abs) -> uint64_t {
            return is_abs ? ref : (ref < c1 ? b1 + ref : b2 + (ref - c1));
        };
        if (n_carry == 2u && !n_abs) n_ref = slot_of(n_ref, false);

        // ---- C. CRC of long values ------------------------------------------------------------
        if (!(KVR_ABLATE & 2) && any_long) {
            constexpr int H = UW / 2;
            uint32_t u[UW];
#pragma unroll
            for (int i = 0; i < UW / 4; ++i) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(tl + 128 * lane + 16 * (i ^ (lane & 7)));
                u[4 * i] = v.x; u[4 * i + 1] = v.y; u[4 * i + 2] = v.z; u[4 * i + 3] = v.w;
            }
            const int qm = m >> 2;
            const int qa = (vx && a_off >= 0) ? (a_off >> 2) : -1;
            const uint32_t amask = ~0u << (8 * (a_off & 3));
            const int qh = qm & (H - 1), qah = qa >= 0 ? (qa & (H - 1)) : -1;
            const bool mb = qm >= H, ab = qa >= H;
            uint32_t ca = 0, cb = 0, sn = 0, wm = 0;
            if (KVR_ABLATE & 8) {
                ca = u[0]; cb = u[1];
            } else if (!__ballot(m != 0 || qa >= 0)) {
#pragma unroll
                for (int kk = 0; kk < H; ++kk) crc4x2(ca, u[kk], cb, u[kk + H], K);
            } else {
#pragma unroll
                for (int kk = 0; kk < H; ++kk) {
                    const bool s_ = kk == qh;
                    sn = s_ ? (mb ? cb : ca) : sn;
                    wm = s_ ? (mb ? u[kk + H] : u[kk]) : wm;
                    const bool r = kk == qah, ra = r && !ab, rb = r && ab;
                    ca = ra ? 0u : ca;
                    cb = rb ? 0u : cb;
                    crc4x2(ca, ra ? (u[kk] & amask) : u[kk], cb, rb ? (u[kk + H] & amask) : u[kk + H], K);
                }
                sn = qm == UW ? cb : sn;
            }
            const uint32_t pa = kmul(ca, ntab(T, NKT + H));
            const uint32_t ps = kmul(ca, ntab(T, NKT + (qm > H ? qm - H : 0)));
            const uint32_t c = qa >= H ? cb : (pa ^ cb);
            const uint32_t snap = qm < H ? sn : (ps ^ sn);
            uint32_t v = 0, f = 1;
            if (vx) {
                if (a_off >= 0) v = c ^ ixv(T, SC - a_off);
                else if (lane == 0 && vx_carry) v = c ^ kmul(c_state, ntab(T, 0));
                else { v = c; f = 0; }
            }
            // segmented Kogge-Stone scan over the whole wave: state at the end of unit l =
            // f ? v : state(l-1) * x^(8*SC) ^ v.  Step d joins lane l's span [l-d+1, l] to the
            // span [l-2d+1, l-d] of lane l-d, so the multiplier is the constant x^(8*SC*d); the
            // shifts cross rows (wave_shr:1 DPP for d = 1, ds_bpermute above), a row-limited
            // row_shr would join non-adjacent spans
            if (!(KVR_ABLATE & 16)) {
                {
                    const uint32_t ov = dpp<0x138>(v), of = dpp<0x138>(f);
                    const uint32_t t_ = kmul(ov, ntab(T, 0));
                    const bool ok = lane >= 1 && !f;
                    v = ok ? (v ^ t_) : v;
                    f = ok ? of : f;
                }
#pragma unroll
                for (int j = 1; j < NKT; ++j) {
                    const int d = 1 << j;
                    const uint32_t ov = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane - d), (int)v);
                    const uint32_t of = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (lane - d), (int)f);
                    const uint32_t t_ = kmul(ov, ntab(T, j));
                    const bool ok = lane >= d && !f;
                    v = ok ? (v ^ t_) : v;
                    f = ok ? of : f;
                }
            }
            uint32_t sin = dpp<0x138>(v);
            if (lane == 0) sin = c_state;
            if (!(KVR_ABLATE & 16) && m != 0) {
                const int r = m & 3;
                uint32_t rp = snap, cf = kmul(sin, ntab(T, NKT + qm));
                for (int b = 0; b < r; ++b) {
                    rp = crc1(rp, (wm >> (8 * b)) & 255u, K);
                    cf = crc1(cf, 0u, K);
                }
                p_ms = slot_of(m_ref, m_abs);   // stored at the next tile's top
                p_crc = ~(cf ^ rp);
            }
            if (out) {
                n_carry = 1;
                c_state = rl32(v, 63);
                n_ve = out_ve;
                n_ref = slot_of(out_ref, out_abs);
            }
        }

        // ---- bookkeeping (the TileRes store waits for the next tile's top) --------------------
        if (in_stripe) {
            p_tres = true;
            p_tile = k;
            p_tr.pool_off = nrec ? b1 : 0ull;
            p_tr.pool_off2 = b2;
            p_tr.count = nrec;
            p_tr.count1 = c1 < nrec ? c1 : nrec;
            total += nrec;
            if (walk) entry = tile_exit;
        }
        carry = n_carry;
        c_vb = n_vb; c_ve = n_ve; c_slot = n_ref;
        if (err_pos != NONE) stop = 1;
        else if (walk && tile_exit == ERRP) {
            stop = 1; err_pos = entry; err_kind = KVR_E_VAL;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain an unused prefetch before exit
    const uint32_t kfirst = k < sd.t_end ? k : sd.t_end;
    for (uint32_t kk = kfirst + lane; kk < sd.t_end; kk += 64) {
        TileRes tr;
        tr.pool_off = 0; tr.pool_off2 = 0; tr.count = 0; tr.count1 = 0;
        tres[sg.tile0 + kk] = tr;
    }
    if (lane == 0) {
        StripeRes r;
        r.entry = stripe_entry;
        r.exit = (err_pos != NONE) ? ERRP : (stripe_entry == NONE ? NONE : entry);
        r.err_pos = err_pos;
        r.err_aux = err_aux;
        r.err_kind = (err_pos != NONE) ? err_kind : 0u;
        r.count = total;
        r.forced = redo_mode ? 1u : 0u;
        r.pad = 0;
        sres[si] = r;
    }
}

}  // namespace v8
}  // namespace kvr
