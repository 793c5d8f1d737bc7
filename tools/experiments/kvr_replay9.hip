/*
 * kvr_replay9.hip — k_replay9 (V9), the hot path (gfx950).
 *
 * The walk of src/store/engine.rs:79-154 (first error in record order; CRC-32/ISO-HDLC of keys
 * and values = crc32fast::hash, src/volume/storage.rs:27) with the outputs of V7/V8 (StripeRes per
 * stripe, TileRes per tile, 32-B tuples in the pool), organised for what bounds those kernels on
 * MI355X: each wave walked ONE record chain, a serial dependency of ~1 us per 8-KiB tile (header
 * read -> length -> next header), and 12-16 waves per CU could not hide it (V8 hops-only: 1.08
 * ms against 0.71 ms of loads).
 *
 * V9 puts FOUR stripes in a wave, one per 16-lane quarter (= one DPP row).  A tile is 2 KiB: lane
 * q of a quarter holds the 128-B unit [128 q, 128 q + 128) of its stripe's current tile.
 *   - Every instruction of the hop loop advances four independent chains (the hop state is per
 *     lane, uniform within a quarter, kept in VGPRs: VALU, not the CU's single scalar unit).
 *   - The per-unit CRC pieces are joined by a segmented scan inside the quarter: DPP row_shr
 *     1, 2, 4, 8 with the constant multipliers x^(8*128*d); no cross-row step.
 *   - Per-stripe state (entry, carry, pool chunk, first error, bookkeeping) lives in VGPRs.
 * Per tile: the landing registers (this tile, loaded during the previous one) go to the quarter's
 * LDS slot, the next tile's loads are issued into them at once (in flight during the whole tile),
 * then: entry search (a stripe's first tile), hops (VALU fast path; the exact general step for
 * anything else), records (one lane per record: key CRC, UTF-8, short values, tuple), unit CRC +
 * scan + finalize for values crossing unit boundaries.
 *
 * LDS (160 KiB, 12 waves): the 64-KiB CRC table area of V8 (paired slice-by-2 rows, nibble tables
 * and IX in the holes) + one 8-KiB slot per wave (four 2-KiB quarter tiles; granule i of unit q
 * at granule i ^ (q & 7): conflict-free ds_write_b128).
 */
#include "kvr_device.h"
#include <type_traits>

namespace kvr {
namespace v9 {

#ifndef KVR9_RT
#define KVR9_RT 512               // 8 waves: the per-lane stripe state needs up to 256 VGPRs
#endif
#ifndef KVR9_TOPPF
#define KVR9_TOPPF 1              // 1: next tile's loads issued at the tile's top; 0: after the records
#endif
constexpr int RT = KVR9_RT;
constexpr int WPB = RT / 64;
constexpr int QPW = 4;                    // stripes (quarters) per wave
constexpr int QL = 16;                    // lanes per quarter
constexpr int TILE = QL * SC;             // 2 KiB
constexpr int UW = SC / 4;
constexpr int SC_LOG = 7;
constexpr uint32_t N32 = 0xFFFFFFFFu;
constexpr uint32_t POOL_CHUNK = 2048;
constexpr uint32_t TILE_RECS = TILE / 5 + 1;
static_assert(POOL_CHUNK >= TILE_RECS, "the rest of a tile's records fits in one fresh chunk");
constexpr int32_t FAR = 1 << 30;
constexpr int KEYW = 6;
constexpr int VALW = SMALL / 4;
constexpr int NKT = 4;                    // scan multipliers x^(8*SC*2^j), j < 4 (in-row steps)
constexpr int NKQ0 = 6;                   // first KQ nibble table (the V8 hole layout: KT 0..5)
constexpr int HIX = 4 * (6 + NQ);
static_assert(HIX + (NIX + 31) / 32 <= 256, "nibble tables and IX fit in the holes");

struct __align__(16) Smem {
    uint32_t T[256 * 64];
    uint32_t tiles[WPB][QPW * TILE / 4];
};
static_assert(sizeof(Smem) <= 163840, "LDS");

#ifndef KVR_ABLATE
#define KVR_ABLATE 0
#endif

// a copy the compiler cannot prove wave-uniform: what is computed from it stays in VGPRs
__device__ __forceinline__ int32_t vdiv(int32_t x) {
    int32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
template <int CTRL, int ROWS = 0xF, bool BC = true>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, BC);
}
// quarter-scope collectives (qb = first lane of the quarter)
__device__ __forceinline__ uint32_t qbc(uint32_t v, int src) {   // lane src's value (any lane)
    return (uint32_t)__builtin_amdgcn_ds_bpermute(4 * src, (int)v);
}
__device__ __forceinline__ uint64_t qbc64(uint64_t v, int src) {
    return ((uint64_t)qbc((uint32_t)(v >> 32), src) << 32) | qbc((uint32_t)v, src);
}
__device__ __forceinline__ uint32_t qballot(bool p, int qb) {      // this quarter's 16 bits
    return (uint32_t)(__ballot(p) >> qb) & 0xFFFFu;
}

// ---------------------------------------------------------------------------------------
// CRC primitives: slice-by-4 on the table area's rows
//   Row b (256 B): dword 8 t + r = table t (t = 0: one byte, t = k: a byte then k zero bytes) for
//   byte b, replica r < 8; dwords [32, 64) are the holes.  A 4-byte step x = c ^ w needs
//   T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3]; lane l (group g = (l >> 3) & 3, replica l & 7)
//   takes table (g + i) & 3 in its i-th lookup, so the 32 lanes of a half-wave hit 32 distinct
//   banks in every lookup.  The address is one v_perm_b32 (byte 1 = the x byte, byte 0 = this
//   lane's offset for lookup i, kept in L).
// ---------------------------------------------------------------------------------------
struct Crc {
    const uint8_t *t;
    uint32_t L;          // byte i: 4 (8 t_i + r), the row offset of this lane's i-th lookup
    uint32_t s[4];       // v_perm selectors of the four lookups
    uint32_t s0;         // selector of a one-byte step (table 0)
};
__device__ __forceinline__ uint32_t tget(const Crc &k, uint32_t x, uint32_t sel) {
    return *reinterpret_cast<const uint32_t *>(k.t + __builtin_amdgcn_perm(x, k.L, sel));
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c);
__device__ __forceinline__ uint32_t crc4(uint32_t c, uint32_t w, const Crc &k) {
    const uint32_t x = c ^ w;
    uint32_t a0 = tget(k, x, k.s[0]), a1 = tget(k, x, k.s[1]), a2 = tget(k, x, k.s[2]), a3 = tget(k, x, k.s[3]);
    asm("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    return xor3(a0, a1, a2) ^ a3;
}
__device__ __forceinline__ void crc4x2(uint32_t &ca, uint32_t wa, uint32_t &cb, uint32_t wb, const Crc &k) {
    const uint32_t xa = ca ^ wa, xb = cb ^ wb;
    uint32_t a0 = tget(k, xa, k.s[0]), a1 = tget(k, xa, k.s[1]), a2 = tget(k, xa, k.s[2]), a3 = tget(k, xa, k.s[3]);
    uint32_t b0 = tget(k, xb, k.s[0]), b1 = tget(k, xb, k.s[1]), b2 = tget(k, xb, k.s[2]), b3 = tget(k, xb, k.s[3]);
    asm("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
    ca = xor3(a0, a1, a2) ^ a3;
    cb = xor3(b0, b1, b2) ^ b3;
}
__device__ __forceinline__ uint32_t crc1(uint32_t c, uint32_t b, const Crc &k) {
    const uint32_t x = c ^ b;
    return (x >> 8) ^ tget(k, x, k.s0);
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
__device__ __forceinline__ const uint32_t *ntab(const uint32_t *T, int c) { return T + 4 * c * 64 + 32; }
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
// the quarter's tile slot (tile byte o < TILE) and per-lane segment reads
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t swz(uint32_t o) { return o ^ ((o >> 3) & 0x70u); }
__device__ __forceinline__ uint32_t lds32(const uint8_t *tl, uint32_t o) {
    return *reinterpret_cast<const uint32_t *>(tl + swz(o));
}

// Reads relative to a tile's first byte, per lane (each quarter has its own segment): the
// TileSeg interface of V7 (b8 / u32 / w32a / lo / len / lim) over plain global loads.  Bytes of
// the segment are returned as stored; b8 gives 0 outside [0, len); w32a reads whole 4-B words
// inside the segment's 16-B-rounded extent (the allocation), 0 past it.
struct SegRd {
    const uint8_t *tb;    // device address of tile byte 0 (16-B aligned)
    int64_t lo;           // segment position of tile byte 0
    uint64_t len;
    int64_t lim;          // tile-relative end of the readable extent
    __device__ __forceinline__ uint32_t b8(int64_t o) const {
        const int64_t p = lo + o;
        return (p >= 0 && (uint64_t)p < len) ? (uint32_t)tb[o] : 0u;
    }
    __device__ __forceinline__ uint32_t w32a(int64_t o) const {   // o 4-aligned
        return (o >= 0 && o + 4 <= lim) ? *reinterpret_cast<const uint32_t *>(tb + o) : 0u;
    }
    __device__ __forceinline__ uint32_t u32(int64_t o) const {
        if (o >= 0 && o + 8 <= lim) {
            const int64_t a = o & ~3ll;
            return __builtin_amdgcn_alignbyte(w32a(a + 4), w32a(a), (uint32_t)o & 3u);
        }
        return b8(o) | (b8(o + 1) << 8) | (b8(o + 2) << 16) | (b8(o + 3) << 24);
    }
};

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

// the same for longer spans, one word at a time (values of 65..128 B inside one unit)
__device__ inline uint32_t crc_span_lds_loop(const uint8_t *tl, const Crc &K, int o, uint32_t n) {
    const int a = o & ~3;
    const uint32_t sh = (uint32_t)o & 3u;
    uint32_t c = ~0u, cur = lds32(tl, (uint32_t)a);
    uint32_t i = 0;
#pragma unroll 1
    for (; 4u * i + 4u <= n; ++i) {
        const uint32_t nx = lds32(tl, (uint32_t)(a + 4 * (int)i + 4));
        c = crc4(c, __builtin_amdgcn_alignbyte(nx, cur, sh), K);
        cur = nx;
    }
    if (n & 3u) {
        const uint32_t tail = __builtin_amdgcn_alignbyte(lds32(tl, (uint32_t)(a + 4 * (int)i + 4)), cur, sh);
        for (uint32_t b = 0; b < (n & 3u); ++b) c = crc1(c, (tail >> (8 * b)) & 255u, K);
    }
    return c;
}

// CRC register update over segment bytes [o, o + n) through global memory (general path)
__device__ inline uint32_t crc_long(const SegRd &ts, uint32_t c, int64_t o, uint64_t n, const Crc &K) {
    const int64_t e = o + (int64_t)n;
    #pragma unroll 1
    while (o < e && ((o & 3) || o < 0 || o + 8 > ts.lim)) {
        c = crc1(c, ts.b8(o), K);
        ++o;
    }
    #pragma unroll 1
    while (o + 4 <= e && o + 8 <= ts.lim) { c = crc4(c, ts.w32a(o), K); o += 4; }
    #pragma unroll 1
    while (o < e) { c = crc1(c, ts.b8(o), K); ++o; }
    return c;
}

struct RecRes {
    uint32_t err, kind;
    uint64_t aux;
};

// the record at tile offset o with every engine.rs check, in engine.rs order
__device__ inline RecRes do_record(const SegRd &ts, const Crc &K, int64_t o, uint32_t j, uint64_t slot, uint32_t seg,
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

// lane's 128-B unit of a tile: eight 16-B loads from ua, the words past the segment's
// 16-B-rounded end read as 0 (ue: end of the readable extent, device address)
__device__ __forceinline__ void load_unit(const uint8_t *ua, const uint8_t *uend, bool full, uint32_t *r) {
    if (full) {
#pragma unroll
        for (int i = 0; i < UW / 4; ++i) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(ua + 16 * i);
            r[4 * i] = a.x; r[4 * i + 1] = a.y; r[4 * i + 2] = a.z; r[4 * i + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < UW / 4; ++i) {
            u32x4 a = {0u, 0u, 0u, 0u};
            if (ua + 16 * i + 16 <= uend) a = *reinterpret_cast<const u32x4 *>(ua + 16 * i);
            r[4 * i] = a.x; r[4 * i + 1] = a.y; r[4 * i + 2] = a.z; r[4 * i + 3] = a.w;
        }
    }
}

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(RT) void k_replay9(const SegDesc *__restrict__ segs,
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
        S.T[b * 64 + d] = tb.crc8[(d >> 3) * 256 + b];
    }
    for (int i = tid; i < (6 + NQ) * 128; i += RT) {
        const int c = i >> 7, ii = (i >> 4) & 7, n = i & 15;
        const int set = c < 6 ? c : KSET_Q + (c - 6);
        S.T[(4 * c + (ii >> 1)) * 64 + 32 + 16 * (ii & 1) + n] = tb.kmul[(set * 8 + ii) * 16 + n];
    }
    for (int j = tid; j < NIX; j += RT) S.T[(HIX + (j >> 5)) * 64 + 32 + (j & 31)] = tb.initx[j];
    __syncthreads();   // the only workgroup barrier

    Crc K;
    {
        const uint32_t g = (uint32_t)(lane >> 3) & 3u, r = (uint32_t)lane & 7u;
        K.t = reinterpret_cast<const uint8_t *>(S.T);
        K.L = 0;
        K.s0 = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t t = (g + i) & 3u;
            K.L |= (4u * (8u * t + r)) << (8 * i);
            K.s[i] = 0x0C0C0000u | ((4u + (3u - t)) << 8) | i;
            if (t == 0u) K.s0 = 0x0C0C0400u | i;
        }
    }
    const uint32_t *T = S.T;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ql = lane & 15, qb = lane & 48, qd = lane >> 4;
    uint8_t *const tl = reinterpret_cast<uint8_t *>(S.tiles[wv]) + TILE * qd;   // the quarter's tile slot
    const uint32_t gq = (blockIdx.x * WPB + (uint32_t)wv) * QPW + (uint32_t)qd;  // quarter index in the grid

    // ---- this quarter's stripe (all per lane, uniform within the quarter) -----------------
    bool live = true;
    uint32_t si = 0;
    uint64_t forced = NONE;
    if (redo_mode) {
        if (gq >= link->n_redo || link->status != 3) live = false;
        else { si = redo[gq].stripe; forced = redo[gq].entry; }
    } else {
        if (gq >= n_stripes) live = false;
        else si = gq;
    }
    if (!__ballot(live)) return;
    const StripeDesc sd = live ? stripes[si] : StripeDesc{0, 0, 0, 0};
    const SegDesc sg = live ? segs[sd.seg] : SegDesc{};
    const uint64_t len = sg.len;
    const int64_t d0 = sg.d0;
    const int64_t shi_i = (int64_t)sd.t_end * TILE - d0;
    const uint64_t s_hi = (uint64_t)shi_i > len ? len : (uint64_t)shi_i;
    const uint8_t *abase = sg.base - d0;                       // 16-B aligned: tile k at abase + k * TILE
    const uint8_t *aend = abase + ((d0 + (int64_t)len + 15) & ~15ll);   // end of the readable extent

    uint64_t entry = redo_mode ? forced : ((sd.t_begin == 0) ? 0ull : NONE);
    bool search = entry == NONE;
    uint64_t stripe_entry = (entry != NONE && entry >= s_hi) ? NONE : entry;
    int stop = live ? ((entry != NONE && entry >= s_hi) ? 2 : 0) : 2;
    if (live && entry != NONE && (int64_t)entry < (int64_t)sd.t_begin * TILE - d0) {   // bug trap
        stop = 2;
        stripe_entry = NONE;
        if (ql == 0) atomicOr(&ctr->overflow, 4u);
    }
    uint64_t err_pos = NONE, err_aux = 0;
    uint32_t err_kind = 0, total = 0;
    uint64_t chunk_base = 0, chunk_left = 0;
    uint32_t carry = 0, c_state = 0;
    uint64_t c_vb = 0, c_ve = 0, c_slot = 0;
    bool p_tres = false;
    TileRes p_tr{};
    uint32_t p_tile = 0;
    uint64_t p_ms = NONE;
    uint32_t p_crc = 0;

    uint32_t w[UW];
    bool loaded = false;
    uint32_t k = sd.t_begin;
    {
        const uint8_t *ua = abase + (int64_t)k * TILE + 128 * ql;
        const bool go = !stop && k < sd.t_end && k < sg.n_tiles;
        const bool full = ua + 128 <= aend;
        if (go) {
            if (__ballot(!full) == 0ull) load_unit(ua, aend, true, w);
            else load_unit(ua, aend, full, w);
            loaded = true;
        }
    }
    for (;;) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (p_tres && ql == 0) tres[sg.tile0 + p_tile] = p_tr;
        if (p_ms != NONE && p_ms < pool_cap) pool[p_ms].crc32 = p_crc;
        p_tres = false;
        p_ms = NONE;
        const bool in_stripe = k < sd.t_end;
        const bool active = !stop && (in_stripe || carry) && k < sg.n_tiles;
        if (__ballot(active) == 0ull) break;
        if (!active) continue;   // a finished quarter idles until the wave is done (its loads were drained)

        const uint8_t *ua0 = abase + (int64_t)k * TILE + 128 * ql;
        if (!loaded) {
            load_unit(ua0, aend, ua0 + 128 <= aend, w);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < UW / 4; ++i) {
            const u32x4 v = {w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
            *reinterpret_cast<u32x4 *>(tl + 128 * ql + 16 * (i ^ (ql & 7))) = v;
        }
        loaded = false;
        if (KVR9_TOPPF && k + 1 < sd.t_end && k + 1 < sg.n_tiles) {
            const uint8_t *ua = ua0 + TILE;
            load_unit(ua, aend, ua + 128 <= aend, w);
            loaded = true;
        }

        if (KVR_ABLATE & 64) {   // loads only (FETCH_SIZE calibration, timing floor)
            const uint32_t x = lds32(tl, 4u * (uint32_t)ql);
            if (x == 0x9E3779B9u && ql == 0) atomicOr(&ctr->overflow, 8u);
            carry = 0;
            if (!KVR9_TOPPF && k + 1 < sd.t_end && k + 1 < sg.n_tiles) {
                const uint8_t *ua = ua0 + TILE;
                load_unit(ua, aend, ua + 128 <= aend, w);
                loaded = true;
            }
            ++k;
            continue;
        }
        const int64_t lo = (int64_t)k * TILE - d0;
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        const int64_t rem = (int64_t)len - lo;
        const int64_t vlo_r = (int64_t)vlo - lo, vhi_r = (int64_t)vhi - lo;
        SegRd ts;
        ts.tb = abase + (int64_t)k * TILE;
        ts.lo = lo;
        ts.len = len;
        ts.lim = (int64_t)(aend - ts.tb);
        const int us = ql * SC, ue = us + SC;

        // ---- stripe entry: the first plausible record start --------------------------------
        if (in_stripe && search) {
            uint32_t u[UW];
#pragma unroll
            for (int i = 0; i < UW / 4; ++i) {
                const u32x4 v = *reinterpret_cast<const u32x4 *>(tl + 128 * ql + 16 * (i ^ (ql & 7)));
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
                const uint32_t fnd = qballot(cand >= 0, qb);
                if (fnd != 0u && ql > __builtin_ctz(fnd)) { m0 = m1 = m2 = m3 = 0u; }
                if (qballot((m0 | m1 | m2 | m3) != 0u, qb) == 0u) break;
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
            const uint32_t fnd = qballot(cand >= 0, qb);
            const int cl = fnd ? __builtin_ctz(fnd) : 0;
            const uint32_t cv = qbc((uint32_t)cand, qb + cl);
            if (fnd != 0u) { entry = (uint64_t)(lo + (int64_t)(int32_t)cv); search = false; stripe_entry = entry; }
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
            if (KVR_ABLATE & 4) p = vhi_r;
#pragma unroll 1
            while (p < vhi_r && !broke && err_rec == N32) {
                uint32_t nb = 0, kmx = 0;
                int32_t myrec = -1;
                uint32_t my_op = 0, my_klen = 0, my_vlen = 0;
#pragma unroll 1
                for (;;) {   // the hops of one batch (<= QL records)
                    // ---- fast hops: header and vlen in the slot, every bound a compare ----------
                    if (!huge && !(KVR_ABLATE & 32)) {
                        int32_t q = vdiv((int32_t)p);
                        uint32_t n = (uint32_t)vdiv((int32_t)nb), kx = (uint32_t)vdiv((int32_t)kmx);
                        uint32_t fany = 0, fo_e2 = 0, fo_ref = N32;
                        int32_t la = -2, lm = 0;
                        uint32_t lmr = 0;
                        const uint32_t rem32 = (uint32_t)rem, vhi32 = (uint32_t)vhi_r;
#pragma unroll 1
                        for (;;) {
                            const uint32_t uq = (uint32_t)q;
                            if (!(uq < vhi32 && n < (uint32_t)QL && uq + 8u <= (uint32_t)TILE)) break;
                            const uint32_t a = uq & ~3u;
                            const uint32_t x0 = lds32(tl, a), x1 = lds32(tl, a + 4u);
                            const uint32_t op = __builtin_amdgcn_alignbyte(x1, x0, uq & 3u) & 255u;
                            const uint32_t klen = (uint32_t)((((uint64_t)x1 << 32) | x0) >> (8u * ((uq & 3u) + 1u)));
                            const uint32_t rq = rem32 - uq;
                            const uint32_t e = uq + 5u + klen;
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
                            const bool me = ql == (int)n;
                            myrec = me ? q : myrec;
                            my_op = me ? op : my_op;
                            my_klen = me ? klen : my_klen;
                            my_vlen = me ? vlen : my_vlen;
                            kx = klen > kx ? klen : kx;
                            const uint32_t lv = set & (vlen > (uint32_t)SMALL ? 1u : 0u) &
                                                ((vb >> SC_LOG) != ((e2 - 1u) >> SC_LOG) ? 1u : 0u);
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
                        nb = n;
                        kmx = kx;
                        if (fany) any_long = true;
                        if (fo_ref != N32) { out = true; out_ve = (uint64_t)(lo + (int64_t)fo_e2); out_ref = fo_ref; out_abs = false; }
                        p = q;
                    }
                    if (!(p < vhi_r && nb < (uint32_t)QL)) break;
                    // ---- one general hop (header or vlen outside the slot, a violation, >2 GiB) --
                    uint32_t op, klen;
                    if (p >= 0 && p + 8 <= TILE) {
                        const uint32_t a = (uint32_t)p & ~3u;
                        const uint32_t x0 = lds32(tl, a), x1 = lds32(tl, a + 4u);
                        op = __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)p & 3u) & 255u;
                        klen = (uint32_t)((((uint64_t)x1 << 32) | x0) >> (8u * (((uint32_t)p & 3u) + 1u)));
                    } else {
                        op = ts.b8(p);
                        klen = rem - p >= 5 ? ts.u32(p + 1) : 0u;
                    }
                    const bool me = ql == (int)nb;
                    myrec = me ? (int32_t)p : myrec;
                    my_op = me ? op : my_op;
                    my_klen = me ? klen : my_klen;
                    ++nb;
                    if (op > 1u || rem - p < 5 || (uint64_t)klen > (uint64_t)(rem - p - 5)) { broke = true; break; }
                    kmx = klen > kmx ? klen : kmx;
                    const int64_t e = p + 5 + (int64_t)klen;
                    if (op == 1u) { p = e; continue; }
                    if (rem - e < 4) { broke = true; break; }
                    uint32_t vlen;
                    if (e + 8 <= TILE) {
                        const uint32_t a = (uint32_t)e & ~3u;
                        vlen = __builtin_amdgcn_alignbyte(lds32(tl, a + 4u), lds32(tl, a), (uint32_t)e & 3u);
                    } else {
                        vlen = ts.u32(e);
                    }
                    my_vlen = ql == (int)nb - 1 ? vlen : my_vlen;
                    const int64_t vb = e + 4;
                    if ((uint64_t)vlen > (uint64_t)(rem - vb)) { broke = true; break; }
                    const int64_t e2 = vb + (int64_t)vlen;
                    if (vlen > (uint32_t)SMALL && (vb >> SC_LOG) != ((e2 - 1) >> SC_LOG)) {
                        const uint64_t idx = nrec + nb - 1;
                        if (vb < TILE) consider((int32_t)vb, (uint64_t)(lo + e2), idx, false, false);
                        else { n_carry = 2; n_vb = (uint64_t)(lo + vb); n_ve = (uint64_t)(lo + e2); n_ref = idx; n_abs = false; }
                    }
                    p = e2;
                }
                // pool slots of the batch (one run: a fresh chunk holds any tile's rest)
                if (nb > chunk_left) {
                    const uint64_t cm = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
                    uint64_t bb = 0;
                    if (ql == 0) {
                        bb = atomicAdd(reinterpret_cast<unsigned long long *>(&ctr->pool_cursor), (unsigned long long)cm);
                        if (bb + cm > pool_cap) atomicOr(&ctr->overflow, 1u);
                    }
                    chunk_base = qbc64(bb, qb);
                    chunk_left = cm;
                    if (nrec) { b2 = chunk_base; c1 = nrec; }
                }
                if (nrec == 0) b1 = chunk_base;
                const uint64_t slot = chunk_base + (uint64_t)ql;
                chunk_base += nb;
                chunk_left -= nb;
                uint32_t rerr = N32, rkind = 0;
                uint64_t raux = 0;
                const uint32_t j = nrec + (uint32_t)ql;
                if (!(KVR_ABLATE & 1) && myrec >= 0) {
                    if (broke && ql == (int)nb - 1) {
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
                                    else t.crc32 = ~crc_long(ts, ~0u, vb, my_vlen, K);
                                } else if ((vb >> SC_LOG) == ((vb + (int)my_vlen - 1) >> SC_LOG)) {   // inside one unit
                                    if ((vb & ~3) + 4 * (UW + 1) <= TILE)
                                        t.crc32 = ~crc_span_lds_loop(tl, K, vb, my_vlen);
                                    else t.crc32 = ~crc_long(ts, ~0u, vb, my_vlen, K);
                                }
                            }
                            if (slot < pool_cap) pool[slot] = t;
                        }
                    }
                }
                // first error of the batch (lowest record index in the quarter)
                if (qballot(rerr != N32, qb)) {
                    uint32_t er = rerr;
#pragma unroll
                    for (int dd = 8; dd >= 1; dd >>= 1) {
                        const uint32_t o = __shfl_xor(er, dd, 16);
                        er = o < er ? o : er;
                    }
                    err_rec = er;
                    const int el = qb + (int)(err_rec - nrec);
                    err_kind = qbc(rkind, el);
                    err_aux = qbc64(raux, el);
                    err_pos = (uint64_t)(lo + (int64_t)(int32_t)qbc((uint32_t)myrec, el));
                }
                nrec = err_rec != N32 ? err_rec : nrec + nb;
            }
            tile_exit = broke ? ERRP : (uint64_t)(lo + p);
        }
        // the next tile's loads: in flight during the CRC phase and the next top (issued after
        // the records' stores, so the top's vmcnt(0) waits only for them)
        if (!KVR9_TOPPF && k + 1 < sd.t_end && k + 1 < sg.n_tiles) {
            const uint8_t *ua = ua0 + TILE;
            load_unit(ua, aend, ua + 128 <= aend, w);
            loaded = true;
        }
        if (c1 == N32) c1 = nrec;
        auto slot_of = [&](uint64_t ref, bool is_abs) -> uint64_t {
            return is_abs ? ref : (ref < c1 ? b1 + ref : b2 + (ref - c1));
        };
        if (n_carry == 2u && !n_abs) n_ref = slot_of(n_ref, false);

        // ---- C. CRC of long values (unit chains, in-row scan, finalize) -----------------------
        if (!(KVR_ABLATE & 2) && any_long) {
            constexpr int H = UW / 2;
            // granule g (words 4g..4g+3) of this lane's unit, from the slot
            auto gran = [&](int g) -> u32x4 {
                return *reinterpret_cast<const u32x4 *>(tl + 128 * ql + 16 * (g ^ (ql & 7)));
            };
            const int qm = m >> 2;
            const int qa = (vx && a_off >= 0) ? (a_off >> 2) : -1;
            const uint32_t amask = ~0u << (8 * (a_off & 3));
            const int qh = qm & (H - 1), qah = qa >= 0 ? (qa & (H - 1)) : -1;
            const bool mb = qm >= H, ab = qa >= H;
            uint32_t ca = 0, cb = 0, sn = 0, wm = 0;
            if (KVR_ABLATE & 8) {
                const u32x4 g0 = gran(0);
                ca = g0.x; cb = g0.y;
            } else if (!__ballot(m != 0 || qa >= 0)) {
#pragma unroll
                for (int g = 0; g < H / 4; ++g) {
                    const u32x4 A = gran(g), B = gran(g + H / 4);
                    crc4x2(ca, A.x, cb, B.x, K);
                    crc4x2(ca, A.y, cb, B.y, K);
                    crc4x2(ca, A.z, cb, B.z, K);
                    crc4x2(ca, A.w, cb, B.w, K);
                }
            } else {
#pragma unroll
                for (int g = 0; g < H / 4; ++g) {
                    const u32x4 A = gran(g), B = gran(g + H / 4);
                    const uint32_t ua[4] = {A.x, A.y, A.z, A.w}, ub[4] = {B.x, B.y, B.z, B.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int kk = 4 * g + e;
                        const bool s_ = kk == qh;
                        sn = s_ ? (mb ? cb : ca) : sn;
                        wm = s_ ? (mb ? ub[e] : ua[e]) : wm;
                        const bool r = kk == qah, ra = r && !ab, rb = r && ab;
                        ca = ra ? 0u : ca;
                        cb = rb ? 0u : cb;
                        crc4x2(ca, ra ? (ua[e] & amask) : ua[e], cb, rb ? (ub[e] & amask) : ub[e], K);
                    }
                }
                sn = qm == UW ? cb : sn;
            }
            const uint32_t pa = kmul(ca, ntab(T, NKQ0 + H));
            const uint32_t ps = kmul(ca, ntab(T, NKQ0 + (qm > H ? qm - H : 0)));
            const uint32_t c = qa >= H ? cb : (pa ^ cb);
            const uint32_t snap = qm < H ? sn : (ps ^ sn);
            uint32_t v = 0, f = 1;
            if (vx) {
                if (a_off >= 0) v = c ^ ixv(T, SC - a_off);
                else if (ql == 0 && vx_carry) v = c ^ kmul(c_state, ntab(T, 0));
                else { v = c; f = 0; }
            }
            // segmented scan inside the quarter (one DPP row): state at the end of unit q =
            // f ? v : state(q-1) * x^(8*SC) ^ v; step d joins spans [q-d+1, q] and [q-2d+1, q-d]
#define KVR9_SCAN(CTRL, D, J)                                                \
            {                                                                \
                const uint32_t ov = dpp<CTRL>(v), of = dpp<CTRL>(f);         \
                const uint32_t t_ = kmul(ov, ntab(T, J));                    \
                const bool ok = ql >= (D) && !f;                             \
                v = ok ? (v ^ t_) : v;                                       \
                f = ok ? of : f;                                             \
            }
            if (!(KVR_ABLATE & 16)) {
                KVR9_SCAN(0x111, 1, 0)
                KVR9_SCAN(0x112, 2, 1)
                KVR9_SCAN(0x114, 4, 2)
                KVR9_SCAN(0x118, 8, 3)
            }
#undef KVR9_SCAN
            uint32_t sin = dpp<0x111>(v);        // row_shr:1: the state at this unit's start
            if (ql == 0) sin = c_state;
            if (!(KVR_ABLATE & 16) && m != 0) {
                const int r = m & 3;
                uint32_t rp = snap, cf = kmul(sin, ntab(T, NKQ0 + qm));
                for (int b = 0; b < r; ++b) {
                    rp = crc1(rp, (wm >> (8 * b)) & 255u, K);
                    cf = crc1(cf, 0u, K);
                }
                p_ms = slot_of(m_ref, m_abs);   // stored at the next tile's top
                p_crc = ~(cf ^ rp);
            }
            const uint32_t v15 = qbc(v, qb + 15);
            if (out) {
                n_carry = 1;
                c_state = v15;
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
        ++k;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!live) return;
    const uint32_t kfirst = k < sd.t_end ? k : sd.t_end;
    for (uint32_t kk = kfirst + (uint32_t)ql; kk < sd.t_end; kk += QL) {
        TileRes tr;
        tr.pool_off = 0; tr.pool_off2 = 0; tr.count = 0; tr.count1 = 0;
        tres[sg.tile0 + kk] = tr;
    }
    if (ql == 0) {
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

}  // namespace v9
}  // namespace kvr
