/*
 * kvr_replay_kernel.hip — k_replay (V6), the hot path (gfx950).
 *
 * One WAVE replays one stripe (consecutive 4-KiB tiles of one segment) exactly as
 * src/store/engine.rs:79-154 walks a segment file, and emits one 32-B kvr_tuple per record with
 * the CRC-32 of its key and of its value (crc32fast::hash semantics, src/volume/storage.rs:27).
 * A workgroup holds 16 independent stripes that share the CRC tables; after the tables are
 * staged in LDS there is no workgroup barrier, so a wave waiting on HBM never holds up another.
 *
 * Per tile, lane l owns the 64-B unit [64 l, 64 l + 64), prefetched one tile ahead into registers
 * with 16-B buffer loads and stored to the wave's LDS tile:
 *   F  framing, exact from the tile entry (the previous tile's exit).  The wave hops header to
 *      header in scalar registers: one hop reads a 256-B window of the tile into the 64 lanes
 *      (one dword each) and decodes op / key_len / val_len with readlanes, so consecutive short
 *      records cost no further LDS round trip.  Records are taken in batches of 64.  Only the
 *      stripe's first tile guesses: it takes its first plausible record start, which k_link
 *      checks against the previous stripe's exit (a wrong guess is re-walked from the true one).
 *   R  records: lane j emits record j of the batch with the engine.rs check the hops did not
 *      already make (UTF-8 of the key), the key CRC, and the CRC of a value of at most 64 B; the
 *      record that broke the chain takes the general path (every check in engine.rs order).
 *      A longer value is folded, per unit, into "which value crosses this unit's end, and where
 *      does it start" / "which value ends inside this unit, and where".
 *   C  long values: each lane CRCs its unit's piece in one pass (a snapshot at the inner end, a
 *      restart at an inner start); a segmented scan across the wave (DPP row shifts, then row
 *      broadcasts; the multipliers x^(8*64*d) come from nibble tables) gives the CRC
 *      register at every unit boundary; the lane holding a value's last byte finishes that CRC.
 *      A value running past the tile hands its register to the next tile of the stripe, so no
 *      variable GF(2) multiply is needed.
 *
 * CRC tables: the slice-by-2 byte tables (T0: one byte, T1: a byte followed by a zero byte) are
 * replicated once per LDS bank: the entry for byte b of table t in lane l's copy sits at byte
 * address b*256 + t*128 + 4 (l & 31), in bank (l & 31), so no lookup of a wave ever conflicts,
 * and its address is a single v_perm_b32 of the register byte and the lane's constant.
 */
#include "kvr_device.h"

namespace kvr {

constexpr int RT = 1024;                  // threads per workgroup
constexpr int WPB = RT / 64;              // stripes (waves) per workgroup
constexpr int UNITS = TILE / SC;          // 64 units per tile = one per lane
static_assert(UNITS == 64, "one 64-B unit per lane");
constexpr uint32_t N32 = 0xFFFFFFFFu;
constexpr uint64_t BEYOND = ~0ull - 2;    // record end not readable from the tile (>= tile end)
constexpr uint32_t POOL_CHUNK = 2048;
constexpr int32_t FAR = 1 << 30;          // "ends beyond the tile" (tile-relative clamp)
constexpr int KEYW = 6;                   // key words the record fast path holds (keys <= 24 B)
constexpr int WIN = (TILE + HALO) / 4;    // dwords of tile + halo

struct WaveLds {                          // one stripe's scratch: the tile and its halo
    uint8_t  tile[TILE + HALO];
};

// The tables come first: every table address is a lane-dependent VGPR plus a constant below
// 64 KiB, which the ds_read instruction carries as its immediate offset.
struct __align__(16) Smem {
    uint32_t KR[8 * 16 * 32];             // [i][n][k]: (n << 4i) * x^(8*64*(k+1)), k < 32
    uint32_t KT[4 * 8 * 16];              // [j][i][n]: (n << 4i) * x^(8*64*2^j), j < 4
    uint32_t KQ[17 * 8 * 16];             // [q][i][n]: (n << 4i) * x^(8*4q), q <= 16
    uint32_t IX[68];                      // 0xFFFFFFFF * x^(8j): initial register pushed through j bytes
    uint32_t C2[2 * 256 * 32];            // lane-replicated slice-by-2 byte tables (64 KiB)
    WaveLds  w[WPB];
};

#ifndef KVR_ABLATE
#define KVR_ABLATE 0   // diagnostic builds only: 1 skip records, 2 skip value CRC, 4 skip hops
#endif

#ifdef KVR_PROF
__device__ unsigned long long g_prof[16];
#define KVR_STAMP(i)                                                        \
    do {                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
        prof_acc[i] += t_ - t_last;                                         \
        t_last = t_;                                                        \
    } while (0)
#else
#define KVR_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ void wsync() {   // LDS writes of this wave visible to its other lanes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t uni64(uint64_t v) {   // wave-uniform value into SGPRs
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// lane l's value, l wave-uniform (v_readlane: no LDS traffic, unlike a shuffle)
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) | __builtin_amdgcn_readlane((uint32_t)v, l);
}
// two consecutive dwords of a wave-spread window as one little-endian 64-bit value, from word i
__device__ __forceinline__ uint64_t win64(uint32_t win, int i) {
    return ((uint64_t)rl32(win, i + 1) << 32) | rl32(win, i);
}

// DPP move (no LDS): CTRL = row_shr:d (0x110 + d), row_bcast:15 (0x142), row_bcast:31 (0x143),
// wave_shr:1 (0x138); lanes without a source read 0
template <int CTRL, int ROWS = 0xF, bool BC = true>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, BC);
}

// ---------------------------------------------------------------------------------------
// CRC primitives
// ---------------------------------------------------------------------------------------
struct Crc {
    const uint8_t *t;   // the lane-replicated slice-by-2 tables (Smem::C2)
    uint32_t L;         // byte 0: 4 (lane & 31) (T0 copy), byte 1: 128 + 4 (lane & 31) (T1 copy)
};
// v_perm_b32 builds the LDS address: byte 1 = a byte of x, byte 0 = this lane's table copy
constexpr uint32_t SEL_T1_B0 = 0x0C0C0401u, SEL_T0_B1 = 0x0C0C0500u, SEL_T0_B0 = 0x0C0C0400u;
__device__ __forceinline__ uint32_t tget(const Crc &k, uint32_t x, uint32_t sel) {
    return *reinterpret_cast<const uint32_t *>(k.t + __builtin_amdgcn_perm(x, k.L, sel));
}
// the register after the two bytes sitting in x's low half (x = register ^ data)
// (both lookups are issued before either is used: the empty asm keeps the scheduler from
// serialising them, which would cost a third LDS round trip per word)
__device__ __forceinline__ uint32_t crc2(const Crc &k, uint32_t x) {
    uint32_t t0 = tget(k, x, SEL_T1_B0), t1 = tget(k, x, SEL_T0_B1);
    asm volatile("" : "+v"(t0), "+v"(t1));
    return (x >> 16) ^ t0 ^ t1;
}
__device__ __forceinline__ uint32_t crc4(uint32_t c, uint32_t w, const Crc &k) { return crc2(k, crc2(k, c ^ w)); }
__device__ __forceinline__ uint32_t crc1(uint32_t c, uint32_t b, const Crc &k) {
    const uint32_t x = c ^ b;
    return (x >> 8) ^ tget(k, x, SEL_T0_B0);
}

// register state v times a constant K (nibble tables; every lane reads table i at once, so the
// 16 entries sit in 16 banks and equal indices broadcast: conflict free)
// (the eight lookups are independent: the empty asm makes the scheduler issue them all before
// the first use instead of one LDS round trip each)
__device__ __forceinline__ uint32_t xor8(uint32_t *t) {
    asm volatile("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]));
    return ((t[0] ^ t[1]) ^ (t[2] ^ t[3])) ^ ((t[4] ^ t[5]) ^ (t[6] ^ t[7]));
}
__device__ __forceinline__ uint32_t kmul(uint32_t v, const uint32_t *K) {
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = K[i * 16 + ((v >> (4 * i)) & 15u)];
    return xor8(t);
}
// v times x^(8*64*(k+1)), k per lane (column k of KR: bank k mod 32, conflict free)
__device__ __forceinline__ uint32_t kmulr(uint32_t v, const uint32_t *KR, uint32_t k) {
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = KR[(i * 16 + ((v >> (4 * i)) & 15u)) * 32 + k];
    return xor8(t);
}

// CRC register update over segment bytes [p, p+n): LDS when resident (tile + halo), HBM otherwise
__device__ inline uint32_t crc_range(const TileView &tv, uint32_t c, uint64_t p, uint64_t n, const Crc &K) {
    if (tv.in_lds(p, n)) {
        int off = (int)((int64_t)p - tv.lo);
        const int end = off + (int)n;
        #pragma unroll 1
        while (off < end && (off & 3)) { c = crc1(c, tv.lds[off], K); ++off; }
        const uint32_t *w = reinterpret_cast<const uint32_t *>(tv.lds);
        #pragma unroll 1
        while (off + 4 <= end) { c = crc4(c, w[off >> 2], K); off += 4; }
        #pragma unroll 1
        while (off < end) { c = crc1(c, tv.lds[off], K); ++off; }
        return c;
    }
    #pragma unroll 1
    for (uint64_t i = 0; i < n; ++i) c = crc1(c, tv.rd8(p + i), K);
    return c;
}

// ---------------------------------------------------------------------------------------
// the stripe's entry: its first plausible record start (LDS only; k_link verifies it)
// ---------------------------------------------------------------------------------------
// End of the record at p, ERRP (broken framing) or BEYOND (a field lies past the tile: the
// record ends beyond it).  p must be inside the tile and < len.
__device__ __forceinline__ uint64_t next_spec(const TileView &tv, uint64_t p) {
    const uint64_t n = tv.len;
    const int64_t off = (int64_t)p - tv.lo;
    const uint32_t op = tv.lds[off];
    if (op > 1u || n - p < 5) return ERRP;
    if (off + 5 > TILE) return BEYOND;
    const uint64_t e = p + 5 + (uint64_t)tv.lds_u32(off + 1);
    if (e > n) return ERRP;
    if (op == 1u) return e;
    if (n - e < 4) return ERRP;
    const int64_t eo = (int64_t)e - tv.lo;
    if (eo + 4 > TILE) return BEYOND;
    const uint64_t e2 = e + 4 + (uint64_t)tv.lds_u32(eo);
    return e2 > n ? ERRP : e2;
}

// Could the first min(klen, 16) key bytes (those inside the tile) begin a valid UTF-8 string
// without NUL?  Keys are String (engine.rs:114): a candidate whose "key" is random value bytes
// fails the UTF-8 test, and one that starts a few bytes before a true header ([0][len LE]
// makes an in-range length whose "key" is the zero bytes of the true length) fails the NUL test.
// Heuristic only: a true record rejected here (a key holding NUL) is found again by the stripe
// link check and the exact re-walk, so results never depend on it.
__device__ __forceinline__ bool key_prefix_ok(const TileView &tv, int off_k, uint32_t klen) {
    int m = TILE - off_k;
    m = m > 16 ? 16 : m;
    m = (uint32_t)m > klen ? (int)klen : m;
    int i = 0;
    #pragma unroll 1
    while (i < m) {
        const uint32_t b = tv.lds[off_k + i];
        if (b == 0u) return false;
        if (b < 0x80u) { ++i; continue; }
        int w;
        uint32_t c_lo = 0x80u, c_hi = 0xBFu;
        if (b >= 0xC2u && b <= 0xDFu) w = 2;
        else if (b >= 0xE0u && b <= 0xEFu) { w = 3; if (b == 0xE0u) c_lo = 0xA0u; if (b == 0xEDu) c_hi = 0x9Fu; }
        else if (b >= 0xF0u && b <= 0xF4u) { w = 4; if (b == 0xF0u) c_lo = 0x90u; if (b == 0xF4u) c_hi = 0x8Fu; }
        else return false;
        if (i + 1 >= m) return true;
        const uint32_t c1 = tv.lds[off_k + i + 1];
        if (c1 < c_lo || c1 > c_hi) return false;
        for (int k = 2; k < w; ++k) {
            if (i + k >= m) return true;
            if ((tv.lds[off_k + i + k] & 0xC0u) != 0x80u) return false;
        }
        i += w;
    }
    return true;
}

__device__ __forceinline__ bool plausible(const TileView &tv, uint64_t p) {
    const uint64_t nx = next_spec(tv, p);
    if (nx == ERRP) return false;
    {
        const int off = (int)((int64_t)p - tv.lo);
        if (off + 5 < TILE && !key_prefix_ok(tv, off + 5, tv.lds_u32(off + 1))) return false;
    }
    const uint64_t n = tv.len;
    if (nx == BEYOND || nx == n) return true;
    const int64_t o = (int64_t)nx - tv.lo;
    if (o + 5 > TILE) return true;                 // next header outside the tile: cannot check cheaply
    if (tv.lds[o] > 1u || n - nx < 5) return false;
    return nx + 5 + (uint64_t)tv.lds_u32(o + 1) <= n;
}

// first plausible record start in [p0, p1) (inside the tile), or NONE
__device__ __noinline__ uint64_t find_cand(const TileView tv, uint64_t p0, uint64_t p1) {
    if (p0 >= p1) return NONE;
    const int o0 = (int)((int64_t)p0 - tv.lo), o1 = (int)((int64_t)p1 - tv.lo);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(tv.lds);
    #pragma unroll 1
    for (int q = o0 >> 2; q <= (o1 - 1) >> 2; ++q) {
        const uint32_t y = w[q] & 0xFEFEFEFEu;                 // bytes 0x00 / 0x01 become 0
        uint32_t z = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
        const int bq = q * 4;
        if (bq < o0) z &= ~0u << (8 * (o0 - bq));
        if (bq + 4 > o1) z &= (1u << (8 * (o1 - bq))) - 1u;
        #pragma unroll 1
        while (z) {
            const int b = __builtin_ctz(z) >> 3;
            const uint64_t p = (uint64_t)(tv.lo + bq + b);
            if (plausible(tv, p)) return p;
            z &= z - 1u;
        }
    }
    return NONE;
}

// ---------------------------------------------------------------------------------------
// records
// ---------------------------------------------------------------------------------------
struct RecRes {          // one record's outcome
    uint32_t err, kind;  // record index of an error (N32: none) and its KVR_E_* kind
    uint64_t aux;
    uint32_t lng;        // its value is longer than SMALL: 1 starts inside the tile, 2 starts later
    int32_t vb;          // value start, tile-relative (lng 1)
    uint64_t vbabs, ve;  // value start / end, segment offsets
};

// parse + emit the record at p with every engine.rs check, in engine.rs order
__device__ inline RecRes do_record(const TileView &tv, const Crc &K, uint64_t p, uint32_t j, uint64_t slot,
                                   uint32_t seg, kvr_tuple *pool, uint64_t pool_cap) {
    RecRes ro;
    ro.err = N32; ro.kind = 0; ro.aux = 0; ro.lng = 0; ro.vb = 0; ro.vbabs = 0; ro.ve = 0;
    const uint64_t len = tv.len;
    const uint32_t op = tv.rd8(p);
    if (len - p < 5) { ro.err = j; ro.kind = KVR_E_KEY_LEN; return ro; }                 // engine.rs:96
    const uint64_t klen = tv.rd32(p + 1);
    const uint64_t kb = p + 5;
    if (len - kb < klen) { ro.err = j; ro.kind = KVR_E_KEY; return ro; }                  // engine.rs:107
    uint64_t vu = 0;
    uint32_t el = 0;
    if (!utf8_check(tv, kb, klen, &vu, &el)) {                                          // engine.rs:114
        ro.err = j; ro.kind = KVR_E_UTF8; ro.aux = vu | ((uint64_t)el << 32); return ro;
    }
    if (op > 1u) { ro.err = j; ro.kind = KVR_E_OPCODE; ro.aux = op; return ro; }          // engine.rs:143
    kvr_tuple t;
    t.rec_off = p;
    t.seg_idx = seg;
    t.key_len = (uint32_t)klen;
    t.key_tag = ~crc_range(tv, ~0u, kb, klen, K);
    t.op = (uint8_t)op;
    t.flags = 0;
    t.reserved = 0;
    t.crc32 = 0;
    t.val_len = 0;
    if (op == 0u) {
        const uint64_t q = kb + klen;
        if (len - q < 4) { ro.err = j; ro.kind = KVR_E_VAL_LEN; return ro; }              // engine.rs:121
        const uint64_t vlen = tv.rd32(q);
        const uint64_t vb = q + 4, ve = vb + vlen;
        if (len - vb < vlen) { ro.err = j; ro.kind = KVR_E_VAL; return ro; }              // engine.rs:130
        t.val_len = (uint32_t)vlen;
        if (vlen <= (uint64_t)SMALL) {
            t.crc32 = ~crc_range(tv, ~0u, vb, vlen, K);
        } else {
            const int64_t vbr = (int64_t)vb - tv.lo;
            ro.lng = vbr < TILE ? 1u : 2u;
            ro.vb = (int32_t)(vbr < TILE ? vbr : 0);
            ro.vbabs = vb;
            ro.ve = ve;
        }
    }
    if (slot < pool_cap) pool[slot] = t;
    return ro;
}

// this lane's 64-B unit of tile k: four 16-B raw buffer loads through a per-tile resource whose
// range is the 16-B words touching the segment, so words outside it read as 0 in hardware (no
// per-word compares, no select of pointers)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load_unit(const uint8_t *abase, int64_t d0, uint64_t len, uint32_t k, int lane,
                                          uint4 &r0, uint4 &r1, uint4 &r2, uint4 &r3) {
    const int64_t t0 = (int64_t)k * TILE;
    const int64_t first = d0 & ~(int64_t)15, endw = (d0 + (int64_t)len + 15) & ~(int64_t)15;
    const int64_t skip = first > t0 ? first - t0 : 0;
    int64_t nrec = endw - t0 - skip;
    nrec = nrec < 0 ? 0 : (nrec > TILE ? TILE : nrec);
    const uint64_t b = (uint64_t)(abase + t0 + skip);
    const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)b), bhi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const int nr = __builtin_amdgcn_readfirstlane((int)nrec);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((uint64_t)bhi << 32) | blo), (short)0, nr, 0x00020000);
    const int vo = lane * SC - (int)skip;   // negative -> out of range -> 0
    const u32x4 a0 = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0);
    const u32x4 a1 = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16, 0, 0);
    const u32x4 a2 = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 32, 0, 0);
    const u32x4 a3 = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 48, 0, 0);
    r0 = make_uint4(a0.x, a0.y, a0.z, a0.w);
    r1 = make_uint4(a1.x, a1.y, a1.z, a1.w);
    r2 = make_uint4(a2.x, a2.y, a2.z, a2.w);
    r3 = make_uint4(a3.x, a3.y, a3.z, a3.w);
}

// halo of tile k: the next HALO bytes after it, LDS-DMA into tile + TILE (lanes 0 .. HALO/16-1)
__device__ __forceinline__ void load_halo(const uint8_t *abase, int64_t d0, uint64_t len, uint32_t k, int lane,
                                          uint8_t *tile) {
    if (lane < HALO / 16) {
        const int64_t pos = (int64_t)k * TILE - d0 + TILE + 16 * lane;
        if (pos < (int64_t)len)
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void *>(abase + (int64_t)k * TILE + TILE + 16 * lane),
                reinterpret_cast<__attribute__((address_space(3))) void *>(
                    (__attribute__((address_space(3))) uint8_t *)(tile + TILE)),
                16, 0, 0);
    }
}

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(RT) void k_replay(const SegDesc *__restrict__ segs,
                                               const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                               StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                               kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                               Tables tb, const RedoEnt *__restrict__ redo,
                                               const LinkResult *__restrict__ link, int redo_mode,
                                               uint32_t pool_chunk) {
    __shared__ Smem S;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 2 * 256 * 32; i += RT) S.C2[i] = tb.crc8[((i >> 5) & 1) * 256 + (i >> 6)];
    for (int i = tid; i < 8 * 16 * 32; i += RT)
        S.KR[i] = tb.kmul[((KSET_R + (i & 31)) * 8 + (i >> 9)) * 16 + ((i >> 5) & 15)];
    for (int i = tid; i < 4 * 8 * 16; i += RT) S.KT[i] = tb.kmul[i];
    for (int i = tid; i < 17 * 8 * 16; i += RT) S.KQ[i] = tb.kmul[KSET_Q * 8 * 16 + i];
    if (tid < 65) S.IX[tid] = tb.initx[tid];
    __syncthreads();   // the only workgroup barrier: from here on every wave is on its own

    const Crc K{reinterpret_cast<const uint8_t *>(S.C2),
                ((uint32_t)(lane & 31) * 4u) | (((uint32_t)(lane & 31) * 4u + 128u) << 8)};
    // the stripe index is wave-uniform: say so, so that the whole stripe state lives in SGPRs
    const uint32_t gw = blockIdx.x * WPB + (uint32_t)__builtin_amdgcn_readfirstlane(wv);
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
    WaveLds &W = S.w[wv];
    const uint32_t *tw = reinterpret_cast<const uint32_t *>(W.tile);
    const StripeDesc sd = stripes[si];
    const SegDesc sg = segs[sd.seg];
    const uint64_t len = sg.len;
    const int64_t d0 = sg.d0;
    const int64_t shi_i = (int64_t)sd.t_end * TILE - d0;
    const uint64_t s_hi = (uint64_t)shi_i > len ? len : (uint64_t)shi_i;
    const uint8_t *abase = sg.base - d0;   // 16-B aligned: tile k starts at abase + k * TILE

    // stripe state (wave-uniform)
    uint64_t entry = redo_mode ? forced : ((sd.t_begin == 0) ? 0ull : NONE);
    bool search = entry == NONE;
    uint64_t stripe_entry = (entry != NONE && entry >= s_hi) ? NONE : entry;
    int stop = (entry != NONE && entry >= s_hi) ? 2 : 0;   // imposed entry beyond the stripe: nothing starts here
    if (entry != NONE && (int64_t)entry < (int64_t)sd.t_begin * TILE - d0) {   // bug trap: k_link never does this
        stop = 2;
        stripe_entry = NONE;
        if (lane == 0) atomicOr(&ctr->overflow, 4u);
    }
    uint64_t err_pos = NONE, err_aux = 0;
    uint32_t err_kind = 0, total = 0;
    uint64_t chunk_base = 0, chunk_left = 0;
    uint32_t carry = 0, c_state = 0, c_idx = 0;   // 1: a long value crosses the tile start (c_state: its register);
    uint64_t c_vb = 0, c_ve = 0;                  // 2: pending (its value starts in a later tile)

    uint4 n0, n1, n2, n3;   // this lane's unit of the next tile (prefetch)
    load_unit(abase, d0, len, sd.t_begin, lane, n0, n1, n2, n3);
    load_halo(abase, d0, len, sd.t_begin, lane, W.tile);
    bool loaded = true;
    uint32_t k = sd.t_begin;
#ifdef KVR_PROF
    unsigned long long t_last = __builtin_amdgcn_s_memtime();
    unsigned long long prof_acc[16] = {};
#endif
    for (;; ++k) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        KVR_STAMP(5);
        const bool in_stripe = k < sd.t_end;
        if (stop || (!in_stripe && !carry) || k >= sg.n_tiles) break;
        if (!loaded) {
            load_unit(abase, d0, len, k, lane, n0, n1, n2, n3);
            load_halo(abase, d0, len, k, lane, W.tile);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        {
            uint4 *tp = reinterpret_cast<uint4 *>(W.tile + lane * SC);
            tp[0] = n0; tp[1] = n1; tp[2] = n2; tp[3] = n3;
        }
        loaded = (k + 1 < sg.n_tiles) && (k + 1 < sd.t_end || carry);
        if (loaded) load_unit(abase, d0, len, k + 1, lane, n0, n1, n2, n3);
        wsync();

        const int64_t lo = (int64_t)k * TILE - d0;      // segment position of LDS byte 0
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        const int64_t rem = (int64_t)len - lo;          // segment bytes from LDS byte 0 on
        const int64_t vhi_r = (int64_t)vhi - lo;
        const TileView tv{sg.base, W.tile, len, lo};
        const int64_t cs_i = lo + (int64_t)lane * SC;
        const uint64_t cs = cs_i < (int64_t)vlo ? vlo : (uint64_t)cs_i;
        const uint64_t ce = (uint64_t)(cs_i + SC) > vhi ? vhi : (uint64_t)(cs_i + SC);

        KVR_STAMP(0);
        // ---- F + R. framing and records -------------------------------------------------------
        if (in_stripe && search) {   // the stripe's entry: the first plausible record start
            const uint64_t cand = cs < ce ? find_cand(tv, cs, ce) : NONE;
            uint64_t mn = cand;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const uint64_t o = __shfl_xor(mn, d, 64);
                mn = o < mn ? o : mn;
            }
            mn = uni64(mn);
            if (mn != NONE) { entry = mn; search = false; stripe_entry = mn; }
        }
        const bool walk = in_stripe && !search && entry < vhi;
        uint64_t tile_exit = entry;
        // the long values touching this tile, folded into every unit's view as they are found
        const int32_t us = lane * SC, ue = us + SC;
        bool vx = false;                     // a long value crosses the end of this unit
        int32_t a_off = -1;                  // ... starting inside the unit at a_off
        bool vx_carry = false;               // ... the value carried in from the previous tile
        int32_t m = 0;                       // a long value ends inside this unit, at m (1 .. 64)
        uint32_t m_slot = 0;
        bool any_long = false;               // (uniform) some long value touches the tile
        bool out = false;                    // (uniform) a value crosses the tile end
        uint64_t out_ve = 0;
        uint32_t out_slot = 0;
        auto consider = [&](int32_t vb, uint64_t ve_abs, uint32_t slot, bool from_carry) {
            const int64_t v64 = (int64_t)ve_abs - lo;
            const int32_t ver = v64 > FAR ? FAR : (int32_t)v64;
            if (vb < ue && ver > ue) { vx = true; a_off = vb >= us ? vb - us : -1; vx_carry = from_carry; }
            if (vb < us && ver > us && ver <= ue) { m = ver - us; m_slot = slot; }
            if (ver > TILE) { out = true; out_ve = ve_abs; out_slot = slot; }
            any_long = true;
        };
        uint32_t n_carry = 0, n_idx = 0, n_state = 0;
        uint64_t n_vb = 0, n_ve = 0;
        if (carry == 1u) consider(-FAR, c_ve, c_idx, true);
        if (carry == 2u) {                   // a value whose record started in an earlier tile
            if ((int64_t)c_vb - lo < TILE) consider((int32_t)((int64_t)c_vb - lo), c_ve, c_idx, false);
            else { n_carry = 2; n_vb = c_vb; n_ve = c_ve; n_idx = c_idx; }   // still further on
        }
        // pool slots: a tile's records take one contiguous run (k_compact reads them so); a tile
        // holds at most TILE / 5 + 1 record starts
        constexpr uint32_t TILE_RECS = TILE / 5 + 1;
        if (walk && chunk_left < TILE_RECS) {
            const uint64_t cm = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
            unsigned long long b = 0;
            if (lane == 0) {
                b = atomicAdd(&ctr->pool_cursor, (unsigned long long)cm);
                if (b + cm > pool_cap) atomicOr(&ctr->overflow, 1u);
            }
            chunk_base = uni64(b);
            chunk_left = cm;
        }
        const uint64_t pool_base = chunk_base;
        uint32_t nrec = 0, err_rec = N32;    // records emitted; index of the tile's first error
        if (walk) {
            int64_t p = (int64_t)entry - lo;
            bool broke = false;              // the chain broke at the last record walked
            if (KVR_ABLATE & 4) p = vhi_r;
#pragma unroll 1
            while (p < vhi_r && !broke && err_rec == N32) {
                // exact hops, a 256-B window per LDS round trip; lane j keeps record nrec + j
                uint32_t nb = 0, kmx = 0;
                int32_t myrec = -1;
                uint32_t my_op = 0, my_klen = 0, my_vlen = 0;
                int wb = -4096;
                uint32_t win = 0;
#pragma unroll 1
                while (p < vhi_r && nb < 64u) {
                    const int pw = (int)(p >> 2);
                    if (pw < wb || pw + 1 >= wb + 64) {
                        wb = pw;
                        win = wb + lane < WIN ? tw[wb + lane] : 0u;
                    }
                    const uint64_t x = win64(win, pw - wb) >> (8u * (uint32_t)(p & 3));
                    const uint32_t op = (uint32_t)x & 255u;
                    const uint64_t klen = (x >> 8) & 0xFFFFFFFFull;
                    if (lane == (int)nb) { myrec = (int32_t)p; my_op = op; my_klen = (uint32_t)klen; }
                    ++nb;
                    const int64_t e = p + 5 + (int64_t)klen;
                    if (op > 1u || rem - p < 5 || e > rem) { broke = true; break; }
                    kmx = (uint32_t)klen > kmx ? (uint32_t)klen : kmx;
                    if (op == 1u) { p = e; continue; }
                    if (rem - e < 4) { broke = true; break; }
                    uint32_t vlen;
                    if (e + 4 <= TILE + HALO) {
                        const int ew = (int)(e >> 2);
                        if (ew >= wb && ew + 1 < wb + 64) vlen = (uint32_t)(win64(win, ew - wb) >> (8u * (uint32_t)(e & 3)));
                        else vlen = uni32(tv.lds_u32(e));
                    } else {
                        vlen = uni32(tv.rd32((uint64_t)(lo + e)));
                    }
                    if (lane == (int)nb - 1) my_vlen = vlen;
                    const int64_t e2 = e + 4 + (int64_t)vlen;
                    if (e2 > rem) { broke = true; break; }
                    p = e2;
                }
                KVR_STAMP(1);
                // the batch's records: lane j emits record nrec + j
                uint32_t rerr = N32, rkind = 0;
                uint64_t raux = 0;
                bool lng = false;            // its value is longer than SMALL and starts in the tile
                int32_t l_b = 0;
                uint64_t l_e = 0;
                uint32_t hand = 0;           // ... or starts past the tile end
                uint64_t pvb = 0, pve = 0;
                const uint32_t j = nrec + (uint32_t)lane;
                const uint64_t slot = pool_base + j;
                if (!(KVR_ABLATE & 1) && myrec >= 0) {
                    if (broke && lane == (int)nb - 1) {   // the record that broke the chain: every check
                        const RecRes r = do_record(tv, K, (uint64_t)(lo + myrec), j, slot, sd.seg, pool, pool_cap);
                        rerr = r.err; rkind = r.kind; raux = r.aux;
                        if (r.err == N32) { rerr = j; rkind = KVR_E_VAL; }   // defensive: a break is an error
                    } else {
                        const uint32_t kc = kmx > 4u * KEYW ? 4u * KEYW : kmx;
                        const uint32_t nw = (kc + 3u) >> 2;   // key words of the longest fast-path key
                        const int kb = myrec + 5;
                        const uint32_t klen = my_klen;
                        uint32_t c = ~0u;
                        bool done = false;
                        if (klen <= 4u * KEYW && kb + (int)klen + 4 <= TILE + HALO) {
                            const int q = kb >> 2;
                            const uint32_t sh = (uint32_t)kb & 3u;
                            uint32_t r[KEYW + 1];
#pragma unroll
                            for (int i = 0; i <= KEYW; ++i) r[i] = (uint32_t)i <= nw ? tw[q + i] : 0u;
                            uint32_t bad = 0, tail = 0;
#pragma unroll
                            for (int i = 0; i < KEYW; ++i) {
                                if ((uint32_t)i < nw) {
                                    const uint32_t kw = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
                                    const uint32_t n = klen > 4u * i ? klen - 4u * i : 0u;
                                    const uint32_t msk = n >= 4u ? ~0u : ((1u << (8 * n)) - 1u);
                                    bad |= kw & msk & 0x80808080u;
                                    const uint32_t cn = crc4(c, kw, K);
                                    c = n >= 4u ? cn : c;
                                    tail = (n > 0u && n < 4u) ? kw : tail;
                                }
                            }
                            for (uint32_t bb = 0; bb < (klen & 3u); ++bb) c = crc1(c, (tail >> (8 * bb)) & 255u, K);
                            done = bad == 0u;
                        }
                        if (!done) {                  // non-ASCII or long key: the full UTF-8 check
                            uint64_t vu = 0;
                            uint32_t el = 0;
                            if (!utf8_check(tv, (uint64_t)(lo + kb), klen, &vu, &el)) {   // engine.rs:114
                                rerr = j; rkind = KVR_E_UTF8; raux = vu | ((uint64_t)el << 32);
                            } else {
                                c = crc_range(tv, ~0u, (uint64_t)(lo + kb), klen, K);
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
                                const int64_t vb = (int64_t)kb + klen + 4;
                                t.val_len = my_vlen;
                                if (my_vlen <= (uint32_t)SMALL) {
                                    t.crc32 = ~crc_range(tv, ~0u, (uint64_t)(lo + vb), my_vlen, K);
                                } else if (vb < TILE) {
                                    lng = true; l_b = (int32_t)vb; l_e = (uint64_t)(lo + vb) + my_vlen;
                                } else {
                                    hand = 2; pvb = (uint64_t)(lo + vb); pve = pvb + my_vlen;
                                }
                            }
                            if (slot < pool_cap) pool[slot] = t;
                        }
                    }
                }
                KVR_STAMP(6);
                // first error of the batch (lowest record index)
                if (__ballot(rerr != N32)) {
                    uint32_t er = rerr;
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) {
                        const uint32_t o = __shfl_xor(er, d, 64);
                        er = o < er ? o : er;
                    }
                    err_rec = uni32(er);
                    const int el = (int)(err_rec - nrec);
                    err_kind = rl32(rkind, el);
                    err_aux = rl64(raux, el);
                    err_pos = (uint64_t)(lo + (int64_t)rl32((uint32_t)myrec, el));
                }
                // the batch's long values before the error, folded into every unit's view
#pragma unroll 1
                for (unsigned long long mm = __ballot(lng && j < err_rec); mm; mm &= mm - 1ull) {
                    const int l = __builtin_ctzll(mm);
                    consider((int32_t)rl32((uint32_t)l_b, l), rl64(l_e, l), (uint32_t)(pool_base + nrec) + (uint32_t)l, false);
                }
                {   // a value starting past the tile end (the tile's last record): hand it over
                    const unsigned long long bp = __ballot(hand == 2u && j < err_rec);
                    if (bp) {
                        const int ol = __builtin_ctzll(bp);
                        n_carry = 2;
                        n_vb = rl64(pvb, ol);
                        n_ve = rl64(pve, ol);
                        n_idx = (uint32_t)(pool_base + nrec) + (uint32_t)ol;
                    }
                }
                nrec = err_rec != N32 ? err_rec : nrec + nb;
                KVR_STAMP(7);
            }
            tile_exit = broke ? ERRP : (uint64_t)(lo + p);
        }
        chunk_base += nrec;
        chunk_left -= nrec;
        wsync();
        if (loaded) load_halo(abase, d0, len, k + 1, lane, W.tile);   // this tile's halo reads are done

        KVR_STAMP(2);
        // ---- C. CRC of long values --------------------------------------------------------
        if (!(KVR_ABLATE & 2) && any_long) {
            KVR_STAMP(8);
            // one pass over the unit (registers) gives both register pieces this lane owns:
            //  - raw CRC of [0, m) (the value ending here), snapshotted on the way, and
            //  - raw CRC of [a, 64) (the value crossing the unit end), restarting at a's word with
            //    the bytes before a zeroed
            const uint4 *up = reinterpret_cast<const uint4 *>(W.tile + lane * SC);   // this lane's unit
            const uint4 v0 = up[0], v1 = up[1], v2 = up[2], v3 = up[3];
            const uint32_t w[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                                    v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
            const int qm = m >> 2;
            const int qa = (vx && a_off >= 0) ? (a_off >> 2) : -1;
            const uint32_t amask = ~0u << (8 * (a_off & 3));
            // two independent chains, words 0..7 (A) and 8..15 (B), each from a zero register
            uint32_t ca = 0, cb = 0, sa = 0, sb = 0, wm = 0;
            if (!__ballot(m != 0 || qa >= 0)) {
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    ca = crc4(ca, w[kk], K);
                    cb = crc4(cb, w[kk + 8], K);
                }
            } else {
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    sa = kk == qm ? ca : sa;
                    sb = kk + 8 == qm ? cb : sb;
                    wm = kk == qm ? w[kk] : (kk + 8 == qm ? w[kk + 8] : wm);
                    const bool ra = kk == qa, rb = kk + 8 == qa;
                    ca = crc4(ra ? 0u : ca, ra ? (w[kk] & amask) : w[kk], K);
                    cb = crc4(rb ? 0u : cb, rb ? (w[kk + 8] & amask) : w[kk + 8], K);
                }
                sa = qm == 8 ? ca : sa;
                sb = qm == 16 ? cb : sb;
            }
            // the piece of the value crossing the unit end: A pushed through B's 32 bytes, then B
            // (A does not count when that value starts in B's half); the raw CRC of the unit's
            // first 4 qm bytes: A's snapshot, or all of A pushed through 4 (qm - 8) bytes, then B's
            const uint32_t pa = kmul(ca, S.KQ + 128 * 8);
            const uint32_t ps = kmul(ca, S.KQ + 128 * (qm > 8 ? qm - 8 : 0));
            const uint32_t c = qa >= 8 ? cb : (pa ^ cb);
            const uint32_t snap = qm <= 8 ? sa : (ps ^ sb);
            KVR_STAMP(9);
            uint32_t v = 0, f = 1;               // segment start f: no inflow from the previous unit
            if (vx) {
                if (a_off >= 0) v = c ^ S.IX[SC - a_off];
                else if (lane == 0 && vx_carry) v = c ^ kmul(c_state, S.KT);   // carried register across unit 0
                else { v = c; f = 0; }
            }
            // segmented scan: state at the end of unit l = f ? v : state(l-1) * x^(8*64) ^ v
#define KVR_SCAN_ROW(CTRL, D, KTAB)                                          \
            {                                                                \
                const uint32_t ov = dpp<CTRL>(v), of = dpp<CTRL>(f);         \
                const uint32_t t_ = kmul(ov, KTAB);                          \
                const bool ok = (lane & 15) >= (D) && !f;                    \
                v = ok ? (v ^ t_) : v;                                       \
                f = ok ? of : f;                                             \
            }
            KVR_SCAN_ROW(0x111, 1, S.KT)
            KVR_SCAN_ROW(0x112, 2, S.KT + 128)
            KVR_SCAN_ROW(0x114, 4, S.KT + 256)
            KVR_SCAN_ROW(0x118, 8, S.KT + 384)
#undef KVR_SCAN_ROW
            {   // rows 1 and 3 take the end of rows 0 and 2 (lane 15, 47): distance (l & 15) + 1 units
                const uint32_t ov = dpp<0x142, 0xA, false>(v), of = dpp<0x142, 0xA, false>(f);
                const uint32_t t_ = kmulr(ov, S.KR, (uint32_t)(lane & 15));
                const bool ok = (lane & 16) != 0 && !f;
                v = ok ? (v ^ t_) : v;
                f = ok ? of : f;
            }
            {   // rows 2 and 3 take the end of row 1 (lane 31): distance (l & 31) + 1 units
                const uint32_t ov = dpp<0x143, 0xC, false>(v);
                const uint32_t t_ = kmulr(ov, S.KR, (uint32_t)(lane & 31));
                const bool ok = lane >= 32 && !f;
                v = ok ? (v ^ t_) : v;
            }
            KVR_STAMP(10);
            uint32_t sin = dpp<0x138>(v);        // wave_shr:1: the state at this unit's start
            if (lane == 0) sin = c_state;
            // the value ending in this unit at m: its register is sin * x^(8m) ^ raw[0, m)
            // (the x^(8m) push: a constant table for 4q bytes + r zero bytes)
            if (m != 0) {
                const int r = m & 3;
                uint32_t rp = snap, cf = kmul(sin, S.KQ + 128 * qm);
                for (int b = 0; b < r; ++b) {
                    rp = crc1(rp, (wm >> (8 * b)) & 255u, K);
                    cf = crc1(cf, 0u, K);
                }
                if (m_slot < pool_cap) pool[m_slot].crc32 = ~(cf ^ rp);
            }
            if (out) {                           // the value running past the tile: hand over its register
                n_carry = 1;
                n_state = rl32(v, 63);
                n_ve = out_ve;
                n_idx = out_slot;
            }
        }

        KVR_STAMP(3);
        // ---- bookkeeping ------------------------------------------------------------------
        if (in_stripe) {
            if (lane == 0) {
                tres[sg.tile0 + k].pool_off = nrec ? pool_base : 0ull;
                tres[sg.tile0 + k].count = nrec;
            }
            total += nrec;
            if (walk) entry = tile_exit;
        }
        carry = n_carry;
        c_state = n_state;
        c_vb = n_vb; c_ve = n_ve; c_idx = n_idx;
        if (err_pos != NONE) stop = 1;
        else if (walk && tile_exit == ERRP) {   // defensive: a broken chain must have reported
            stop = 1; err_pos = entry; err_kind = KVR_E_VAL;
        }
        wsync();
        KVR_STAMP(4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain an unused prefetch before exit
#ifdef KVR_PROF
    if (lane == 0)
        for (int i = 0; i < 16; ++i) atomicAdd(&g_prof[i], prof_acc[i]);
#endif
    // tiles of the stripe that were never reached (error stop / pass-through) hold no tuples
    const uint32_t kfirst = k < sd.t_end ? k : sd.t_end;
    for (uint32_t kk = kfirst + lane; kk < sd.t_end; kk += 64) {
        tres[sg.tile0 + kk].pool_off = 0;
        tres[sg.tile0 + kk].count = 0;
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

}  // namespace kvr
