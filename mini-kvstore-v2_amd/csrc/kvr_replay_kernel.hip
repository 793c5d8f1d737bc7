/*
 * kvr_replay_kernel.hip — k_replay, the hot path (gfx950).
 *
 * One WAVE replays one stripe (consecutive 4-KiB tiles of one segment) exactly as
 * src/store/engine.rs:79-154 walks a segment file, and emits one 32-B kvr_tuple per record with
 * the CRC-32 of its key and value (crc32fast::hash semantics, src/volume/storage.rs:27).
 * A workgroup holds 4 independent stripes; after the CRC tables are staged in LDS there is no
 * workgroup barrier at all, so a wave waiting on a header hop or on HBM never holds up another.
 *
 * Per tile, lane l owns the 64-B unit [64 l, 64 l + 64):
 *   load  the unit arrives in registers (prefetched one tile ahead with 16-B global loads) and is
 *         written to the wave's LDS tile for random access; the next 256 B (halo) come by LDS-DMA
 *   F     framing: the record starts, exactly, from the tile entry (the previous tile's exit).
 *         Sparse tiles: all lanes hop header to header together (LDS broadcast reads), lane j
 *         keeps record j.  Dense tiles (or past 64 records): every lane speculates a chain through
 *         its unit and the wave stitches the sub-chains by pointer jumping.  The stripe's first
 *         tile takes its first plausible record start; k_link verifies it.
 *   R     records: engine.rs checks in engine.rs order, key CRC, CRC of values <= 64 B, tuple.
 *         Longer values register the first unit boundary they cross.
 *   C     long values: each lane CRCs, from its registers, its unit's piece of the value crossing
 *         the unit's end; a 6-step segmented scan across the wave (multipliers are the constants
 *         x^(8*64*2^j)) gives the CRC register at every unit boundary; the lane holding a value's
 *         last byte finishes that CRC.  A value running past the tile hands its register to the
 *         next tile of the stripe (walked in order), so no variable GF(2) multiply is needed.
 */
#include "kvr_device.h"

namespace kvr {

constexpr int WPB = NT / 64;              // stripes (waves) per workgroup
constexpr int UNITS = TILE / SC;          // 64 units per tile = one per lane
static_assert(UNITS == 64, "one 64-B unit per lane");
constexpr uint16_t N16 = 0xFFFFu;
constexpr uint32_t N32 = 0xFFFFFFFFu;
constexpr uint32_t X_BEYOND = 0xFFFFFFFEu, X_ERR = 0xFFFFFFFFu;
constexpr uint64_t BEYOND = ~0ull - 2;    // record end not readable from the tile (>= tile end)
constexpr int T_END = 64, T_ERR = 65, T_MM = 66;
constexpr uint32_t POOL_CHUNK = 2048;
constexpr uint32_t HOP_MAX = 64;          // records found by hopping (one per lane)
constexpr uint32_t DENSE = 48;            // previous tile's records above which we speculate at once
constexpr int MAXLONG = UNITS + 2;        // long values touching a tile (one per first-crossed boundary + pending)
constexpr int32_t VNONE = -1, VCARRY = -2;
constexpr int32_t FAR = 1 << 30;          // "ends beyond the tile" (tile-relative clamp)

struct WaveLds {                          // one stripe's scratch
    uint8_t  tile[TILE + HALO];
    uint32_t sc_exit[UNITS];
    uint16_t sc_cand[UNITS], sc_cnt[UNITS], sc_last[UNITS];
    uint8_t  reach[UNITS];
    int32_t  lvb[MAXLONG], lve[MAXLONG];
    uint32_t lidx[MAXLONG];
    uint32_t bkey[UNITS + 1];
    uint32_t nlong, pad[3];
};

struct __align__(16) Smem {
    uint32_t T[4 * 256];                  // slice-by-4 byte tables
    uint32_t KT[6 * 8 * 16];              // [j][nibble i][n]: (n << 4i) * x^(8*64*2^j)
    uint32_t KQ[17 * 8 * 16];             // [q][nibble i][n]: (n << 4i) * x^(8*4q)
    uint32_t IX[68];                      // 0xFFFFFFFF * x^(8j): initial register pushed through j bytes
    WaveLds w[WPB];
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

// ---------------------------------------------------------------------------------------
// CRC primitives on the LDS tables
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t crc4(uint32_t c, uint32_t w, const uint32_t *T) {
    c ^= w;
    return T[768 + (c & 255u)] ^ T[512 + ((c >> 8) & 255u)] ^ T[256 + ((c >> 16) & 255u)] ^ T[c >> 24];
}

__device__ __forceinline__ uint32_t crc1(uint32_t c, uint32_t b, const uint32_t *T) {
    return (c >> 8) ^ T[(c ^ b) & 255u];
}

// register state v times the constant x^(8*64*2^j): K = KT + 128 j
__device__ __forceinline__ uint32_t kmul(uint32_t v, const uint32_t *K) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= K[i * 16 + ((v >> (4 * i)) & 15u)];
    return r;
}

// CRC register update over segment bytes [p, p+n): LDS when resident (tile + halo), HBM otherwise
__device__ inline uint32_t crc_range(const TileView &tv, uint32_t c, uint64_t p, uint64_t n, const uint32_t *T) {
    if (tv.in_lds(p, n)) {
        int off = (int)((int64_t)p - tv.lo);
        const int end = off + (int)n;
        #pragma unroll 1
        while (off < end && (off & 3)) { c = crc1(c, tv.lds[off], T); ++off; }
        const uint32_t *w = reinterpret_cast<const uint32_t *>(tv.lds);
        #pragma unroll 1
        while (off + 4 <= end) { c = crc4(c, w[off >> 2], T); off += 4; }
        #pragma unroll 1
        while (off < end) { c = crc1(c, tv.lds[off], T); ++off; }
        return c;
    }
    #pragma unroll 1
    for (uint64_t i = 0; i < n; ++i) c = crc1(c, tv.rd8(p + i), T);
    return c;
}

// ---------------------------------------------------------------------------------------
// speculative framing inside the tile (LDS only)
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
// Heuristic only: a true record rejected here (a key holding NUL) is found again by the exact
// chain walk or by the stripe link check, so results never depend on it.
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

// Walk from p while p < pe: records walked (a record whose framing fails counts: its parse
// reports the error), last record start, exit offset (X_BEYOND / X_ERR)
__device__ inline uint32_t walk_spec(const TileView &tv, uint64_t p, uint64_t pe, uint32_t *exit_off,
                                     uint16_t *last_off) {
    uint32_t cnt = 0;
    uint16_t last = N16;
    uint32_t x;
    for (;;) {
        if (p >= pe) {
            const uint64_t r = p - (uint64_t)tv.lo;
            x = r < (uint64_t)X_BEYOND ? (uint32_t)r : X_BEYOND;
            break;
        }
        const uint64_t nx = next_spec(tv, p);
        ++cnt;
        last = (uint16_t)((int64_t)p - tv.lo);
        if (nx == ERRP) { x = X_ERR; break; }
        if (nx == BEYOND) { x = X_BEYOND; break; }
        p = nx;
    }
    *exit_off = x;
    *last_off = last;
    return cnt;
}

// lane 0: the true chain enters the unit holding y at y; re-walk it and the following units
// whose speculation disagrees with the true chain (bounded per call)
__device__ void repair(WaveLds &W, const TileView &tv, uint64_t y, uint64_t vhi) {
    const int64_t lo = tv.lo;
    for (int k = 0; k < UNITS; ++k) {
        const int t = (int)(((int64_t)y - lo) / SC);
        const int64_t ce = lo + (int64_t)(t + 1) * SC;
        const uint64_t pe = (uint64_t)ce > vhi ? vhi : (uint64_t)ce;
        uint32_t x;
        uint16_t last;
        const uint32_t cnt = walk_spec(tv, y, pe, &x, &last);
        W.sc_cand[t] = (uint16_t)((int64_t)y - lo);
        W.sc_exit[t] = x;
        W.sc_cnt[t] = (uint16_t)cnt;
        W.sc_last[t] = last;
        if (x >= X_BEYOND || lo + (int64_t)x >= (int64_t)vhi) return;
        if (W.sc_cand[x / SC] == x) return;        // back in step with the speculation
        y = (uint64_t)(lo + (int64_t)x);
    }
}

struct Stitched { uint16_t ent; uint32_t cnt, base, total; uint64_t exit; };

// Stitch the per-unit chains from the exact position e (vlo <= e < vhi) by pointer jumping:
// per lane its unit's entry on the true chain (or N16) and record count/base; the tile exit.
__device__ __noinline__ Stitched stitch(WaveLds &W, const TileView tv, uint64_t e, uint64_t vhi, Counters *ctr) {
    const int lane = threadIdx.x & 63;
    const int64_t lo = tv.lo;
    const int s0 = (int)(((int64_t)e - lo) / SC);
    const uint16_t e_off = (uint16_t)((int64_t)e - lo);
    const uint32_t vhi_off = (uint32_t)((int64_t)vhi - lo);
    Stitched R;
    for (int guard = 0; guard < 2 * UNITS + 8; ++guard) {
        if (W.sc_cand[s0] != e_off) {
            if (lane == 0) repair(W, tv, e, vhi);
            wsync();
            continue;
        }
        const uint16_t c = W.sc_cand[lane];
        const uint32_t x = W.sc_exit[lane];
        int T;
        if (c == N16) T = T_END;
        else if (x == X_ERR) T = T_ERR;
        else if (x >= vhi_off) T = T_END;              // includes X_BEYOND
        else { const int t = (int)(x / SC); T = (W.sc_cand[t] == x) ? t : T_MM; }
        W.reach[lane] = lane == s0 ? 1 : 0;
        wsync();
        int J = T;
        bool reach = lane == s0;
        for (int r = 0; r < 7 && __any(J < UNITS); ++r) {   // J <- J o J, reach <- reach U J(reach)
            if (J < UNITS && reach) W.reach[J] = 1;
            const int jn = J < UNITS ? __shfl(J, J, 64) : J;
            wsync();
            reach = W.reach[lane] != 0;
            J = jn;
        }
        const unsigned long long rm = __ballot(reach);
        const int smax = 63 - __builtin_clzll(rm);
        const int Tl = (int)rl32((uint32_t)T, smax);
        const uint32_t xs = rl32(x, smax);
        if (Tl == T_MM) {
            if (lane == 0) repair(W, tv, (uint64_t)(lo + (int64_t)xs), vhi);
            wsync();
            continue;
        }
        R.ent = reach ? c : N16;
        R.cnt = reach ? W.sc_cnt[lane] : 0u;
        uint32_t inc = R.cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            if (lane >= d) inc += o;
        }
        R.base = inc - R.cnt;
        R.total = rl32(inc, 63);
        uint64_t xe;
        if (Tl == T_ERR) xe = ERRP;
        else if (xs != X_BEYOND) xe = (uint64_t)(lo + (int64_t)xs);
        else xe = next_rec(tv, (uint64_t)(lo + (int64_t)W.sc_last[smax]));   // exact, halo / HBM
        R.exit = uni64(xe);
        return R;
    }
    if (lane == 0) atomicOr(&ctr->overflow, 2u);   // unreachable: every round repairs one more unit (bug trap)
    R.ent = N16; R.cnt = 0; R.base = 0; R.total = 0; R.exit = ERRP;
    return R;
}

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------

// ---------------------------------------------------------------------------------------
// 48 bytes of the tile + halo starting at any byte offset off (off + 52 <= TILE + HALO):
// 13 aligned dword reads issued together, realigned in registers.
// ---------------------------------------------------------------------------------------
struct Win { uint32_t q[12]; };

__device__ __forceinline__ Win lds_window(const uint8_t *lds, int off) {
    const uint32_t *tw = reinterpret_cast<const uint32_t *>(lds) + (off >> 2);
    const uint32_t sh = (uint32_t)off & 3u;
    uint32_t r[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) r[i] = tw[i];
    Win w;
#pragma unroll
    for (int i = 0; i < 12; ++i) w.q[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
    return w;
}

// the u32 at window byte offset t (t <= 44), t per lane: a select chain over the 12 words
__device__ __forceinline__ uint32_t win_u32(const Win &w, uint32_t t) {
    const uint32_t j = t >> 2, s = t & 3u;
    uint32_t lo = w.q[0], hi = w.q[1];
#pragma unroll
    for (int i = 1; i < 11; ++i) {
        lo = j == (uint32_t)i ? w.q[i] : lo;
        hi = j == (uint32_t)i ? w.q[i + 1] : hi;
    }
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}

// Fast path for the common record shape: header, a key of at most 36 ASCII bytes and the value
// length inside the tile + halo, no error.  Fills the tuple (crc32 of a value <= SMALL still to
// do) and returns true; anything else returns false and takes the general path.
__device__ __forceinline__ bool rec_fast(const TileView &tv, const uint32_t *T, uint64_t p, uint32_t kmax,
                                         kvr_tuple &t, uint64_t &vb, uint64_t &vlen) {
    const int64_t off = (int64_t)p - tv.lo;
    const uint64_t len = tv.len;
    if (off < 0 || off + 52 > TILE + HALO || len - p < 9) return false;
    const Win w = lds_window(tv.lds, (int)off);
    const uint32_t op = w.q[0] & 255u;
    const uint32_t klen = __builtin_amdgcn_alignbyte(w.q[1], w.q[0], 1);
    if (op > 1u || klen > kmax || len - p - 5 < klen) return false;
    // key bytes start at window byte 5: key word i = bytes 5+4i .. 8+4i
    uint32_t bad = 0, c = ~0u, tail = 0;
    const uint32_t nw = (kmax + 3u) >> 2;                                 // wave-uniform trip count
    for (uint32_t i = 0; i < nw; ++i) {
        uint32_t kw = w.q[1];
#pragma unroll
        for (int s = 1; s < 10; ++s) kw = i == (uint32_t)(s - 1) ? __builtin_amdgcn_alignbyte(w.q[s + 1], w.q[s], 1) : kw;
        const uint32_t n = klen > 4u * i ? klen - 4u * i : 0u;           // key bytes in this word
        const uint32_t m = n >= 4u ? ~0u : ((1u << (8 * n)) - 1u);
        bad |= kw & m & 0x80808080u;                                     // non-ASCII: the full check
        const uint32_t cn = crc4(c, kw, T);
        c = n >= 4u ? cn : c;
        tail = (n > 0u && n < 4u) ? kw : tail;
    }
    if (bad) return false;
    for (uint32_t b = 0; b < (klen & 3u); ++b) c = crc1(c, (tail >> (8 * b)) & 255u, T);
    t.rec_off = p;
    t.key_len = klen;
    t.key_tag = ~c;
    t.op = (uint8_t)op;
    t.flags = 0;
    t.reserved = 0;
    t.crc32 = 0;
    t.val_len = 0;
    vb = p + 5 + klen;
    vlen = 0;
    if (op == 0u) {
        if (len - vb < 4) return false;
        vlen = win_u32(w, 5 + klen);
        vb += 4;
        if (len - vb < vlen) return false;
        t.val_len = (uint32_t)vlen;
    }
    return true;
}

// next record start after the record at p (exact, = next_rec): one window read when the header
// and a key of at most 36 bytes sit in the tile + halo; next_rec otherwise
__device__ __forceinline__ uint64_t hop_next(const TileView &tv, uint64_t p) {
    const int64_t off = (int64_t)p - tv.lo;
    const uint64_t len = tv.len;
    if (off >= 0 && off + 52 <= TILE + HALO && len - p >= 9) {
        const Win w = lds_window(tv.lds, (int)off);
        const uint32_t op = w.q[0] & 255u;
        const uint32_t klen = __builtin_amdgcn_alignbyte(w.q[1], w.q[0], 1);
        if (op <= 1u && klen <= 36u) {
            const uint64_t e = p + 5 + klen;
            if (e > len) return ERRP;
            if (op == 1u) return e;
            if (len - e < 4) return ERRP;
            const uint64_t e2 = e + 4 + (uint64_t)win_u32(w, 5 + klen);
            return e2 > len ? ERRP : e2;
        }
    }
    return next_rec(tv, p);
}

struct RecRes {          // one record's outcome
    uint32_t err, kind;  // record index of an error (N32: none) and its KVR_E_* kind
    uint64_t aux;
    uint32_t hand;       // 1: its long value crosses the tile end, 2: its value starts in a later tile
    uint64_t vb, ve, slot;
    uint32_t klen;       // key length (fast-path sizing for the next tile)
};

// parse + emit the record at p (engine.rs order of checks); long values register with the tile
__device__ __forceinline__ RecRes do_record(const TileView &tv, WaveLds &W, const uint32_t *T, uint64_t p, uint32_t j,
                                         uint64_t slot, uint32_t seg, kvr_tuple *pool, uint64_t pool_cap,
                                         uint32_t kmax) {
    RecRes ro;
    ro.err = N32; ro.kind = 0; ro.aux = 0; ro.hand = 0; ro.vb = 0; ro.ve = 0; ro.slot = slot; ro.klen = 0;
    {
        kvr_tuple t;
        uint64_t vb, vlen;
        if (rec_fast(tv, T, p, kmax, t, vb, vlen)) {
            t.seg_idx = seg;
            ro.klen = t.key_len;
            if (t.op == 0u) {
                if (vlen <= (uint64_t)SMALL) {
                    t.crc32 = ~crc_range(tv, ~0u, vb, vlen, T);
                } else {
                    const uint64_t ve = vb + vlen;
                    const int64_t vbr = (int64_t)vb - tv.lo, ver = (int64_t)ve - tv.lo;
                    if (vbr < TILE) {
                        const uint32_t L = atomicAdd(&W.nlong, 1u);
                        W.lvb[L] = (int32_t)vbr;
                        W.lve[L] = ver > FAR ? FAR : (int32_t)ver;
                        W.lidx[L] = (uint32_t)slot;
                        W.bkey[vbr / SC + 1] = ((uint32_t)(vbr + 1) << 7) | L;
                        if (ver > TILE) { ro.hand = 1; ro.vb = vb; ro.ve = ve; }
                    } else {
                        ro.hand = 2; ro.vb = vb; ro.ve = ve;
                    }
                }
            }
            if (slot < pool_cap) pool[slot] = t;
            return ro;
        }
    }
    const uint64_t len = tv.len;
    const int64_t lo = tv.lo;
    const uint32_t op = tv.rd8(p);
    if (len - p < 5) { ro.err = j; ro.kind = KVR_E_KEY_LEN; return ro; }                 // engine.rs:96
    const uint64_t klen = tv.rd32(p + 1);
    const uint64_t kb = p + 5;
    ro.klen = klen > 36u ? 36u : (uint32_t)klen;
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
    t.key_tag = ~crc_range(tv, ~0u, kb, klen, T);
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
            t.crc32 = ~crc_range(tv, ~0u, vb, vlen, T);
        } else {
            const int64_t vbr = (int64_t)vb - lo, ver = (int64_t)ve - lo;
            if (vbr < TILE) {
                const uint32_t L = atomicAdd(&W.nlong, 1u);
                W.lvb[L] = (int32_t)vbr;
                W.lve[L] = ver > FAR ? FAR : (int32_t)ver;
                W.lidx[L] = (uint32_t)slot;
                W.bkey[vbr / SC + 1] = ((uint32_t)(vbr + 1) << 7) | L;
                if (ver > TILE) { ro.hand = 1; ro.vb = vb; ro.ve = ve; }   // runs past the tile
            } else {                       // the value starts in a later tile
                ro.hand = 2; ro.vb = vb; ro.ve = ve;
            }
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

__global__ __launch_bounds__(NT, 3) void k_replay(const SegDesc *__restrict__ segs,
                                               const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                               StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                               kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                               Tables tb, const RedoEnt *__restrict__ redo,
                                               const LinkResult *__restrict__ link, int redo_mode,
                                               uint32_t pool_chunk) {
    __shared__ Smem S;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 4 * 256; i += NT) S.T[i] = tb.crc8[i];
    for (int i = tid; i < 6 * 8 * 16; i += NT) S.KT[i] = tb.kmul[i];
    for (int i = tid; i < 17 * 8 * 16; i += NT) S.KQ[i] = tb.kmul[8 * 8 * 16 + i];
    if (tid < 65) S.IX[tid] = tb.initx[tid];
    __syncthreads();   // the only workgroup barrier: from here on every wave is on its own

    const uint32_t gw = blockIdx.x * WPB + wv;
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
    uint32_t err_kind = 0, total = 0, prev_n = 0, kmax = 36;   // kmax: key bytes the record fast path takes
    uint64_t chunk_base = 0, chunk_left = 0;
    uint32_t carry = 0, c_state = 0;      // 1: a long value crosses the tile start (c_state valid);
    uint64_t c_vb = 0, c_ve = 0, c_idx = 0;   // 2: pending (its value starts in a later tile)

    uint4 nx0, nx1, nx2, nx3;   // this lane's unit of the next tile (prefetch)
    load_unit(abase, d0, len, sd.t_begin, lane, nx0, nx1, nx2, nx3);
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
            load_unit(abase, d0, len, k, lane, nx0, nx1, nx2, nx3);
            load_halo(abase, d0, len, k, lane, W.tile);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        {
            uint4 *tp = reinterpret_cast<uint4 *>(W.tile + lane * SC);
            tp[0] = nx0; tp[1] = nx1; tp[2] = nx2; tp[3] = nx3;
        }
        loaded = (k + 1 < sg.n_tiles) && (k + 1 < sd.t_end || carry);
        if (loaded) load_unit(abase, d0, len, k + 1, lane, nx0, nx1, nx2, nx3);
        if (lane == 0) W.nlong = 0;
        W.bkey[lane + 1] = 0u;
        wsync();

        const int64_t lo = (int64_t)k * TILE - d0;
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        const TileView tv{sg.base, W.tile, len, lo};
        const int64_t cs_i = lo + (int64_t)lane * SC;
        const uint64_t cs = cs_i < (int64_t)vlo ? vlo : (uint64_t)cs_i;
        const uint64_t ce = (uint64_t)(cs_i + SC) > vhi ? vhi : (uint64_t)(cs_i + SC);

        KVR_STAMP(0);
        // ---- F. framing ------------------------------------------------------------------------
        if (in_stripe && search) {   // the stripe's entry: the first plausible record start
            const uint64_t cand = cs < ce ? find_cand(tv, cs, ce) : NONE;
            uint64_t m = cand;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const uint64_t o = __shfl_xor(m, d, 64);
                m = o < m ? o : m;
            }
            m = uni64(m);
            if (m != NONE) { entry = m; search = false; stripe_entry = m; }
        }
        const bool walk = in_stripe && !search && entry < vhi;
        uint64_t tile_exit = entry;
        uint32_t n_hop = 0, myrec = N32;
        Stitched st;
        st.ent = N16; st.cnt = 0; st.base = 0; st.total = 0;
        if (walk) {
            uint64_t p = entry;
            if (KVR_ABLATE & 4) { n_hop = 0; p = vhi; }
            else if (prev_n <= DENSE) {   // exact hops, all lanes together (LDS broadcast reads)
                while (p < vhi && n_hop < HOP_MAX) {
                    if (lane == (int)n_hop) myrec = (uint32_t)((int64_t)p - lo);
                    ++n_hop;
                    p = uni64(hop_next(tv, p));
                    if (p == ERRP) break;
                }
            }
            tile_exit = p;
            if (p != ERRP && p < vhi) {   // dense: speculate per unit from the exact position p
                uint16_t cand16 = N16, last16 = N16;
                uint32_t x = X_BEYOND, cnt = 0;
                const uint64_t p0 = cs > p ? cs : p;
                if (p0 < ce) {
                    const uint64_t cand = find_cand(tv, p0, ce);
                    if (cand != NONE) {
                        cand16 = (uint16_t)((int64_t)cand - lo);
                        cnt = walk_spec(tv, cand, ce, &x, &last16);
                    }
                }
                W.sc_cand[lane] = cand16;
                W.sc_exit[lane] = x;
                W.sc_cnt[lane] = (uint16_t)cnt;
                W.sc_last[lane] = last16;
                wsync();
                st = stitch(W, tv, p, vhi, ctr);
                tile_exit = st.exit;
            }
        }
        const uint32_t nrec = n_hop + st.total;
        // pool slots for this tile's records (bulk chunks)
        if (nrec > chunk_left) {
            const uint64_t m = nrec > pool_chunk ? nrec : pool_chunk;
            unsigned long long b = 0;
            if (lane == 0) {
                b = atomicAdd(&ctr->pool_cursor, (unsigned long long)m);
                if (b + m > pool_cap) atomicOr(&ctr->overflow, 1u);
            }
            chunk_base = uni64(b);
            chunk_left = m;
        }
        const uint64_t pool_base = chunk_base;
        chunk_base += nrec;
        chunk_left -= nrec;
        // a value whose record started in an earlier tile begins in this one: register it
        uint32_t n_carry = 0;
        uint64_t n_vb = 0, n_ve = 0, n_idx = 0;
        if (carry == 2u) {
            if ((int64_t)c_vb - lo < TILE) {
                if (lane == 0) {
                    const int32_t pvb = (int32_t)((int64_t)c_vb - lo);
                    const int64_t ve = (int64_t)c_ve - lo;
                    W.lvb[0] = pvb;
                    W.lve[0] = ve > FAR ? FAR : (int32_t)ve;
                    W.lidx[0] = (uint32_t)c_idx;
                    W.bkey[pvb / SC + 1] = (uint32_t)(pvb + 1) << 7;
                    W.nlong = 1;
                }
                carry = 0;
                n_vb = c_vb; n_ve = c_ve; n_idx = c_idx;   // in case it also runs past this tile
            } else {                        // still further on: hand it over untouched
                n_carry = 2; n_vb = c_vb; n_ve = c_ve; n_idx = c_idx;
            }
        }
        wsync();

        KVR_STAMP(1);
        // ---- R. records ----------------------------------------------------------------------
        RecRes ro;
        ro.err = N32; ro.kind = 0; ro.aux = 0; ro.hand = 0; ro.vb = 0; ro.ve = 0; ro.slot = 0; ro.klen = 0;
        uint32_t my_kmax = 0;
        uint32_t hand = 0;
        uint64_t pvb = 0, pve = 0, pidx = 0;
        {   // this lane's records: its hop record (record index = lane), then its unit's speculated ones
            const uint32_t has_hop = myrec != N32 ? 1u : 0u;
            const uint32_t nmine = (KVR_ABLATE & 1) ? 0u : has_hop + (st.ent != N16 ? st.cnt : 0u);
            uint64_t ps = (uint64_t)(lo + (int64_t)st.ent);
            for (uint32_t i = 0; i < nmine; ++i) {
                const bool h = i < has_hop;
                const uint64_t p = h ? (uint64_t)(lo + (int64_t)myrec) : ps;
                const uint32_t j = h ? (uint32_t)lane : n_hop + st.base + (i - has_hop);
                ro = do_record(tv, W, S.T, p, j, pool_base + j, sd.seg, pool, pool_cap, kmax);
                if (ro.hand) { hand = ro.hand; pvb = ro.vb; pve = ro.ve; pidx = ro.slot; }
                my_kmax = ro.klen > my_kmax ? ro.klen : my_kmax;
                if (ro.err != N32) break;
                if (!h && i + 1 < nmine) ps = next_spec(tv, ps);
            }
        }
        KVR_STAMP(6);
        // first error of the tile (lowest record index); longest key (fast-path bound of the next tile)
        uint32_t err_rec = N32;
        if (__ballot(ro.err != N32)) {
            err_rec = ro.err;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const uint32_t o = __shfl_xor(err_rec, d, 64);
                err_rec = o < err_rec ? o : err_rec;
            }
            err_rec = uni32(err_rec);
        }
        if (nrec && ((k - sd.t_begin) & 15u) == 0u) {   // refresh the fast path's key bound now and then
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const uint32_t ok = __shfl_xor(my_kmax, d, 64);
                my_kmax = ok > my_kmax ? ok : my_kmax;
            }
            kmax = uni32(my_kmax) < 4u ? 4u : uni32(my_kmax);
        } else if (__ballot(my_kmax > kmax)) {
            kmax = 36u;                                  // a longer key appeared: widen at once
        }
        if (err_rec != N32) {
            const int el = __builtin_ctzll(__ballot(ro.err == err_rec));
            err_kind = rl32(ro.kind, el);
            err_aux = rl64(ro.aux, el);
            // the failing record's start: hop records live in myrec, speculated ones are re-found
            uint64_t ep = NONE;
            if (ro.err == err_rec) {
                if (err_rec < n_hop) ep = (uint64_t)(lo + (int64_t)myrec);
                else {
                    uint64_t p = (uint64_t)(lo + (int64_t)st.ent);
                    for (uint32_t i = n_hop + st.base; i < err_rec; ++i) p = next_spec(tv, p);
                    ep = p;
                }
            }
            err_pos = rl64(ep, el);
        }
        KVR_STAMP(7);
        // a long value crossing the tile end / starting later (one at most): its lane hands it over
        {
            const unsigned long long bp = __ballot(hand == 2u), bc = __ballot(hand == 1u);
            if (bp | bc) {
                const int ol = __builtin_ctzll(bp | bc);
                n_vb = rl64(pvb, ol);
                n_ve = rl64(pve, ol);
                n_idx = rl64(pidx, ol);
                if (bp) n_carry = 2;
            }
        }
        wsync();
        if (loaded) load_halo(abase, d0, len, k + 1, lane, W.tile);   // this tile's halo reads are done

        KVR_STAMP(2);
        // ---- C. CRC of long values --------------------------------------------------------
        const uint32_t nlong = uni32(W.nlong);
        if (!(KVR_ABLATE & 2) && (nlong != 0u || carry == 1u)) {
            // which value crosses the end of this lane's unit: latest long value starting before
            // it (prefix max of boundary keys), if it reaches past it
            uint32_t key = W.bkey[lane + 1];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(key, d, 64);
                if (lane >= d && o > key) key = o;
            }
            const int32_t pb = SC * (lane + 1);
            int32_t Vend = VNONE;
            if (key != 0u) {
                const int32_t L = (int32_t)(key & 127u);
                if (W.lve[L] > pb) Vend = L;
            } else if (carry == 1u && (int64_t)c_ve - lo > (int64_t)pb) {
                Vend = VCARRY;
            }
            KVR_STAMP(8);
            int32_t Vst = __shfl_up(Vend, 1, 64);
            if (lane == 0) Vst = carry == 1u ? VCARRY : VNONE;
            const int32_t us = SC * lane;
            const uint4 *up = reinterpret_cast<const uint4 *>(W.tile + us);   // this lane's unit
            const uint4 cu0 = up[0], cu1 = up[1], cu2 = up[2], cu3 = up[3];
            const uint32_t w[16] = {cu0.x, cu0.y, cu0.z, cu0.w, cu1.x, cu1.y, cu1.z, cu1.w,
                                    cu2.x, cu2.y, cu2.z, cu2.w, cu3.x, cu3.y, cu3.z, cu3.w};
            // One pass over the unit's bytes gives both register pieces this lane owns:
            //  - raw CRC of [0, m) (bytes of the value crossing the unit start, if it ends here at m),
            //    snapshotted on the way, and
            //  - raw CRC of [a, 64) (the value crossing the unit end; a > 0 if it starts here), by
            //    restarting the register at a's word with the bytes before a zeroed.
            int32_t m = 0;                               // 1 .. 64 if the start-crossing value ends here
            if (Vst != VNONE) {
                const int64_t ve_rel = Vst == VCARRY ? (int64_t)c_ve - lo : (int64_t)W.lve[Vst];
                if (ve_rel <= (int64_t)us + SC) m = (int32_t)(ve_rel - us);
            }
            int32_t a = 0;
            bool starts = false;
            if (Vend >= 0 && W.lvb[Vend] >= us) { a = W.lvb[Vend] - us; starts = true; }
            const int qm = m >> 2, qa = starts ? (a >> 2) : -1;
            uint32_t c = 0, snap = 0, wm = 0;
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                snap = kk == qm ? c : snap;
                wm = kk == qm ? w[kk] : wm;
                c = kk == qa ? 0u : c;
                const int sh = kk == qa ? 8 * (a & 3) : 0;   // bytes of a's word before a are zeroed
                c = crc4(c, w[kk] & (~0u << sh), S.T);
            }
            snap = qm == 16 ? c : snap;
            KVR_STAMP(9);
            uint32_t v = 0, f = 1;
            if (Vend != VNONE) {
                if (starts) v = c ^ S.IX[SC - a];
                else if (lane == 0) v = c ^ kmul(c_state, S.KT);   // the carried register across unit 0
                else { v = c; f = 0; }
            }
            // segmented scan across the wave: state at boundary s+1 = f ? v : state(s) * X(64) ^ v
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int d = 1 << j;
                const uint32_t ov = __shfl_up(v, d, 64);
                const uint32_t of = __shfl_up(f, d, 64);
                if (lane >= d && !f) { v ^= kmul(ov, S.KT + 128 * j); f = of; }
            }
            KVR_STAMP(10);
            uint32_t sin = __shfl_up(v, 1, 64);
            if (lane == 0) sin = c_state;
            // the value crossing the unit's start ends in this unit at m: its register is
            // sin * x^(8m) ^ raw[0, m)  (the x^(8m) push: a constant table for 4q bytes + r zero bytes)
            if (m != 0) {
                const int r = m & 3;
                uint32_t rp = snap, cf = kmul(sin, S.KQ + 128 * qm);
                for (int b = 0; b < r; ++b) {
                    rp = crc1(rp, (wm >> (8 * b)) & 255u, S.T);
                    cf = crc1(cf, 0u, S.T);
                }
                const uint64_t idx = Vst == VCARRY ? c_idx : (uint64_t)W.lidx[Vst];
                if (idx < pool_cap) pool[idx].crc32 = ~(cf ^ rp);
            }
            // a value running past the tile: hand over its register state
            const int32_t Vo = (int32_t)rl32((uint32_t)Vend, 63);
            if (Vo != VNONE) {
                n_carry = 1;
                c_state = rl32(v, 63);
                if (Vo == VCARRY) { n_vb = c_vb; n_ve = c_ve; n_idx = c_idx; }
            }
        }

        KVR_STAMP(3);
        // ---- bookkeeping ------------------------------------------------------------------
        if (in_stripe) {
            const uint32_t n_ok = err_rec < nrec ? err_rec : nrec;
            if (lane == 0) {
                tres[sg.tile0 + k].pool_off = n_ok ? pool_base : 0ull;
                tres[sg.tile0 + k].count = n_ok;
            }
            total += n_ok;
            if (walk) entry = tile_exit;
            prev_n = nrec;
        }
        carry = n_carry;
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
