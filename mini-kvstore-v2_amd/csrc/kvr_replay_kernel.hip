/*
 * kvr_replay_kernel.hip — k_replay, the hot path (gfx950).
 *
 * One workgroup replays one stripe (consecutive tiles of one segment) exactly as
 * src/store/engine.rs:79-154 walks a segment file, and emits one 32-B kvr_tuple per record with
 * the CRC-32 of its key and value (crc32fast::hash semantics, src/volume/storage.rs:27).
 *
 * Per 16-KiB tile (geometry in kvr_device.h), with the next tile's LDS-DMA in flight:
 *   F  framing: the record starts of the tile, exactly, from the tile entry (the previous
 *      tile's exit).  Sparse tiles: lane 0 hops header to header (a few LDS round trips per
 *      record).  Dense tiles (or after HOP_BUDGET hops): every thread speculates a record chain
 *      through its 64-B sub-chunk and wave 0 stitches the sub-chains by pointer jumping.
 *      The stripe's first tile has no known entry: its first plausible record start is taken
 *      and k_link verifies it against the previous stripe's exit.
 *   R  records, one thread per record: engine.rs checks in engine.rs order (key length, key,
 *      UTF-8, opcode, value length, value), key CRC, CRC of values <= SMALL bytes, the tuple.
 *      Longer values register the first 64-B unit boundary they cross.
 *   C  CRC of long values, one thread per 64-B unit: every thread CRCs its unit's piece of the
 *      value crossing the unit's end; a segmented scan over the 256 units (multipliers are the
 *      constants x^(8*64*2^j), nibble tables) turns pieces into register states at every unit
 *      boundary; the thread whose unit holds a value's last byte finishes that CRC from the
 *      state at its unit start.  A value running past the tile hands its register state to the
 *      next tile (the stripe walks its tiles in order), so no variable GF(2) multiply is needed.
 * Barriers are raw s_barrier + lgkmcnt waits so the next tile's LDS-DMA stays in flight.
 */
#include "kvr_device.h"

namespace kvr {

constexpr uint16_t N16 = 0xFFFFu;        // no offset
constexpr uint32_t N32 = 0xFFFFFFFFu;
constexpr uint32_t X_BEYOND = 0xFFFFFFFEu, X_ERR = 0xFFFFFFFFu;
constexpr uint64_t BEYOND = ~0ull - 2;   // record end not readable from the tile (>= tile end)
constexpr int16_t T_END = NT, T_ERR = NT + 1, T_MM = NT + 2;
constexpr uint32_t POOL_CHUNK = 2048;
constexpr int MAXREC = TILE / 5 + 2;     // record starts in one tile (a record is >= 5 B)
constexpr int MAXLONG = NT + 2;          // long values touching a tile: one per first-crossed boundary (+ pending)
constexpr uint32_t HOP_BUDGET = 40;      // exact hops by one lane before switching to speculation
constexpr uint32_t DENSE = 48;           // records in the previous tile above which we speculate at once
constexpr int32_t VNONE = -1, VCARRY = -2;
constexpr int32_t FAR = 1 << 30;         // "ends beyond the tile" (tile-relative clamp)

struct SpecLds {                 // framing speculation (dense tiles)
    uint32_t sc_exit[NT];        // exit offset from lo (X_BEYOND / X_ERR)
    uint32_t sc_base[NT];        // index of the sub-chunk's first record among the speculated ones
    uint16_t sc_cand[NT], sc_last[NT], sc_cnt[NT], sc_entry[NT];
    int16_t  nxt[NT], nxt0[NT];
    uint8_t  reach[NT];
};

struct LongLds {                 // long values of the tile (after framing)
    int32_t  lvb[MAXLONG];       // value start, tile-relative
    int32_t  lve[MAXLONG];       // value end, tile-relative, clamped to FAR
    uint32_t lidx[MAXLONG];      // pool slot of the record's tuple
    uint32_t bkey[NT + 1];       // boundary b: key of the long value whose first crossed boundary is b
    int32_t  vc[NT + 1];         // value crossing boundary b: L, VCARRY or VNONE
};

struct ScanLds {
    uint64_t x[2][NT];           // ping-pong (state | segment flag << 32)
    uint32_t sx[NT];             // inclusive states: register at the end of every unit
};

struct __align__(16) RSmem {
    uint8_t  buf[2][TILE + HALO];
    uint32_t T[4 * 256];         // slice-by-4 CRC tables
    uint32_t KT[8 * 8 * 16];     // [j][nibble i][n]: (n << 4i) * x^(8*64*2^j)
    uint32_t IX[68];             // 0xFFFFFFFF * x^(8j): initial register pushed through j bytes
    union { uint16_t rec[MAXREC]; ScanLds sc; } r;
    union { SpecLds sp; LongLds lg; } u;
    uint32_t wt[4];
    uint64_t entry, tile_exit, err_pos, err_aux, stripe_entry, pool_base, chunk_base, chunk_left;
    uint64_t c_vb, c_ve, c_idx;           // carried long value: 1 = crosses the tile start (c_state
    uint64_t n_vb, n_ve, n_idx;           //   valid), 2 = pending (starts in a later tile); n_* = next tile's
    uint32_t carry, c_state, n_carry, n_state;
    uint32_t err_kind, nrec, nlong, total, search, stop, prev_n, cand_min, need_spec, spec_total, err_rec;
};

#define KVR_BARRIER()                                          \
    do {                                                       \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     \
        __builtin_amdgcn_s_barrier();                          \
        asm volatile("" ::: "memory");                         \
    } while (0)

#ifdef KVR_PROF
__device__ unsigned long long g_prof[16];
#define KVR_STAMP(i)                                                        \
    do {                                                                    \
        if (threadIdx.x == 0) {                                             \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
            atomicAdd(&g_prof[i], t_ - t_last);                             \
            t_last = t_;                                                    \
        }                                                                   \
    } while (0)
#else
#define KVR_STAMP(i) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------
// CRC primitives on the LDS byte tables
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
        while (off < end && (off & 3)) { c = crc1(c, tv.lds[off], T); ++off; }
        const uint32_t *w = reinterpret_cast<const uint32_t *>(tv.lds);
        while (off + 4 <= end) { c = crc4(c, w[off >> 2], T); off += 4; }
        while (off < end) { c = crc1(c, tv.lds[off], T); ++off; }
        return c;
    }
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
__device__ inline uint64_t find_cand(const TileView &tv, uint64_t p0, uint64_t p1) {
    if (p0 >= p1) return NONE;
    const int o0 = (int)((int64_t)p0 - tv.lo), o1 = (int)((int64_t)p1 - tv.lo);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(tv.lds);
    for (int q = o0 >> 2; q <= (o1 - 1) >> 2; ++q) {
        const uint32_t y = w[q] & 0xFEFEFEFEu;                 // bytes 0x00 / 0x01 become 0
        uint32_t z = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
        const int bq = q * 4;
        if (bq < o0) z &= ~0u << (8 * (o0 - bq));
        if (bq + 4 > o1) z &= (1u << (8 * (o1 - bq))) - 1u;
        while (z) {
            const int b = __builtin_ctz(z) >> 3;
            const uint64_t p = (uint64_t)(tv.lo + bq + b);
            if (plausible(tv, p)) return p;
            z &= z - 1u;
        }
    }
    return NONE;
}

// Walk from p while p < pe: records walked, last record start, exit offset (X_BEYOND/X_ERR)
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
        ++cnt;                                     // a record whose framing fails is still one:
        last = (uint16_t)((int64_t)p - tv.lo);     // its parse reports the error
        if (nx == ERRP) { x = X_ERR; break; }
        if (nx == BEYOND) { x = X_BEYOND; break; }
        p = nx;
    }
    *exit_off = x;
    *last_off = last;
    return cnt;
}

// ---------------------------------------------------------------------------------------
// stitching of the speculated sub-chains (wave 0)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int wave_max_i32(int v) {
    for (int d = 32; d >= 1; d >>= 1) {
        const int o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}

// lane 0: the true chain enters the sub-chunk holding y at y; re-walk it and the following
// sub-chunks whose speculation disagrees with the true chain (bounded per call)
__device__ void repair(SpecLds &P, const TileView &tv, uint64_t y, uint64_t vhi) {
    const int64_t lo = tv.lo;
    for (int k = 0; k < 64; ++k) {
        const int t = (int)(((int64_t)y - lo) / SC);
        const int64_t ce = lo + (int64_t)(t + 1) * SC;
        const uint64_t pe = (uint64_t)ce > vhi ? vhi : (uint64_t)ce;
        uint32_t x;
        uint16_t last;
        const uint32_t cnt = walk_spec(tv, y, pe, &x, &last);
        P.sc_cand[t] = (uint16_t)((int64_t)y - lo);
        P.sc_exit[t] = x;
        P.sc_cnt[t] = (uint16_t)cnt;
        P.sc_last[t] = last;
        if (x >= X_BEYOND || lo + (int64_t)x >= (int64_t)vhi) return;
        if (P.sc_cand[x / SC] == x) return;        // back in step with the speculation
        y = (uint64_t)(lo + (int64_t)x);
    }
}

// Stitch from the exact position e (vlo <= e < vhi): publishes sc_entry / sc_base of the
// sub-chunks on the true chain, S.spec_total and S.tile_exit.
__device__ void stitch(RSmem &S, const TileView &tv, uint64_t e, uint64_t vhi, Counters *ctr) {
    SpecLds &P = S.u.sp;
    const int lane = threadIdx.x;
    const int64_t lo = tv.lo;
    const int s0 = (int)(((int64_t)e - lo) / SC);
    const uint16_t e_off = (uint16_t)((int64_t)e - lo);
    const uint32_t vhi_off = (uint32_t)((int64_t)vhi - lo);
    for (int guard = 0; guard < 2 * NT + 8; ++guard) {
        if (P.sc_cand[s0] != e_off) {
            if (lane == 0) repair(P, tv, e, vhi);
            wave_sync_lds();
            continue;
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            const uint16_t c = P.sc_cand[s];
            const uint32_t x = P.sc_exit[s];
            int16_t T;
            if (c == N16) T = T_END;
            else if (x == X_ERR) T = T_ERR;
            else if (x >= vhi_off) T = T_END;          // includes X_BEYOND
            else { const int t = (int)(x / SC); T = (P.sc_cand[t] == x) ? (int16_t)t : T_MM; any = true; }
            P.nxt0[s] = T;
            P.nxt[s] = T;
            P.reach[s] = (s == s0) ? 1 : 0;
        }
        wave_sync_lds();
        for (int r = 0; r < 8 && __any(any); ++r) {   // J <- J o J, reach <- reach U J(reach)
            int16_t jn[4];
            any = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int s = 4 * lane + j;
                const int16_t J = P.nxt[s];
                jn[j] = J < NT ? P.nxt[J] : J;
                any |= jn[j] < NT;
                if (J < NT && P.reach[s]) P.reach[J] = 1;
            }
            wave_sync_lds();
#pragma unroll
            for (int j = 0; j < 4; ++j) P.nxt[4 * lane + j] = jn[j];
            wave_sync_lds();
        }
        int smax = -1;
#pragma unroll
        for (int j = 0; j < 4; ++j) if (P.reach[4 * lane + j]) smax = 4 * lane + j;
        smax = wave_max_i32(smax);
        const int16_t Tl = P.nxt0[smax];
        if (Tl == T_MM) {
            if (lane == 0) repair(P, tv, (uint64_t)(lo + (int64_t)P.sc_exit[smax]), vhi);
            wave_sync_lds();
            continue;
        }
        // accepted path: entries and record index bases
        uint16_t ent[4];
        uint32_t c4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            const bool on = P.reach[s] != 0;
            ent[j] = on ? P.sc_cand[s] : N16;
            c4[j] = on ? P.sc_cnt[s] : 0u;
        }
        const uint32_t tot = c4[0] + c4[1] + c4[2] + c4[3];
        uint32_t inc = tot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            if (lane >= d) inc += o;
        }
        uint32_t base = inc - tot;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            P.sc_entry[s] = ent[j];
            P.sc_base[s] = base;
            base += c4[j];
        }
        const uint32_t total = __shfl(inc, 63, 64);
        if (lane == 0) {
            S.spec_total = total;
            uint64_t x;
            if (Tl == T_ERR) x = ERRP;
            else if (P.sc_exit[smax] != X_BEYOND) x = (uint64_t)(lo + (int64_t)P.sc_exit[smax]);
            else x = next_rec(tv, (uint64_t)(lo + (int64_t)P.sc_last[smax]));   // exact, halo / HBM
            S.tile_exit = x;
        }
        return;
    }
    if (lane == 0) {   // unreachable: every round repairs one more sub-chunk for good (bug trap)
        S.spec_total = 0;
        S.tile_exit = ERRP;
        atomicOr(&ctr->overflow, 2u);
    }
}

// async HBM -> LDS copy of tile k and its halo (16-B LDS-DMA per lane; wave w of instruction i
// lands at byte (i * NT + w * 64) * 16; the halo, the next HALO bytes, lands at TILE)
__device__ __forceinline__ void issue_tile(const SegDesc &sg, uint32_t k, uint8_t *dst) {
    const int tid = threadIdx.x, wave = tid >> 6;
    const int64_t lo = (int64_t)k * TILE - (int64_t)sg.d0;
    const uint8_t *abase = sg.base - sg.d0 + (int64_t)k * TILE;
#pragma unroll
    for (int i = 0; i < TILE / 16 / NT; ++i) {
        const int w = i * NT + tid;
        const int64_t pos = lo + 16 * (int64_t)w;
        if (pos + 16 > 0 && pos < (int64_t)sg.len) {
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void *>(abase + 16 * w),
                reinterpret_cast<__attribute__((address_space(3))) void *>(
                    (__attribute__((address_space(3))) uint8_t *)(dst + (i * NT + wave * 64) * 16)),
                16, 0, 0);
        }
    }
    if (tid < HALO / 16) {
        const int64_t pos = lo + TILE + 16 * (int64_t)tid;
        if (pos < (int64_t)sg.len) {
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void *>(abase + TILE + 16 * tid),
                reinterpret_cast<__attribute__((address_space(3))) void *>(
                    (__attribute__((address_space(3))) uint8_t *)(dst + TILE)),
                16, 0, 0);
        }
    }
}

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT, 3) void k_replay(const SegDesc *__restrict__ segs,
                                                  const StripeDesc *__restrict__ stripes,
                                                  StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                                  kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                                  Tables tb, const RedoEnt *__restrict__ redo,
                                                  const LinkResult *__restrict__ link, int redo_mode,
                                                  uint32_t pool_chunk) {
    __shared__ RSmem S;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t si;
    uint64_t forced = NONE;
    if (redo_mode) {
        if (blockIdx.x >= link->n_redo || link->status != 3) return;
        si = redo[blockIdx.x].stripe;
        forced = redo[blockIdx.x].entry;
    } else {
        si = blockIdx.x;
    }
    const StripeDesc sd = stripes[si];
    const SegDesc sg = segs[sd.seg];
    const uint64_t len = sg.len;
    const int64_t d0 = sg.d0;
    const int64_t shi_i = (int64_t)sd.t_end * TILE - d0;
    const uint64_t s_hi = (uint64_t)shi_i > len ? len : (uint64_t)shi_i;

    for (int i = tid; i < 4 * 256; i += NT) S.T[i] = tb.crc8[i];
    for (int i = tid; i < 8 * 8 * 16; i += NT) S.KT[i] = tb.kmul[i];
    if (tid < 65) S.IX[tid] = tb.initx[tid];
    if (tid == 0) {
        S.carry = 0; S.n_carry = 0;
        S.err_kind = 0; S.err_pos = NONE; S.err_aux = 0; S.err_rec = N32;
        S.total = 0; S.stop = 0; S.prev_n = 0;
        S.chunk_left = 0; S.chunk_base = 0;
        S.nrec = 0; S.need_spec = 0; S.cand_min = N32; S.nlong = 0;
        const uint64_t e = redo_mode ? forced : ((sd.t_begin == 0) ? 0ull : NONE);
        S.search = (e == NONE);
        S.entry = e;
        S.stripe_entry = (e != NONE && e >= s_hi) ? NONE : e;
        if (e != NONE && e >= s_hi) S.stop = 2;   // imposed entry beyond the stripe: nothing starts here
        const int64_t slo_i = (int64_t)sd.t_begin * TILE - d0;
        if (e != NONE && (int64_t)e < slo_i) {     // k_link never imposes an entry before the stripe (bug trap)
            S.stop = 2;
            S.stripe_entry = NONE;
            atomicOr(&ctr->overflow, 4u);
        }
        S.tile_exit = S.entry;
    }
    issue_tile(sg, sd.t_begin, S.buf[0]);
#ifdef KVR_PROF
    unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif
    uint32_t k = sd.t_begin;
    int cur = 0;
    bool loaded = true;   // tile k has been issued into buf[cur]
    for (;; ++k, cur ^= 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        KVR_BARRIER();
        const bool in_stripe = k < sd.t_end;
        if (S.stop || (!in_stripe && !S.carry) || k >= sg.n_tiles) break;
        if (!loaded) {   // not prefetched (stripe end): load now
            issue_tile(sg, k, S.buf[cur]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            KVR_BARRIER();
        }
        // prefetch the next tile while this one is processed
        loaded = (k + 1 < sg.n_tiles) && (k + 1 < sd.t_end || S.carry);
        if (loaded) issue_tile(sg, k + 1, S.buf[cur ^ 1]);
        KVR_STAMP(0);

        const int64_t lo = (int64_t)k * TILE - d0;
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        uint8_t *tile = S.buf[cur];
        const TileView tv{sg.base, tile, len, lo};
        const int64_t cs_i = lo + (int64_t)tid * SC;
        const uint64_t cs = cs_i < (int64_t)vlo ? vlo : (uint64_t)cs_i;
        const uint64_t ce = (uint64_t)(cs_i + SC) > vhi ? vhi : (uint64_t)(cs_i + SC);

        // ---- F. framing --------------------------------------------------------------------
        if (in_stripe && S.search) {   // the stripe's entry: the first plausible record start
            if (cs < ce) {
                const uint64_t cand = find_cand(tv, cs, ce);
                if (cand != NONE) atomicMin(&S.cand_min, (uint32_t)((int64_t)cand - lo));
            }
            KVR_BARRIER();
            if (tid == 0 && S.cand_min != N32) {
                S.entry = (uint64_t)(lo + (int64_t)S.cand_min);
                S.search = 0;
                S.stripe_entry = S.entry;
                S.tile_exit = S.entry;
            }
            KVR_BARRIER();
        }
        const bool walk = in_stripe && !S.search && S.entry < vhi;
        if (walk) {
            if (tid == 0) {   // exact hops while the tile looks sparse
                uint64_t p = S.entry;
                uint32_t n = 0;
                if (S.prev_n <= DENSE) {
                    while (p < vhi && n < HOP_BUDGET) {
                        S.r.rec[n++] = (uint16_t)((int64_t)p - lo);
                        p = next_rec(tv, p);
                        if (p == ERRP) break;
                    }
                }
                S.nrec = n;
                S.tile_exit = p;
                S.need_spec = (p != ERRP && p < vhi) ? 1u : 0u;
            }
            KVR_BARRIER();
            if (S.need_spec) {   // dense: speculate per sub-chunk from the exact position e
                const uint64_t e = S.tile_exit;
                uint16_t cand16 = N16, last16 = N16;
                uint32_t x = X_BEYOND, cnt = 0;
                const uint64_t p0 = cs > e ? cs : e;
                if (p0 < ce) {
                    const uint64_t cand = find_cand(tv, p0, ce);
                    if (cand != NONE) {
                        cand16 = (uint16_t)((int64_t)cand - lo);
                        cnt = walk_spec(tv, cand, ce, &x, &last16);
                    }
                }
                S.u.sp.sc_cand[tid] = cand16;
                S.u.sp.sc_exit[tid] = x;
                S.u.sp.sc_cnt[tid] = (uint16_t)cnt;
                S.u.sp.sc_last[tid] = last16;
                KVR_BARRIER();
                if (tid < 64) stitch(S, tv, e, vhi, ctr);
                KVR_BARRIER();
                const uint16_t ent = S.u.sp.sc_entry[tid];
                if (ent != N16) {   // materialize the record starts of this sub-chunk
                    uint32_t o = S.nrec + S.u.sp.sc_base[tid];
                    uint64_t p = (uint64_t)(lo + (int64_t)ent);
                    const uint32_t c = S.u.sp.sc_cnt[tid];
                    for (uint32_t i = 0; i < c; ++i) {
                        S.r.rec[o + i] = (uint16_t)((int64_t)p - lo);
                        if (i + 1 < c) p = next_spec(tv, p);
                    }
                }
                KVR_BARRIER();
                if (tid == 0) S.nrec += S.spec_total;
            }
        }
        // tile setup: pool slots, long-value registry (zeroed after the speculation arrays die)
        {
            const bool pend = S.carry == 2u && (int64_t)S.c_vb - lo < TILE;
            const int32_t pvb = pend ? (int32_t)((int64_t)S.c_vb - lo) : 0;
            const uint32_t pb1 = pend ? (uint32_t)(pvb / SC + 1) : 0u;
            S.u.lg.bkey[tid + 1] = (pend && pb1 == (uint32_t)tid + 1) ? (((uint32_t)pvb + 1u) << 9) : 0u;
            if (tid == 0) {
                const uint32_t n = S.nrec;
                if (n > S.chunk_left) {                   // bulk pool allocation
                    const uint64_t m = n > pool_chunk ? n : pool_chunk;
                    S.chunk_base = atomicAdd(&ctr->pool_cursor, (unsigned long long)m);
                    S.chunk_left = m;
                    if (S.chunk_base + m > pool_cap) atomicOr(&ctr->overflow, 1u);
                }
                S.pool_base = S.chunk_base;
                S.chunk_base += n;
                S.chunk_left -= n;
                S.nlong = 0;
                S.n_carry = 0;
                if (pend) {   // a value whose record started in an earlier tile begins in this one
                    const int64_t ve = (int64_t)S.c_ve - lo;
                    S.u.lg.lvb[0] = pvb;
                    S.u.lg.lve[0] = ve > FAR ? FAR : (int32_t)ve;
                    S.u.lg.lidx[0] = (uint32_t)S.c_idx;
                    S.nlong = 1;
                    S.carry = 0;
                } else if (S.carry == 2u) {               // still further on: hand it over untouched
                    S.n_carry = 2; S.n_vb = S.c_vb; S.n_ve = S.c_ve; S.n_idx = S.c_idx;
                }
            }
        }
        KVR_BARRIER();
        KVR_STAMP(1);

        // ---- R. records: one thread per record ------------------------------------------------
        const uint32_t nrec = S.nrec;
        uint32_t my_err = N32, my_kind = 0;
        uint64_t my_aux = 0;
        for (uint32_t j = tid; j < nrec; j += NT) {
            const uint64_t p = (uint64_t)(lo + (int64_t)S.r.rec[j]);
            const uint64_t slot = S.pool_base + j;
            const uint32_t op = tv.rd8(p);
            if (len - p < 5) { my_err = j; my_kind = KVR_E_KEY_LEN; break; }            // engine.rs:96
            const uint64_t klen = tv.rd32(p + 1);
            const uint64_t kb = p + 5;
            if (len - kb < klen) { my_err = j; my_kind = KVR_E_KEY; break; }             // engine.rs:107
            uint64_t vu = 0;
            uint32_t el = 0;
            if (!utf8_check(tv, kb, klen, &vu, &el)) {                                   // engine.rs:114
                my_err = j; my_kind = KVR_E_UTF8; my_aux = vu | ((uint64_t)el << 32); break;
            }
            if (op > 1u) { my_err = j; my_kind = KVR_E_OPCODE; my_aux = op; break; }     // engine.rs:143
            kvr_tuple t;
            t.rec_off = p;
            t.seg_idx = sd.seg;
            t.key_len = (uint32_t)klen;
            t.key_tag = ~crc_range(tv, ~0u, kb, klen, S.T);
            t.op = (uint8_t)op;
            t.flags = 0;
            t.reserved = 0;
            t.crc32 = 0;
            t.val_len = 0;
            if (op == 0u) {
                const uint64_t q = kb + klen;
                if (len - q < 4) { my_err = j; my_kind = KVR_E_VAL_LEN; break; }         // engine.rs:121
                const uint64_t vlen = tv.rd32(q);
                const uint64_t vb = q + 4, ve = vb + vlen;
                if (len - vb < vlen) { my_err = j; my_kind = KVR_E_VAL; break; }         // engine.rs:130
                t.val_len = (uint32_t)vlen;
                if (vlen <= (uint64_t)SMALL) {
                    t.crc32 = ~crc_range(tv, ~0u, vb, vlen, S.T);
                } else {
                    const int64_t vbr = (int64_t)vb - lo, ver = (int64_t)ve - lo;
                    if (vbr < TILE) {
                        const uint32_t L = atomicAdd(&S.nlong, 1u);
                        S.u.lg.lvb[L] = (int32_t)vbr;
                        S.u.lg.lve[L] = ver > FAR ? FAR : (int32_t)ver;
                        S.u.lg.lidx[L] = (uint32_t)slot;
                        S.u.lg.bkey[vbr / SC + 1] = ((uint32_t)(vbr + 1) << 9) | L;
                        if (ver > TILE) { S.n_vb = vb; S.n_ve = ve; S.n_idx = slot; }   // runs past the tile
                    } else {            // the value starts in a later tile
                        S.n_carry = 2; S.n_vb = vb; S.n_ve = ve; S.n_idx = slot;
                    }
                }
            }
            if (slot < pool_cap) pool[slot] = t;
        }
        if (my_err != N32) atomicMin(&S.err_rec, my_err);
        KVR_BARRIER();
        KVR_STAMP(2);
        if (my_err != N32 && my_err == S.err_rec) {
            S.err_pos = (uint64_t)(lo + (int64_t)S.r.rec[my_err]);
            S.err_kind = my_kind;
            S.err_aux = my_aux;
        }

        // ---- C. CRC of long values -----------------------------------------------------------
        if (S.nlong != 0 || S.carry == 1u) {
            LongLds &G = S.u.lg;
            // which value crosses boundary tid + 1 (the end of unit tid): latest long value
            // starting before it (prefix max of keys), if it reaches past it
            uint32_t key = G.bkey[tid + 1];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(key, d, 64);
                if (lane >= d && o > key) key = o;
            }
            if (lane == 63) S.wt[wave] = key;
            KVR_BARRIER();
            for (int w = 0; w < wave; ++w) key = S.wt[w] > key ? S.wt[w] : key;
            const int32_t pb = SC * (tid + 1);
            int32_t Vend = VNONE;
            if (key != 0u) {
                const int32_t L = (int32_t)(key & 511u);
                if (G.lve[L] > pb) Vend = L;
            } else if (S.carry == 1u && (int64_t)S.c_ve - lo > (int64_t)pb) {
                Vend = VCARRY;
            }
            G.vc[tid + 1] = Vend;
            if (tid == 0) G.vc[0] = S.carry == 1u ? VCARRY : VNONE;
            KVR_BARRIER();
            const int32_t Vst = G.vc[tid];
            const int32_t us = SC * tid;
            const uint4 *up = reinterpret_cast<const uint4 *>(tile + us);
            const uint4 q0 = up[0], q1 = up[1], q2 = up[2], q3 = up[3];
            const uint32_t w[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                                    q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
            // piece of the value crossing the unit's end: register contribution at that boundary
            uint32_t v = 0;
            uint32_t f = 1;   // segment start (the scan does not look further left)
            if (Vend != VNONE) {
                int32_t a = 0;
                bool starts = false;
                if (Vend >= 0 && G.lvb[Vend] >= us) { a = G.lvb[Vend] - us; starts = true; }
                uint32_t c = 0;
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) {   // bytes before the value are zeroed (branch-free)
                    const int sh = min(max(8 * (a - 4 * kk), 0), 32);
                    c = crc4(c, w[kk] & (uint32_t)(~0ull << sh), S.T);
                }
                if (starts) v = c ^ S.IX[SC - a];
                else if (tid == 0) v = c ^ kmul(S.c_state, S.KT);   // carried state across unit 0
                else { v = c; f = 0; }
            }
            // segmented scan over the 256 units (Kogge-Stone through LDS; step j shifts by 2^j
            // units = the constant x^(8*64*2^j)): state at boundary s+1 = f ? v : state(s)*X(64) ^ v
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int d = 1 << j;
                uint64_t *xb = S.r.sc.x[j & 1];
                xb[tid] = (uint64_t)v | ((uint64_t)f << 32);
                KVR_BARRIER();
                if (tid >= d && !f) {
                    const uint64_t o = xb[tid - d];
                    v ^= kmul((uint32_t)o, S.KT + 128 * j);
                    f = (uint32_t)(o >> 32);
                }
            }
            S.r.sc.sx[tid] = v;
            KVR_BARRIER();
            KVR_STAMP(3);
            // the value crossing the unit's start ends in this unit: finish its CRC
            if (Vst != VNONE) {
                const int64_t ve_rel = Vst == VCARRY ? (int64_t)S.c_ve - lo : (int64_t)G.lve[Vst];
                if (ve_rel <= (int64_t)us + SC) {
                    const int m = (int)(ve_rel - us);   // 1 .. 64
                    uint32_t c = tid == 0 ? S.c_state : S.r.sc.sx[tid - 1];
#pragma unroll
                    for (int kk = 0; kk < 16; ++kk) {
                        const uint32_t cn = crc4(c, w[kk], S.T);
                        c = 4 * kk + 4 <= m ? cn : c;
                    }
                    for (int b = m & ~3; b < m; ++b) c = crc1(c, tile[us + b], S.T);
                    const uint64_t idx = Vst == VCARRY ? S.c_idx : (uint64_t)G.lidx[Vst];
                    if (idx < pool_cap) pool[idx].crc32 = ~c;
                }
            }
            if (tid == NT - 1) {   // a value running past the tile: hand over its register state
                const int32_t Vo = G.vc[NT];
                if (Vo != VNONE) {
                    S.n_carry = 1;
                    S.n_state = v;
                    if (Vo == VCARRY) { S.n_vb = S.c_vb; S.n_ve = S.c_ve; S.n_idx = S.c_idx; }
                }
            }
        }
        KVR_STAMP(4);
        // bookkeeping (thread 0): tile result, next entry, carried value
        KVR_BARRIER();
        if (tid == 0) {
            const uint32_t n = S.nrec;
            const uint32_t n_ok = S.err_rec < n ? S.err_rec : n;
            if (in_stripe) {
                tres[sg.tile0 + k].pool_off = n_ok ? S.pool_base : 0ull;
                tres[sg.tile0 + k].count = n_ok;
                S.total += n_ok;
                if (walk) S.entry = S.tile_exit;
                S.prev_n = n;
            }
            S.carry = S.n_carry;
            S.c_vb = S.n_vb; S.c_ve = S.n_ve; S.c_idx = S.n_idx; S.c_state = S.n_state;
            if (S.err_pos != NONE) S.stop = 1;
            else if (walk && S.tile_exit == ERRP) {   // defensive: a broken chain must have reported
                S.stop = 1; S.err_pos = S.entry; S.err_kind = KVR_E_VAL;
            }
            S.nrec = 0; S.need_spec = 0; S.cand_min = N32; S.err_rec = N32;
            S.tile_exit = S.entry;
        }
        KVR_STAMP(5);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain an unused prefetch before exit
    // tiles of the stripe that were never reached (error stop / pass-through) hold no tuples
    const uint32_t kfirst = k < sd.t_end ? k : sd.t_end;
    for (uint32_t kk = kfirst + tid; kk < sd.t_end; kk += NT) {
        tres[sg.tile0 + kk].pool_off = 0;
        tres[sg.tile0 + kk].count = 0;
    }
    if (tid == 0) {
        StripeRes r;
        r.entry = S.stripe_entry;
        r.exit = (S.err_pos != NONE) ? ERRP : (S.stripe_entry == NONE ? NONE : S.entry);
        r.err_pos = S.err_pos;
        r.err_aux = S.err_aux;
        r.err_kind = (S.err_pos != NONE) ? S.err_kind : 0u;
        r.count = S.total;
        r.forced = redo_mode ? 1u : 0u;
        r.pad = 0;
        sres[si] = r;
    }
}

}  // namespace kvr
