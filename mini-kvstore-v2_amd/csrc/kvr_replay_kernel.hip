/*
 * kvr_replay_kernel.hip — k_replay, the hot path (gfx950).
 *
 * One workgroup replays one stripe (consecutive tiles of one segment) exactly as
 * src/store/engine.rs:79-154 walks a segment file, and emits one 32-B kvr_tuple per record with
 * the CRC-32 of its key and value (crc32fast::hash semantics, src/volume/storage.rs:27).
 *
 * Per 16-KiB tile (see kvr_device.h for the geometry):
 *   0  wait for the tile's LDS-DMA; start the DMA of the next tile into the other buffer
 *   1  every thread speculates a record chain through its 64-B sub-chunk (no HBM reads)
 *   2  wave 0 stitches the sub-chains from the tile entry (pointer jumping) and repairs wrong
 *      speculation; it publishes per sub-chunk: accepted entry, tuple index, covering record
 *   3  every thread parses its records exactly (error kinds in engine.rs order, UTF-8 check,
 *      key CRC), writes their tuples, and CRCs every value byte of its sub-chunk: short values
 *      whole, long ones as a shifted share XOR-ed into an LDS accumulator per record
 *   4  one thread per long record folds the shares and writes (or XORs, when the value spans
 *      tiles) the CRC into the tuple
 * Barriers are raw s_barrier + lgkmcnt waits so the next tile's LDS-DMA stays in flight.
 */
#include "kvr_device.h"

namespace kvr {

constexpr uint16_t N16 = 0xFFFFu;        // no offset
constexpr uint16_t CARRY16 = 0xFFFEu;    // covering record started in an earlier tile
constexpr uint32_t X_BEYOND = 0xFFFFFFFEu, X_ERR = 0xFFFFFFFFu;
constexpr uint64_t BEYOND = ~0ull - 2;   // record end not readable from the tile (>= tile end)
constexpr int16_t T_END = NT, T_ERR = NT + 1, T_MM = NT + 2;
constexpr uint32_t POOL_CHUNK = 2048;

struct __align__(16) RSmem {
    uint8_t  buf[2][TILE];
    uint32_t nt[16 * 32];
    uint32_t sc_exit[NT];       // exit offset from lo (X_BEYOND / X_ERR)
    uint32_t sc_base[NT];       // tuple index of the sub-chunk's first record within the tile
    uint32_t acc[NT + 1];       // per long record: XOR of shifted unit shares
    uint32_t tail[NT + 1];      // per long record: raw CRC of its last share in this tile
    uint16_t sc_cand[NT], sc_last[NT], sc_cnt[NT], sc_entry[NT], sc_cover[NT];
    int16_t  nxt[NT], nxt0[NT];
    uint8_t  reach[NT];
    uint64_t entry, tile_exit, err_pos, err_aux, stripe_entry, pool_base, chunk_base, chunk_left;
    uint64_t c_vb, c_ve, c_idx;                 // carried long value (started in an earlier tile)
    uint32_t has_carry, err_kind, tile_count, total, search, stop, tile_found, last_off;
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

__device__ __forceinline__ bool plausible(const TileView &tv, uint64_t p) {
    const uint64_t nx = next_spec(tv, p);
    if (nx == ERRP) return false;
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
        if (nx == ERRP) { x = X_ERR; break; }
        ++cnt;
        last = (uint16_t)((int64_t)p - tv.lo);
        if (nx == BEYOND) { x = X_BEYOND; break; }
        p = nx;
    }
    *exit_off = x;
    *last_off = last;
    return cnt;
}

// ---------------------------------------------------------------------------------------
// stitching (wave 0)
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
__device__ void repair(RSmem &S, const TileView &tv, uint64_t y, uint64_t vhi) {
    const int64_t lo = tv.lo;
    for (int k = 0; k < 64; ++k) {
        const int t = (int)(((int64_t)y - lo) / SC);
        const int64_t ce = lo + (int64_t)(t + 1) * SC;
        const uint64_t pe = (uint64_t)ce > vhi ? vhi : (uint64_t)ce;
        uint32_t x;
        uint16_t last;
        const uint32_t cnt = walk_spec(tv, y, pe, &x, &last);
        S.sc_cand[t] = (uint16_t)((int64_t)y - lo);
        S.sc_exit[t] = x;
        S.sc_cnt[t] = (uint16_t)cnt;
        S.sc_last[t] = last;
        if (x >= X_BEYOND || lo + (int64_t)x >= (int64_t)vhi) return;
        if (S.sc_cand[x / SC] == x) return;        // back in step with the speculation
        y = (uint64_t)(lo + (int64_t)x);
    }
}

// Stitch from the tile entry e (vlo <= e < vhi).  Publishes sc_entry / sc_base / sc_cover,
// S.tile_count, S.tile_exit, S.last_off and the tile's pool range.
__device__ void stitch(RSmem &S, const TileView &tv, uint64_t e, uint64_t vhi, Counters *ctr, uint64_t pool_cap,
                       uint32_t pool_chunk) {
    const int lane = threadIdx.x;
    const int64_t lo = tv.lo;
    const int s0 = (int)(((int64_t)e - lo) / SC);
    const uint16_t e_off = (uint16_t)((int64_t)e - lo);
    const uint32_t vhi_off = (uint32_t)((int64_t)vhi - lo);
    for (int guard = 0; guard < 2 * NT + 8; ++guard) {
        if (S.sc_cand[s0] != e_off) {
            if (lane == 0) repair(S, tv, e, vhi);
            wave_sync_lds();
            continue;
        }
        bool any = false;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            const uint16_t c = S.sc_cand[s];
            const uint32_t x = S.sc_exit[s];
            int16_t T;
            if (c == N16) T = T_END;
            else if (x == X_ERR) T = T_ERR;
            else if (x >= vhi_off) T = T_END;          // includes X_BEYOND
            else { const int t = (int)(x / SC); T = (S.sc_cand[t] == x) ? (int16_t)t : T_MM; any = true; }
            S.nxt0[s] = T;
            S.nxt[s] = T;
            S.reach[s] = (s == s0) ? 1 : 0;
        }
        wave_sync_lds();
        for (int r = 0; r < 8 && __any(any); ++r) {   // J <- J o J, reach <- reach U J(reach)
            int16_t jn[4];
            any = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int s = 4 * lane + j;
                const int16_t J = S.nxt[s];
                jn[j] = J < NT ? S.nxt[J] : J;
                any |= jn[j] < NT;
                if (J < NT && S.reach[s]) S.reach[J] = 1;
            }
            wave_sync_lds();
#pragma unroll
            for (int j = 0; j < 4; ++j) S.nxt[4 * lane + j] = jn[j];
            wave_sync_lds();
        }
        int smax = -1;
#pragma unroll
        for (int j = 0; j < 4; ++j) if (S.reach[4 * lane + j]) smax = 4 * lane + j;
        smax = wave_max_i32(smax);
        const int16_t Tl = S.nxt0[smax];
        if (Tl == T_MM) {
            if (lane == 0) repair(S, tv, (uint64_t)(lo + (int64_t)S.sc_exit[smax]), vhi);
            wave_sync_lds();
            continue;
        }
        // accepted path: entries, tuple index bases, covering records
        uint16_t ent[4], lst[4];
        uint32_t c4[4];
        int lastrec = -1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            const bool on = S.reach[s] != 0;
            ent[j] = on ? S.sc_cand[s] : N16;
            c4[j] = on ? S.sc_cnt[s] : 0u;
            lst[j] = on ? S.sc_last[s] : N16;
            if (on && lst[j] != N16) lastrec = lst[j];
        }
        const uint32_t tot = c4[0] + c4[1] + c4[2] + c4[3];
        uint32_t inc = tot;
        int cov = lastrec;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            const int oc = __shfl_up(cov, d, 64);
            if (lane >= d) { inc += o; cov = oc > cov ? oc : cov; }
        }
        uint32_t base = inc - tot;
        int cur = __shfl_up(cov, 1, 64);                  // last record start before this lane
        if (lane == 0) cur = -1;
        const uint16_t init_cover = S.has_carry ? CARRY16 : N16;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            S.sc_entry[s] = ent[j];
            S.sc_base[s] = base;
            S.sc_cover[s] = cur < 0 ? init_cover : (uint16_t)cur;
            base += c4[j];
            if (lst[j] != N16) cur = lst[j];
        }
        const uint32_t total = __shfl(inc, 63, 64);
        if (lane == 0) {
            S.tile_count = total;
            S.last_off = S.sc_last[smax];
            uint64_t x;
            if (Tl == T_ERR) x = ERRP;
            else if (S.sc_exit[smax] != X_BEYOND) x = (uint64_t)(lo + (int64_t)S.sc_exit[smax]);
            else x = next_rec(tv, (uint64_t)(lo + (int64_t)S.sc_last[smax]));   // exact, may read HBM
            S.tile_exit = x;
            if (total > S.chunk_left) {                   // bulk pool allocation
                const uint64_t n = total > pool_chunk ? total : pool_chunk;
                S.chunk_base = atomicAdd(&ctr->pool_cursor, (unsigned long long)n);
                S.chunk_left = n;
                if (S.chunk_base + n > pool_cap) atomicOr(&ctr->overflow, 1u);
            }
            S.pool_base = S.chunk_base;
            S.chunk_base += total;
            S.chunk_left -= total;
        }
        return;
    }
    if (lane == 0) {   // unreachable: every round repairs one more sub-chunk for good (bug trap)
        S.tile_count = 0;
        S.tile_exit = ERRP;
        atomicOr(&ctr->overflow, 2u);
    }
}

// ---------------------------------------------------------------------------------------
// CRC shares
// ---------------------------------------------------------------------------------------
// Raw CRC of tile bytes [s, e) (LDS offsets, inside one 64-B unit), with the value's initial
// register 0xFFFFFFFF folded in as an XOR over the value's first 4 bytes [vi, vi+4).
__device__ __forceinline__ uint32_t unit_raw(const RSmem &S, const uint8_t *tile, int s, int e, bool last, int vi) {
    const int wend = last ? (e & ~15) : e;
    uint32_t c = 0;
    for (int w = s & ~15; w < wend; w += 16) {
        uint4 d = *reinterpret_cast<const uint4 *>(tile + w);
        const int k = s - w;   // leading bytes outside the share: zero (no effect on a raw CRC)
        if (k > 0) {
            d.x &= k >= 4 ? 0u : (~0u << (8 * k));
            d.y &= k >= 8 ? 0u : (k <= 4 ? ~0u : (~0u << (8 * (k - 4))));
            d.z &= k >= 12 ? 0u : (k <= 8 ? ~0u : (~0u << (8 * (k - 8))));
            d.w &= k <= 12 ? ~0u : (~0u << (8 * (k - 12)));
        }
        if (vi >= w - 3 && vi < w + 16) {        // init bytes of the value overlap this word
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int bpos = vi + q;
                if (bpos >= w && bpos < w + 16 && bpos >= s && bpos < e) {
                    const int wi = (bpos - w) >> 2, sh = 8 * ((bpos - w) & 3);
                    if (wi == 0) d.x ^= 0xFFu << sh;
                    else if (wi == 1) d.y ^= 0xFFu << sh;
                    else if (wi == 2) d.z ^= 0xFFu << sh;
                    else d.w ^= 0xFFu << sh;
                }
            }
        }
        c = nslice16(c, d, S.nt);
    }
    for (int x = s > wend ? s : wend; x < e; ++x) {
        uint32_t b = tile[x];
        if (x >= vi && x < vi + 4) b ^= 0xFFu;
        c = nbyte(c, b, S.nt);
    }
    return c;
}

struct RecInfo { uint64_t vb, ve; uint32_t vlen; bool set; bool ok; };

// header of a record known to be valid (on the accepted chain); HBM fallback for straddling fields
__device__ __forceinline__ RecInfo parse_hdr(const TileView &tv, uint64_t p) {
    RecInfo r;
    r.ok = false; r.set = false; r.vb = 0; r.ve = 0; r.vlen = 0;
    const uint64_t n = tv.len;
    if (p >= n || n - p < 5) return r;
    const uint32_t op = tv.rd8(p);
    const uint64_t kb = p + 5, klen = tv.rd32(p + 1);
    if (n - kb < klen) return r;
    if (op == 1u) { r.ok = true; r.vb = r.ve = kb + klen; return r; }
    if (op != 0u) return r;
    const uint64_t q = kb + klen;
    if (n - q < 4) return r;
    r.vlen = tv.rd32(q);
    r.vb = q + 4;
    r.ve = r.vb + r.vlen;
    if (r.ve > n) return r;
    r.set = true;
    r.ok = true;
    return r;
}

// does this SET record's value go through the unit-share path?  (Values of at most SMALL
// bytes are CRC'd whole by their walker, reading HBM for the rare bytes past the tile.)
__device__ __forceinline__ bool is_long(const RecInfo &r) {
    return r.set && r.vlen > (uint32_t)SMALL;
}

// share of value [vb, ve) inside unit [us, ue) (segment positions) for slot `slot`
__device__ __forceinline__ void add_share(RSmem &S, const uint8_t *tile, int64_t lo, uint64_t vlo, uint64_t vhi,
                                          uint64_t vb, uint64_t ve, uint64_t us, uint64_t ue, int slot,
                                          const uint32_t *__restrict__ pw16) {
    const uint64_t a = vb > us ? vb : us;
    const uint64_t bpos = ve < vhi ? ve : vhi;       // end of the value's piece in this tile
    const uint64_t e = bpos < ue ? bpos : ue;
    if (a >= e) return;
    const int so = (int)((int64_t)a - lo), eo = (int)((int64_t)e - lo);
    // the init bytes [vb, vb + 4) may straddle the previous tile: keep their (negative) offset
    const int64_t vio = (int64_t)vb - lo;
    const int vi = vio < -16 ? -16 : (int)vio;
    const bool last = (e == bpos);
    const uint32_t raw = unit_raw(S, tile, so, eo, last, vi);
    if (last) {
        S.tail[slot] = raw;
    } else {
        const uint32_t bf = (uint32_t)((int64_t)bpos - lo) & ~15u;
        const uint32_t m = pw16[(bf - (uint32_t)eo) >> 4];
        atomicXor(&S.acc[slot], m == GF_ONE ? raw : gf_mul(raw, m));
    }
}

// async HBM -> LDS copy of tile k (16-B LDS-DMA per lane; wave w of instruction i lands at
// byte (i * NT + w * 64) * 16, i.e. word i * NT + threadIdx.x)
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
    const int tid = threadIdx.x;
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

    for (int i = tid; i < 16 * 32; i += NT) S.nt[i] = tb.nib[i];
    if (tid == 0) {
        S.has_carry = 0;
        S.err_kind = 0;
        S.err_pos = NONE;
        S.err_aux = 0;
        S.total = 0;
        S.stop = 0;
        S.chunk_left = 0;
        S.chunk_base = 0;
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
        if (S.stop || (!in_stripe && !S.has_carry) || k >= sg.n_tiles) break;
        if (!loaded) {   // not prefetched (stripe end): load now
            issue_tile(sg, k, S.buf[cur]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            KVR_BARRIER();
        }
        // prefetch the next tile while this one is processed
        loaded = (k + 1 < sg.n_tiles) && (k + 1 < sd.t_end || S.has_carry);
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

        // 1. speculative sub-chains
        const bool walk = in_stripe && (S.search || S.entry < vhi);
        S.acc[tid] = 0;
        S.tail[tid] = 0;
        if (tid == 0) { S.acc[NT] = 0; S.tail[NT] = 0; S.tile_count = 0; S.tile_found = 0; S.tile_exit = S.entry; }
        if (walk) {
            const uint64_t lower = S.search ? vlo : S.entry;
            uint16_t cand16 = N16, last16 = N16;
            uint32_t x = X_BEYOND;
            uint32_t cnt = 0;
            const uint64_t p0 = cs > lower ? cs : lower;
            if (p0 < ce) {
                const uint64_t cand = find_cand(tv, p0, ce);
                if (cand != NONE) {
                    cand16 = (uint16_t)((int64_t)cand - lo);
                    cnt = walk_spec(tv, cand, ce, &x, &last16);
                }
            }
            S.sc_cand[tid] = cand16;
            S.sc_exit[tid] = x;
            S.sc_cnt[tid] = (uint16_t)cnt;
            S.sc_last[tid] = last16;
        }
        KVR_BARRIER();
        KVR_STAMP(1);
        // 2. stitch (wave 0)
        if (walk) {
            if (tid < 64) {
                uint64_t e = S.entry;
                if (S.search) {   // the stripe's entry: the first plausible record start
                    uint32_t m = N16;
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t c = S.sc_cand[4 * tid + j];
                        m = c < m ? c : m;
                    }
                    for (int d = 32; d >= 1; d >>= 1) {
                        const uint32_t o = __shfl_xor(m, d, 64);
                        m = o < m ? o : m;
                    }
                    e = (m == N16) ? NONE : (uint64_t)(lo + (int64_t)m);
                }
                if (e != NONE) {
                    stitch(S, tv, e, vhi, ctr, pool_cap, pool_chunk);
                    if (tid == 0) {
                        S.tile_found = 1;
                        if (S.search) { S.search = 0; S.stripe_entry = e; }
                    }
                }
            }
        } else if (tid < 64) {   // no record starts here: every sub-chunk is covered by the carry
            S.sc_entry[4 * tid + 0] = S.sc_entry[4 * tid + 1] = S.sc_entry[4 * tid + 2] = S.sc_entry[4 * tid + 3] = N16;
            const uint16_t c = S.has_carry ? CARRY16 : N16;
            S.sc_cover[4 * tid + 0] = S.sc_cover[4 * tid + 1] = S.sc_cover[4 * tid + 2] = S.sc_cover[4 * tid + 3] = c;
        }
        KVR_BARRIER();
        KVR_STAMP(2);

        // 3. records of this sub-chunk + CRC shares of every value byte in it
        uint64_t my_err = NONE, my_aux = 0;
        uint32_t my_kind = 0;
        const bool found = walk && S.tile_found;
        if (found || !walk) {
            const uint16_t ent = found ? S.sc_entry[tid] : N16;
            uint64_t own_vb = 0, own_ve = 0;
            bool own_long = false;
            if (ent != N16) {
                uint64_t p = (uint64_t)(lo + (int64_t)ent);
                uint64_t slot = S.pool_base + S.sc_base[tid];
                while (p < ce) {
                    const uint32_t op = tv.rd8(p);
                    if (len - p < 5) { my_err = p; my_kind = KVR_E_KEY_LEN; break; }            // engine.rs:96
                    const uint64_t klen = tv.rd32(p + 1);
                    const uint64_t kb = p + 5;
                    if (len - kb < klen) { my_err = p; my_kind = KVR_E_KEY; break; }             // engine.rs:107
                    uint64_t vu = 0;
                    uint32_t el = 0;
                    if (!utf8_check(tv, kb, klen, &vu, &el)) {                                   // engine.rs:114
                        my_err = p; my_kind = KVR_E_UTF8; my_aux = vu | ((uint64_t)el << 32); break;
                    }
                    if (op > 1u) { my_err = p; my_kind = KVR_E_OPCODE; my_aux = op; break; }     // engine.rs:143
                    kvr_tuple t;
                    t.rec_off = p;
                    t.seg_idx = sd.seg;
                    t.key_len = (uint32_t)klen;
                    t.key_tag = ~crc_range(tv, ~0u, kb, klen, S.nt);
                    t.op = (uint8_t)op;
                    t.flags = 0;
                    t.reserved = 0;
                    t.crc32 = 0;
                    uint64_t nx;
                    own_long = false;
                    if (op == 0u) {
                        const uint64_t q = kb + klen;
                        if (len - q < 4) { my_err = p; my_kind = KVR_E_VAL_LEN; break; }         // engine.rs:121
                        const uint64_t vlen = tv.rd32(q);
                        const uint64_t vb = q + 4, ve = vb + vlen;
                        if (len - vb < vlen) { my_err = p; my_kind = KVR_E_VAL; break; }         // engine.rs:130
                        t.val_len = (uint32_t)vlen;
                        if (vlen > (uint64_t)SMALL) {
                            own_long = true; own_vb = vb; own_ve = ve;
                        } else {
                            t.crc32 = ~crc_range(tv, ~0u, vb, vlen, S.nt);
                        }
                        nx = ve;
                    } else {
                        t.val_len = 0;
                        nx = kb + klen;
                    }
                    if (slot < pool_cap) pool[slot] = t;
                    ++slot;
                    p = nx;
                }
                if (my_err != NONE) {
                    own_long = false;
                    atomicMin(reinterpret_cast<unsigned long long *>(&S.err_pos), (unsigned long long)my_err);
                }
            }
            // shares: the covering long value, then this sub-chunk's own long value
            const uint16_t cov = S.sc_cover[tid];
            if (cov != N16 && cs < ce) {
                uint64_t vb, ve;
                int slot;
                bool lng;
                if (cov == CARRY16) {
                    vb = S.c_vb; ve = S.c_ve; slot = NT; lng = true;
                } else {
                    const RecInfo r = parse_hdr(tv, (uint64_t)(lo + (int64_t)cov));
                    vb = r.vb; ve = r.ve; slot = cov / SC; lng = r.ok && is_long(r);
                }
                if (lng) add_share(S, tile, lo, vlo, vhi, vb, ve, cs, ce, slot, tb.pw16);
            }
            if (own_long) add_share(S, tile, lo, vlo, vhi, own_vb, own_ve, cs, ce, tid, tb.pw16);
        }
        KVR_BARRIER();
        KVR_STAMP(3);
        if (my_err != NONE && my_err == S.err_pos) {
            S.err_kind = my_kind;
            S.err_aux = my_aux;
        }

        // 4. fold the shares of every long value with bytes in this tile
        if (found && S.sc_entry[tid] != N16 && S.sc_last[tid] != N16) {
            const RecInfo r = parse_hdr(tv, (uint64_t)(lo + (int64_t)S.sc_last[tid]));
            if (r.ok && is_long(r) && r.vb < vhi) {
                const uint64_t idx = S.pool_base + S.sc_base[tid] + S.sc_cnt[tid] - 1u;
                const uint32_t bo = (uint32_t)((int64_t)(r.ve < vhi ? r.ve : vhi) - lo);
                const uint32_t a = S.acc[tid];
                uint32_t st = S.tail[tid] ^ (a ? gf_mul(a, tb.pw1[bo & 15u]) : 0u);
                st = (r.ve <= vhi) ? ~st : gf_mul(st, gf_xpow(r.ve - vhi, tb.xw));
                if (idx < pool_cap) pool[idx].crc32 = st;
            }
        }
        if (tid == 0 && S.has_carry && S.c_vb < vhi && S.c_ve > vlo) {
            const uint32_t bo = (uint32_t)((int64_t)(S.c_ve < vhi ? S.c_ve : vhi) - lo);
            const uint32_t a = S.acc[NT];
            uint32_t st = S.tail[NT] ^ (a ? gf_mul(a, tb.pw1[bo & 15u]) : 0u);
            st = (S.c_ve <= vhi) ? ~st : gf_mul(st, gf_xpow(S.c_ve - vhi, tb.xw));
            if (S.c_idx < pool_cap) atomicXor(&pool[S.c_idx].crc32, st);
        }
        KVR_STAMP(4);
        // bookkeeping (thread 0): tile result, next entry, carried value
        KVR_BARRIER();
        if (tid == 0) {
            if (in_stripe) {
                tres[sg.tile0 + k].pool_off = S.tile_count ? S.pool_base : 0ull;
                tres[sg.tile0 + k].count = S.tile_count;
                S.total += S.tile_count;
                if (found) S.entry = S.tile_exit;
            }
            if (found) {
                const RecInfo r = parse_hdr(tv, (uint64_t)(lo + (int64_t)S.last_off));
                if (r.ok && is_long(r) && r.ve > vhi) {
                    S.has_carry = 1; S.c_vb = r.vb; S.c_ve = r.ve;
                    S.c_idx = S.pool_base + S.tile_count - 1u;
                } else {
                    S.has_carry = 0;
                }
            } else if (S.has_carry && S.c_ve <= vhi) {
                S.has_carry = 0;
            }
            if (S.err_pos != NONE) S.stop = 1;
            else if (found && S.tile_exit == ERRP) {   // defensive: a broken chain must have reported
                S.stop = 1; S.err_pos = S.entry; S.err_kind = KVR_E_VAL;
            }
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
