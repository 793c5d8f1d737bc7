/*
 * kvr_kernels.hip — the replay kernels (gfx950).
 *
 *   k_replay   one workgroup per stripe: stage tiles in LDS, walk the framing of
 *              src/store/engine.rs:79-154 in parallel, CRC-32 every key and value
 *              (storage.rs:27 semantics), emit 32-B tuples into a pool.
 *   k_link     one workgroup: verify every stripe's speculated entry against its predecessor's
 *              exit, pick the first error in (segment, offset) order (engine.rs:55-56) and
 *              list the stripes that must be re-walked from their true entry.
 *   k_tsum / k_tscan / k_compact
 *              exclusive scan of per-tile tuple counts and a gather of the pool into the dense
 *              output in (segment, offset) order, with per-record CRC verification.
 *   k_gen_fill / k_gen_manifest
 *              device side of the synthetic generator (kvr_gen_common.h).
 */
#include "kvr_device.h"
#include "kvr_gen_common.h"

namespace kvr {

struct __align__(16) Piece {   // a run of value bytes inside the tile, LDS coordinates [a, b)
    uint32_t a, b;
    uint32_t init;              // CRC register before byte a (0xFFFFFFFF at a value's start)
    uint32_t acc;               // XOR of shifted non-final unit CRCs
    uint32_t tail;              // raw CRC of the final intersection
    uint32_t done;              // the value ends inside this tile
    uint64_t slot;              // pool index of the record's tuple
};

struct __align__(16) Smem {
    uint8_t  tile[TILE];
    uint32_t crc[16 * 256];
    uint32_t pw16[TILE / 16 + 4];
    uint32_t pw1[20];
    uint64_t sc_cand[NT], sc_exit[NT], sc_errpos[NT], sc_entry[NT];
    uint32_t sc_cnt[NT], sc_base[NT];
    Piece    pc[MAXP];
    int16_t  cov[NT], sin_[NT];
    int16_t  nxt[NT], nxt0[NT];
    uint8_t  reach[NT];
    uint64_t entry, tile_exit, open_v0, open_v1, open_slot, pool_base, err_pos, err_aux, stripe_entry;
    uint32_t open_state, has_open, err_kind, n_pieces, tile_count, total, search, stop, tile_found, pad;
};

// ---------------------------------------------------------------------------------------
// Stitching the speculated sub-chains (wave 0).
//
// Sub-chunk s was walked from its first plausible start cand[s] to exit[s] (the first record
// start at/after its end).  Entered at cand[s], the chain moves to the sub-chunk holding exit[s]
// — a consistent transition only if that sub-chunk's cand equals exit[s].  The true chain of the
// tile starts at the entry e in sub-chunk s0 = sub(e); its sub-chunks are the nodes reachable
// from s0 through consistent transitions, found by pointer jumping (8 doubling rounds over 256
// nodes).  If the path stops at an inconsistent transition (MM), the true entry of the next
// sub-chunk is known, so lane 0 re-walks it (and the following mismatching ones) from there
// and the stitch repeats.  Each repair fixes one more sub-chunk for good, so it terminates.
// ---------------------------------------------------------------------------------------
constexpr int16_t T_END = NT, T_ERR = NT + 1, T_MM = NT + 2;

__device__ __forceinline__ int sub_of(uint64_t x, int64_t lo) { return (int)(((int64_t)x - lo) / SC); }

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
    for (int d = 32; d >= 1; d >>= 1) {
        const int o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// lane 0: the true chain enters sub-chunk sub(y) at y; re-walk it and every following
// sub-chunk whose speculation disagrees with the true chain (bounded per call).
__device__ void repair(Smem &S, const TileView &tv, uint64_t y, uint64_t vhi) {
    const int64_t lo = tv.lo;
    for (int k = 0; k < 64; ++k) {
        const int t = sub_of(y, lo);
        const int64_t ce = lo + (int64_t)(t + 1) * SC;
        const uint64_t pe = (uint64_t)ce > vhi ? vhi : (uint64_t)ce;
        uint64_t ex, ep;
        const uint32_t cnt = walk_chain(tv, y, pe, &ex, &ep);
        S.sc_cand[t] = y;
        S.sc_exit[t] = ex;
        S.sc_errpos[t] = ep;
        S.sc_cnt[t] = cnt;
        if (ex == ERRP || ex >= vhi) return;
        if (S.sc_cand[sub_of(ex, lo)] == ex) return;   // back in step with the speculation
        y = ex;
    }
}

// Wave 0 stitches the 256 speculated sub-chains from the tile entry e (vlo <= e < vhi).
// Writes sc_entry / sc_base, S.tile_count and S.tile_exit, allocates the tile's pool range.
__device__ void stitch(Smem &S, const TileView &tv, uint64_t e, uint64_t vhi, Counters *ctr, uint64_t pool_cap) {
    const int lane = threadIdx.x;   // 0..63
    const int64_t lo = tv.lo;
    const int s0 = sub_of(e, lo);
    for (int guard = 0; guard < 2 * NT + 8; ++guard) {
        if (S.sc_cand[s0] != e) {                       // the entry itself was not speculated
            if (lane == 0) repair(S, tv, e, vhi);
            wave_sync_lds();
            continue;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            const uint64_t c = S.sc_cand[s], x = S.sc_exit[s];
            int16_t T;
            if (c == NONE || x >= vhi) T = (x == ERRP && c != NONE) ? T_ERR : T_END;
            else {
                const int t = sub_of(x, lo);
                T = (S.sc_cand[t] == x) ? (int16_t)t : T_MM;
            }
            S.nxt0[s] = T;
            S.nxt[s] = T;
            S.reach[s] = (s == s0) ? 1 : 0;
        }
        wave_sync_lds();
#pragma unroll 1
        for (int r = 0; r < 8; ++r) {                   // J <- J o J, reach <- reach U J(reach)
            int16_t jn[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int s = 4 * lane + j;
                const int16_t J = S.nxt[s];
                jn[j] = J < NT ? S.nxt[J] : J;
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
            if (lane == 0) repair(S, tv, S.sc_exit[smax], vhi);
            wave_sync_lds();
            continue;
        }
        // accepted: entries, record index bases, tile totals
        uint64_t ent[4];
        uint32_t c4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 4 * lane + j;
            const bool on = S.reach[s] != 0;
            ent[j] = on ? S.sc_cand[s] : NONE;
            c4[j] = on ? S.sc_cnt[s] : 0u;
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
            S.sc_entry[4 * lane + j] = ent[j];
            S.sc_base[4 * lane + j] = base;
            base += c4[j];
        }
        const uint32_t total = __shfl(inc, 63, 64);
        if (lane == 0) {
            S.tile_count = total;
            S.tile_exit = (Tl == T_ERR) ? ERRP : S.sc_exit[smax];
            const uint64_t pb = total ? atomicAdd(&ctr->pool_cursor, (unsigned long long)total) : 0ull;
            S.pool_base = pb;
            if (pb + total > pool_cap) atomicOr(&ctr->overflow, 1u);
        }
        return;
    }
    if (lane == 0) {   // unreachable: every round repairs one more sub-chunk for good (bug trap)
        S.tile_count = 0;
        S.tile_exit = ERRP;
        S.pool_base = 0;
        atomicOr(&ctr->overflow, 2u);
    }
}

// CRC contribution of unit u to piece j (see kvr_device.h header)
__device__ __forceinline__ void unit_crc(Smem &S, int j, int u) {
    Piece &P = S.pc[j];
    const int us = u * UNIT, ue = us + UNIT;
    const int s = (int)P.a > us ? (int)P.a : us;
    const int e = (int)P.b < ue ? (int)P.b : ue;
    if (s >= e) return;
    const bool last = (e == (int)P.b);
    const int wend = last ? (e & ~15) : e;
    uint32_t c = 0;
    int w = s & ~15;
    if (w < wend) {
        uint4 d = *reinterpret_cast<const uint4 *>(S.tile + w);
        const int k = s - w;   // leading bytes outside the piece: zero (no effect on a raw CRC)
        if (k > 0) {
            uint32_t m0 = k >= 4 ? 0u : (~0u << (8 * k));
            uint32_t m1 = k >= 8 ? 0u : (k <= 4 ? ~0u : (~0u << (8 * (k - 4))));
            uint32_t m2 = k >= 12 ? 0u : (k <= 8 ? ~0u : (~0u << (8 * (k - 8))));
            uint32_t m3 = k <= 12 ? ~0u : (~0u << (8 * (k - 12)));
            d.x &= m0; d.y &= m1; d.z &= m2; d.w &= m3;
        }
        c = slice16(c, d, S.crc);
        for (w += 16; w < wend; w += 16) c = slice16(c, *reinterpret_cast<const uint4 *>(S.tile + w), S.crc);
    }
    for (int x = s > wend ? s : wend; x < e; ++x) c = crc_byte(c, S.tile[x], S.crc);
    if (last) {
        P.tail = c;
    } else {
        const uint32_t bf = P.b & ~15u;
        const uint32_t m = S.pw16[(bf - (uint32_t)ue) >> 4];
        atomicXor(&P.acc, m == 0x80000000u ? c : gf_mul(c, m));
    }
}

__global__ __launch_bounds__(NT) void k_replay(const SegDesc *__restrict__ segs,
                                               const StripeDesc *__restrict__ stripes,
                                               StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                               kvr_tuple *__restrict__ pool, uint64_t pool_cap,
                                               Counters *ctr, const uint32_t *__restrict__ g_crc,
                                               const uint32_t *__restrict__ g_pw16,
                                               const uint32_t *__restrict__ g_pw1,
                                               const RedoEnt *__restrict__ redo,
                                               const LinkResult *__restrict__ link, int redo_mode) {
    __shared__ Smem S;
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

    for (int i = tid; i < 16 * 256; i += NT) S.crc[i] = g_crc[i];
    for (int i = tid; i <= TILE / 16; i += NT) S.pw16[i] = g_pw16[i];
    if (tid < 17) S.pw1[tid] = g_pw1[tid];
    if (tid == 0) {
        S.has_open = 0;
        S.err_kind = 0;
        S.err_pos = NONE;
        S.err_aux = 0;
        S.total = 0;
        S.stop = 0;
        uint64_t e;
        if (redo_mode) e = forced;
        else e = (sd.t_begin == 0) ? 0ull : NONE;
        S.search = (e == NONE);
        S.entry = e;
        S.stripe_entry = (e != NONE && e >= s_hi) ? NONE : e;
        if (e != NONE && e >= s_hi) S.stop = 2;   // imposed entry beyond the stripe: no record starts here
    }
    __syncthreads();

    uint32_t k = sd.t_begin;
    for (;; ++k) {
        const bool in_stripe = k < sd.t_end;
        if (S.stop) break;
        if (!in_stripe && !S.has_open) break;
        if (k >= sg.n_tiles) break;
        const int64_t lo = (int64_t)k * TILE - d0;
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        const TileView tv{sg.base, S.tile, len, lo};

        // 1. stage the tile: coalesced 16-B loads (only words that overlap the segment)
        {
            const uint8_t *abase = sg.base - d0 + (int64_t)k * TILE;
            uint4 v[TILE / 16 / NT];
#pragma unroll
            for (int i = 0; i < TILE / 16 / NT; ++i) {
                const int w = i * NT + tid;
                const int64_t pos = lo + 16 * (int64_t)w;
                if (pos + 16 > 0 && pos < (int64_t)len) v[i] = *reinterpret_cast<const uint4 *>(abase + 16 * w);
            }
#pragma unroll
            for (int i = 0; i < TILE / 16 / NT; ++i) {
                const int w = i * NT + tid;
                const int64_t pos = lo + 16 * (int64_t)w;
                if (pos + 16 > 0 && pos < (int64_t)len) *reinterpret_cast<uint4 *>(S.tile + 16 * w) = v[i];
            }
        }
        S.cov[tid] = -1;
        S.sin_[tid] = -1;
        if (tid == 0) {
            S.n_pieces = 0;
            S.tile_count = 0;
            S.tile_found = 0;
            S.tile_exit = S.entry;
            if (S.has_open) {   // value of a record opened in an earlier tile
                const uint64_t a = S.open_v0 > vlo ? S.open_v0 : vlo;
                const uint64_t b = S.open_v1 < vhi ? S.open_v1 : vhi;
                const bool done = S.open_v1 <= vhi;
                if (a < b) {
                    Piece &P = S.pc[0];
                    P.a = (uint32_t)(a - lo);
                    P.b = (uint32_t)(b - lo);
                    P.init = S.open_state;
                    P.acc = 0;
                    P.tail = 0;
                    P.done = done ? 1u : 0u;
                    P.slot = S.open_slot;
                    S.n_pieces = 1;
                } else if (done && S.open_slot < pool_cap) {
                    pool[S.open_slot].crc32 = ~S.open_state;
                }
                if (done) S.has_open = 0;
            }
        }
        __syncthreads();

        // 2. speculative sub-chains, 3. stitch (wave 0)
        const bool walk = in_stripe && (S.search || S.entry < vhi);
        if (walk) {
            const uint64_t lower = S.search ? vlo : S.entry;
            uint64_t cand = NONE, ex = NONE, ep = NONE;
            uint32_t cnt = 0;
            {
                const int64_t cs_i = lo + (int64_t)tid * SC, ce_i = cs_i + SC;
                uint64_t cs = cs_i < (int64_t)vlo ? vlo : (uint64_t)cs_i;
                const uint64_t ce = (uint64_t)ce_i > vhi ? vhi : (uint64_t)ce_i;
                if (cs < lower) cs = lower;
                if (cs < ce) {
                    cand = find_cand(tv, cs, ce);
                    if (cand != NONE) cnt = walk_chain(tv, cand, ce, &ex, &ep);
                }
            }
            S.sc_cand[tid] = cand;
            S.sc_exit[tid] = ex;
            S.sc_errpos[tid] = ep;
            S.sc_cnt[tid] = cnt;
            __syncthreads();
            if (tid < 64) {
                uint64_t e = S.entry;
                if (S.search) {   // the stripe's entry: the first plausible record start
                    uint64_t m = NONE;
                    for (int j = 0; j < 4; ++j) {
                        const uint64_t c = S.sc_cand[4 * tid + j];
                        if (c < m) m = c;
                    }
                    e = wave_min_u64(m);
                }
                if (e != NONE) {
                    stitch(S, tv, e, vhi, ctr, pool_cap);
                    if (tid == 0) {
                        S.tile_found = 1;
                        if (S.search) { S.search = 0; S.stripe_entry = e; }
                    }
                }
            }
            __syncthreads();
        }

        // 4. process the accepted records: exact checks, tuples, small CRCs, big pieces
        uint64_t my_err = NONE, my_aux = 0;
        uint32_t my_kind = 0;
        if (walk && S.tile_found) {
            uint64_t p = S.sc_entry[tid];
            if (p != NONE) {
                uint64_t slot = S.pool_base + S.sc_base[tid];
                const int64_t ce_i = lo + (int64_t)(tid + 1) * SC;
                const uint64_t ce = (uint64_t)ce_i > vhi ? vhi : (uint64_t)ce_i;
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
                    t.key_tag = ~crc_range(tv, ~0u, kb, klen, S.crc);
                    t.op = (uint8_t)op;
                    t.flags = 0;
                    t.reserved = 0;
                    uint64_t nx;
                    if (op == 0u) {
                        const uint64_t q = kb + klen;
                        if (len - q < 4) { my_err = p; my_kind = KVR_E_VAL_LEN; break; }         // engine.rs:121
                        const uint64_t vlen = tv.rd32(q);
                        const uint64_t vb = q + 4, ve = vb + vlen;
                        if (len - vb < vlen) { my_err = p; my_kind = KVR_E_VAL; break; }         // engine.rs:130
                        t.val_len = (uint32_t)vlen;
                        t.crc32 = 0;
                        if (ve <= vhi && vlen <= (uint64_t)SMALL) {
                            t.crc32 = ~crc_range(tv, ~0u, vb, vlen, S.crc);
                        } else {
                            if (vb < vhi) {
                                const uint32_t pj = atomicAdd(&S.n_pieces, 1u);
                                Piece &P = S.pc[pj];
                                P.a = (uint32_t)(vb - lo);
                                P.b = (uint32_t)((ve < vhi ? ve : vhi) - lo);
                                P.init = ~0u;
                                P.acc = 0;
                                P.tail = 0;
                                P.done = ve <= vhi ? 1u : 0u;
                                P.slot = slot;
                            }
                            if (ve > vhi) {   // the value continues in the next tile(s)
                                S.open_v0 = vb;
                                S.open_v1 = ve;
                                S.open_slot = slot;
                                S.open_state = ~0u;
                                S.has_open = 1;
                            }
                        }
                        nx = ve;
                    } else {
                        t.val_len = 0;
                        t.crc32 = 0;
                        nx = kb + klen;
                    }
                    if (slot < pool_cap) pool[slot] = t;
                    ++slot;
                    p = nx;
                }
                if (my_err != NONE) atomicMin(reinterpret_cast<unsigned long long *>(&S.err_pos), (unsigned long long)my_err);
            }
        }
        __syncthreads();
        if (my_err != NONE && my_err == S.err_pos) {
            S.err_kind = my_kind;
            S.err_aux = my_aux;
        }
        // 5. big pieces: unit map, unit CRCs, combine
        const uint32_t np = S.n_pieces;
        if (np) {
            if ((uint32_t)tid < np) {
                const Piece &P = S.pc[tid];
                const int u0 = (int)P.a / UNIT, u1 = (int)(P.b - 1) / UNIT;
                for (int u = u0; u <= u1; ++u) {
                    if (u == u0 && (int)P.a > u * UNIT) S.sin_[u] = (int16_t)tid;
                    else S.cov[u] = (int16_t)tid;
                }
            }
            __syncthreads();
            const int j0 = S.cov[tid], j1 = S.sin_[tid];
            if (j0 >= 0) unit_crc(S, j0, tid);
            if (j1 >= 0) unit_crc(S, j1, tid);
            __syncthreads();
            if ((uint32_t)tid < np) {
                const Piece &P = S.pc[tid];
                uint32_t st = P.tail;
                if (P.acc) st ^= gf_mul(P.acc, S.pw1[P.b & 15u]);
                if (P.init) {
                    const uint32_t n = P.b - P.a;
                    st ^= gf_mul(P.init, gf_mul(S.pw16[n >> 4], S.pw1[n & 15u]));
                }
                if (P.done) {
                    if (P.slot < pool_cap) pool[P.slot].crc32 = ~st;
                } else {
                    S.open_state = st;
                }
            }
        }
        __syncthreads();
        if (tid == 0) {
            if (in_stripe) {
                tres[sg.tile0 + k].pool_off = S.tile_count ? S.pool_base : 0ull;
                tres[sg.tile0 + k].count = S.tile_count;
                S.total += S.tile_count;
                if (walk && S.tile_found) S.entry = S.tile_exit;
            }
            if (S.err_pos != NONE) S.stop = 1;
            else if (in_stripe && walk && S.tile_found && S.tile_exit == ERRP) {   // defensive
                S.stop = 1; S.err_pos = S.entry; S.err_kind = KVR_E_VAL;
            }
        }
        __syncthreads();
    }
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

// ---------------------------------------------------------------------------------------
// k_link — one workgroup of 1024 threads.
// ---------------------------------------------------------------------------------------
constexpr int LT = 1024;

__device__ __forceinline__ uint64_t stripe_hi(const StripeDesc &d, const SegDesc &g) {
    const int64_t h = (int64_t)d.t_end * TILE - (int64_t)g.d0;
    return (uint64_t)h > g.len ? g.len : (uint64_t)h;
}

__global__ __launch_bounds__(LT) void k_link(const SegDesc *__restrict__ segs, uint32_t n_segs,
                                             const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                             const StripeRes *__restrict__ sres, RedoEnt *__restrict__ redo,
                                             uint32_t redo_cap, LinkResult *res, uint32_t *seg_bad,
                                             uint32_t *seg_err) {
    __shared__ int32_t cm[LT];
    __shared__ uint32_t first_problem, nredo;
    const int tid = threadIdx.x;
    for (uint32_t g = tid; g < n_segs; g += LT) { seg_bad[g] = ~0u; seg_err[g] = ~0u; }
    if (tid == 0) { first_problem = ~0u; nredo = 0; }
    const uint32_t per = (n_stripes + LT - 1) / LT;
    const uint32_t b = tid * per, e = min(b + per, n_stripes);
    int32_t m = -1;
    for (uint32_t s = b; s < e; ++s) if (sres[s].entry != NONE) m = (int32_t)s;
    cm[tid] = m;
    __syncthreads();
    for (int d = 1; d < LT; d <<= 1) {   // inclusive max-scan of chunk maxima
        const int32_t o = tid >= d ? cm[tid - d] : -1;
        __syncthreads();
        if (o > cm[tid]) cm[tid] = o;
        __syncthreads();
    }
    const int32_t run0 = tid ? cm[tid - 1] : -1;

    // pass 1: consistency of every stripe with its predecessor's exit
    int32_t run = run0;
    for (uint32_t s = b; s < e; ++s) {
        const StripeRes r = sres[s];
        const StripeDesc d = stripes[s];
        const SegDesc g = segs[d.seg];
        const bool first = (s == g.stripe0);
        bool bad = false, after_err = false;
        if (!first) {
            const uint64_t xp = run >= 0 ? sres[run].exit : NONE;
            if (xp == ERRP) after_err = true;
            else if (r.entry == NONE) bad = xp < stripe_hi(d, g);
            else bad = (r.entry != xp);
        }
        if (bad && !after_err) atomicMin(&seg_bad[d.seg], s);
        if (r.err_kind != 0 && !after_err && !bad) atomicMin(&seg_err[d.seg], s);
        if (r.entry != NONE) run = (int32_t)s;
    }
    __syncthreads();
    for (uint32_t g = tid; g < n_segs; g += LT) {
        const uint32_t bb = __hip_atomic_load(&seg_bad[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t ee = __hip_atomic_load(&seg_err[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (bb != ~0u || ee != ~0u) atomicMin(&first_problem, g);
    }
    __syncthreads();
    const uint32_t fp = first_problem;
    bool unresolved = false;
    uint32_t fbad = ~0u, ferr = ~0u;
    if (fp != ~0u) {
        fbad = __hip_atomic_load(&seg_bad[fp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ferr = __hip_atomic_load(&seg_err[fp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unresolved = fbad < ferr;
    }
    // pass 2: re-walk list (stripes whose entry disagrees with the true chain so far)
    if (unresolved) {
        run = run0;
        for (uint32_t s = b; s < e; ++s) {
            const StripeRes r = sres[s];
            const StripeDesc d = stripes[s];
            const SegDesc g = segs[d.seg];
            if (d.seg <= fp && s != g.stripe0) {
                const uint64_t xp = run >= 0 ? sres[run].exit : NONE;
                bool bad = false;
                if (xp != ERRP) {
                    if (r.entry == NONE) bad = xp < stripe_hi(d, g);
                    else bad = (r.entry != xp);
                }
                const uint32_t se = __hip_atomic_load(&seg_err[d.seg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (bad && s < se) {
                    const uint32_t i = atomicAdd(&nredo, 1u);
                    if (i < redo_cap) { redo[i].stripe = s; redo[i].pad = 0; redo[i].entry = xp; }
                }
            }
            if (r.entry != NONE) run = (int32_t)s;
        }
    }
    __syncthreads();
    if (tid == 0) {
        LinkResult L;
        L.first_problem_seg = fp;
        L.n_redo = nredo < redo_cap ? nredo : redo_cap;
        L.passes = res->passes + 1;
        L.err_kind = 0; L.err_seg = 0; L.err_pos = 0; L.err_aux = 0;
        if (fp == ~0u) {
            L.status = 0;
        } else if (unresolved) {
            L.status = 3;
        } else {
            const StripeRes r = sres[ferr];
            L.status = 1;
            L.err_kind = r.err_kind;
            L.err_seg = fp;
            L.err_pos = r.err_pos;
            L.err_aux = r.err_aux;
        }
        *res = L;
    }
}

// ---------------------------------------------------------------------------------------
// Scan of per-tile counts and the ordered gather pool -> out.
// ---------------------------------------------------------------------------------------
constexpr int CT = 256;           // threads per compaction block
constexpr int CPT = 4;            // tiles per thread
constexpr int CB = CT * CPT;      // tiles per compaction block

__global__ __launch_bounds__(CT) void k_tsum(const TileRes *__restrict__ tres, uint32_t n_tiles,
                                             uint64_t *__restrict__ bsum, const LinkResult *__restrict__ link) {
    if (link->status != 0) return;
    __shared__ uint64_t red[CT];
    const uint32_t t0 = blockIdx.x * CB + threadIdx.x * CPT;
    uint64_t s = 0;
    for (int i = 0; i < CPT; ++i) if (t0 + i < n_tiles) s += tres[t0 + i].count;
    red[threadIdx.x] = s;
    __syncthreads();
    for (int d = CT / 2; d > 0; d >>= 1) {
        if (threadIdx.x < d) red[threadIdx.x] += red[threadIdx.x + d];
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(1024) void k_tscan(uint64_t *__restrict__ bsum, uint32_t nb, Counters *ctr,
                                                const LinkResult *__restrict__ link) {
    if (link->status != 0) return;
    __shared__ uint64_t sh[1024];
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? bsum[i] : 0ull;
        sh[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < 1024; d <<= 1) {
            const uint64_t o = threadIdx.x >= (uint32_t)d ? sh[threadIdx.x - d] : 0ull;
            __syncthreads();
            sh[threadIdx.x] += o;
            __syncthreads();
        }
        if (i < nb) bsum[i] = carry + sh[threadIdx.x] - v;   // exclusive
        const uint64_t tot = sh[1023];
        __syncthreads();
        carry += tot;
    }
    if (threadIdx.x == 0) ctr->total_tuples = carry;
}

__global__ __launch_bounds__(CT) void k_compact(const TileRes *__restrict__ tres, uint32_t n_tiles,
                                                const uint64_t *__restrict__ bsum,
                                                const kvr_tuple *__restrict__ pool, uint64_t pool_cap,
                                                kvr_tuple *__restrict__ out, uint64_t out_cap,
                                                const uint32_t *__restrict__ expected, uint64_t n_expected,
                                                Counters *ctr, const LinkResult *__restrict__ link) {
    if (link->status != 0 || ctr->overflow) return;
    __shared__ uint64_t off[CB + 1];
    __shared__ uint64_t part[CT];
    const uint32_t tb = blockIdx.x * CB;
    uint64_t loc[CPT];
    uint64_t s = 0;
    for (int i = 0; i < CPT; ++i) {
        const uint32_t t = tb + threadIdx.x * CPT + i;
        loc[i] = s;
        s += t < n_tiles ? tres[t].count : 0u;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < CT; d <<= 1) {
        const uint64_t o = threadIdx.x >= (uint32_t)d ? part[threadIdx.x - d] : 0ull;
        __syncthreads();
        part[threadIdx.x] += o;
        __syncthreads();
    }
    const uint64_t base = bsum[blockIdx.x] + part[threadIdx.x] - s;
    for (int i = 0; i < CPT; ++i) off[threadIdx.x * CPT + i] = base + loc[i];
    __syncthreads();
    // one wave per tile: lanes move whole 32-B tuples
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t fails = 0;
    for (int i = wave; i < CB; i += CT / 64) {
        const uint32_t t = tb + i;
        if (t >= n_tiles) break;
        const uint32_t cnt = tres[t].count;
        const uint64_t src = tres[t].pool_off, dst = off[i];
        for (uint32_t j = lane; j < cnt; j += 64) {
            if (src + j >= pool_cap) continue;
            kvr_tuple tp = pool[src + j];
            const uint64_t o = dst + j;
            if (expected && o < n_expected && tp.op == 0) {
                tp.flags |= KVR_TF_VERIFIED;
                if (expected[o] != tp.crc32) { tp.flags |= KVR_TF_CRC_FAIL; ++fails; }
            }
            if (o < out_cap) out[o] = tp;
        }
    }
    for (int d = 32; d >= 1; d >>= 1) fails += __shfl_xor(fails, d, 64);
    if (lane == 0 && fails) atomicAdd(&ctr->crc_fail, (unsigned long long)fails);
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
