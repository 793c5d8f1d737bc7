/*
 * kvr_replay_kernel.hip — k_replay, the hot path (gfx950).
 *
 * One WAVE replays one stripe (consecutive 8-KiB tiles of one segment) exactly as
 * src/store/engine.rs:79-154 walks a segment file, and emits one 32-B kvr_tuple per record with
 * the CRC-32 of its key and of its value (crc32fast::hash semantics, src/volume/storage.rs:27).
 * A workgroup holds 16 independent stripes that share the CRC tables; after the tables are staged
 * there is no workgroup barrier.
 *
 * Per tile, lane l owns the 128-B unit [128 l, 128 l + 128), held in 32 registers; the next tile's
 * load goes into the same registers as soon as the CRC phase is done with them.
 *   F  framing, lane-parallel: stride prediction, verified.  Lane j decodes the
 *      record that would start at entry + j L (L = the last record's length) from a window of
 *      the segment bytes: opcode, key length, value length, every engine.rs framing check, and
 *      where its successor starts.  The first lane whose record is broken or whose successor is
 *      not the next prediction ends the round; the records before it and its own are the exact
 *      chain.  Equal-sized records (the benchmark shapes) take one round per tile; a broken
 *      record, varying lengths or a segment more than 2 GiB past the tile continue in the exact
 *      scalar hop loop (on the CU's scalar unit), which also reports the error of a broken
 *      record with every engine.rs check in engine.rs order.
 *      Only a stripe's first tile guesses: it takes its first plausible record start, which
 *      k_link checks against the previous stripe's exit (a wrong guess is re-walked).
 *   R  records: the lanes on the chain emit their record in parallel: the UTF-8 check of the key
 *      (engine.rs:114), the key CRC and the CRC of a value of at most 64 B or lying inside one
 *      unit, from the window the decode already holds.
 *   C  long values: each lane CRCs its unit from registers in two independent chains, with a
 *      snapshot where a value ends and a restart where one starts; a segmented XOR scan across
 *      the wave (DPP only, each piece first pushed to its consumer with x^(8*128*d) from a
 *      per-lane column of nibble tables) gives the CRC register at every unit boundary; the lane
 *      holding a value's last byte finishes that CRC.  A value running past the tile hands its
 *      register to the next tile of the stripe, so no variable GF(2) multiply is needed.
 *
 * CRC tables: slice-by-4 byte tables replicated per LDS bank group (see Crc), so no lookup of a
 * wave ever conflicts and its address is a single v_perm_b32 of the register byte and a lane
 * constant.
 */
#include "kvr_device.h"
#include <type_traits>

namespace kvr {

// threads per workgroup: 16 stripes, one per wave.  The 32 tile registers leave room for four
// waves per SIMD (under 128 VGPRs) when the next tile is loaded into the same registers once the
// current one is done with (no separate prefetch buffer)
#ifndef KVR_RT
#define KVR_RT 1024
#endif
constexpr int RT = KVR_RT;
constexpr int NWAVE = RT / 64;            // waves per workgroup
constexpr int WPB = NWAVE;                // stripes per workgroup (one per wave)
constexpr int RT_REWALK = RT / 2;         // k_rewalk's workgroup
constexpr int UW = SC / 4;                // dwords of a lane's unit
constexpr int SC_LOG = 7;
static_assert(SC == 1 << SC_LOG, "unit size");
static_assert(TILE == 64 * SC, "one unit per lane");
static_assert(UW == 32, "unit = 32 dwords");
static_assert(TILE == 1 << 13, "tile of a segment position: (pos + d0) >> 13 (the piece mode)");
constexpr uint32_t N32 = 0xFFFFFFFFu;
constexpr uint32_t POOL_CHUNK = 2048;     // pool slots a wave claims at once
constexpr uint32_t TILE_RECS = TILE / 5 + 1;   // most record starts a tile can hold
static_assert(POOL_CHUNK >= TILE_RECS, "the rest of a tile's records fits in one fresh chunk");
constexpr int32_t FAR = 1 << 30;          // "ends beyond the tile" (tile-relative clamp)
constexpr int KEYW = 6;                   // key words the record fast path reads at once (<= 24 B)
constexpr int VALW = SMALL / 4;           // value words of a short value
constexpr int WINW = KEYW + 3;            // decode window: dwords from the candidate's aligned word

// Every table starts below 64 KiB, or is reached through a perm-built address that carries the
// 64-KiB bit: a lookup is then one address VGPR plus a constant the ds_read instruction carries as
// its 16-bit immediate offset, with no add (the byte tables C2 are the hot ones: 4 lookups a word).
constexpr int KR_PITCH = 66;              // KR's row pitch in dwords (see kmul_col)
#ifndef KVR_KQLPAD   // 1: KQL's rows padded like KR's (0: 64 dwords, one v_perm a lookup)
#define KVR_KQLPAD 1
#endif
constexpr int KQL_PITCH = KVR_KQLPAD ? KR_PITCH : 64;
struct __align__(16) Smem {
    uint32_t KQ2[2 * 8 * 16];             // [h][i][n]: (n << 4i) * x^(8*4q), q = SC/8 (h 0), SC/4 (h 1): the two
                                          // lane-uniform pushes of the finalize
    uint32_t KQ4[2 * 8 * 16];             // the same for x^(8*32) (h 0) and x^(8*96) (h 1): k_piece's 4-chain combine
    uint32_t IX[NIX + 3];                 // 0xFFFFFFFF * x^(8j): initial register pushed through j bytes
    uint32_t MK[NWAVE][64];               // per wave: long-value marks by unit (framing)
    uint32_t BAL[4];                      // the workgroup's progress sum and wave count (KVR_PBAL / KVR_RBAL)
    uint32_t C2[256 * 64];                // byte tables, row b = 256 B (64 KiB), see Crc
    uint32_t KR[8 * 16 * KR_PITCH];       // [i][n][k]: (n << 4i) * x^(8*SC*(k+1)), k < 64  (above 64 KiB,
    uint32_t KQL[8 * 16 * KQL_PITCH];     // [i][n][q]: (n << 4i) * x^(8*4q), q per lane (columns > SC/4: 0)  see kmul_col)
};
constexpr uint32_t KR_OFF = (uint32_t)offsetof(Smem, KR), KQL_OFF = (uint32_t)offsetof(Smem, KQL);
// k_piece's LDS: the tables it reads (no KQL, no MK) and, per wave, the header windows of
// the records in its group (WROW[wave][dword][lane]: lane j holds record qg + j's window, written when
// it has landed, read back by the group's flush), so the windows hold no registers across the CRC
#ifndef KVR_PWMAX   // k_piece's waves per workgroup the LDS is laid out for
#define KVR_PWMAX 16
#endif
constexpr int PWIN = 13;                  // dwords of a header window (48 B from its first byte, realigned)
struct __align__(16) SmemP {
    uint32_t KQ2[2 * 8 * 16];
    uint32_t KQ4[2 * 8 * 16];
    uint32_t IX[NIX + 3];
    uint32_t BAL[4];
    uint32_t C2[256 * 64];
    uint32_t KR[8 * 16 * KR_PITCH];
    uint32_t WROW[KVR_PWMAX][PWIN][64];
};
constexpr uint32_t KR_OFF_P = (uint32_t)offsetof(SmemP, KR);
static_assert(offsetof(SmemP, C2) < 65536 && KR_OFF_P >= 65536, "k_piece's tables: ds_read immediates, kmul_col's 64-KiB bit");
static_assert(offsetof(SmemP, WROW) % 16 == 0, "k_piece's window rows: 16-B slots (KVR_PWDMA)");
static_assert(sizeof(SmemP) <= 163840, "k_piece's LDS");
static_assert(offsetof(Smem, C2) < 65536, "the byte tables' base fits a ds_read immediate");
static_assert(KR_OFF >= 65536 && KQL_OFF - 65536 < 65536, "kmul_col's 64-KiB bit");

// wave priority (s_setprio) of the serial phases: the framing and the records phase are the
// tile's critical path and share the CU with 15 other waves, so they issue ahead of waves in
// their bulk CRC; the scan + finalize chain is raised too
// (0 with KVR_RBAL 2: the progress balance sets the priority, one level for every phase)
#ifndef KVR_HOP_PRIO
#define KVR_HOP_PRIO 0
#endif
#ifndef KVR_REC_PRIO
#define KVR_REC_PRIO 0
#endif
#ifndef KVR_FIN_PRIO
#define KVR_FIN_PRIO 0
#endif
// k_replay's progress balance (as k_piece's KVR_PBAL): 2 = four priority levels from the wave's
// progress against its workgroup's mean, per tile (cfg4 -3 %, cfg5 -3.5 % against none); 1 = the
// phase priorities above, one level up for a wave behind the mean
#ifndef KVR_RBAL
#define KVR_RBAL 2
#endif
#define KVR_SETPRIO(p)                                                                   \
    do {                                                                                 \
        if (KVR_RBAL && rbal_up) __builtin_amdgcn_s_setprio((p) + 1 > 3 ? 3 : (p) + 1); \
        else __builtin_amdgcn_s_setprio(p);                                              \
    } while (0)
#ifndef KVR_LANEFRAME   // 1: lane-parallel framing (0: the exact scalar hop loop for every record)
#define KVR_LANEFRAME 1
#endif
#ifndef KVR_PSEL   // 1: per-lane v_perm selectors pick each lane group's byte (no rotation of x per step)
#define KVR_PSEL 1
#endif
#ifndef KVR_CANDFRAME   // 1: candidate-chain rounds for what the stride round leaves (records of varying lengths)
#define KVR_CANDFRAME 1
#endif
#ifndef KVR_UMODE   // 1: runs of SETs of one key and one value length go through the piece mode (uniform_run)
#define KVR_UMODE 1
#endif
#ifndef KVR_PCHAINS   // k_piece's CRC chains per piece: 2 (16 words each) or 4 (8 words each)
#define KVR_PCHAINS 2
#endif
#ifndef KVR_PABLATE   // diagnostic builds of k_piece only (results wrong): 1 no CRC, 2 no push + scan, 8 no
#define KVR_PABLATE 0   // realignment, 16 no verification or emission (flush only advances), 32 window loads
                        // past the resource (no memory access), 64 no window load instructions (32, 64 only with 16),
                        // 128 no tuple stores, 256 no key CRC, 512 every record as predicted, 1024 no window reads
                        // from LDS (with 512)
#endif
#ifndef KVR_PBAL   // k_piece: 1 = wave priorities from each wave's progress against its workgroup's mean
#define KVR_PBAL 1     // (without, oldest-first issue finishes a CU's 16 stripes in 4 waves of 4)
#endif
#ifndef KVR_PBAL_EVERY   // k_piece: steps between two balance updates (a power of two)
#define KVR_PBAL_EVERY 1
#endif
#ifndef KVR_PBAL_D   // the progress band (1/4096 of a run) around the mean of priorities 1 and 2
#define KVR_PBAL_D 64
#endif
#ifndef KVR_PSEARCH   // k_piece: tiles it searches for the stripe's entry before handing the search on
#define KVR_PSEARCH 16
#endif
#ifndef KVR_PCHECK   // k_piece: records whose headers are checked before a run starts (1: none)
#define KVR_PCHECK 8
#endif
#ifndef KVR_UMIN    // the shortest value the piece mode takes (pieces are 128 B: shorter values waste lanes)
#define KVR_UMIN 128
#endif
constexpr uint32_t UMAXV = 1u << 24;     // the piece mode's longest value (window offsets stay in 32 bits)
constexpr int UKEYW = 9;                 // ... and longest key: 4 UKEYW bytes, in the 48-B header window
#ifndef KVR_SUCC   // 1: the candidate chain follows precomputed successor slots (0: a ballot per record)
#define KVR_SUCC 1
#endif
#ifndef KVR_TOPWAIT   // 1: wait for the tile's load at the top of the loop (0: where its registers are
#define KVR_TOPWAIT 0   // first read, so the framing round's window loads go out under the tile's load;
#endif                  // cfg2 1.326-1.332 vs 1.334-1.342 ms, cfg4 1.805-1.819 vs 1.813-1.857, medians)
#ifndef KVR_UNIFOLD   // 1: a stride round of equal SETs folds its long values into the units by arithmetic
#define KVR_UNIFOLD 1
#endif
#ifndef KVR_FAST_BACKOFF   // tiles the scalar hop loop keeps after a lane-parallel round found < 3 records
#define KVR_FAST_BACKOFF 16   // (4: cfg4 1.80 ms; 16: 1.75 with the loop-top change, r03_topwait_backoff_ab.txt)
#endif
#ifndef KVR_ABLATE
#define KVR_ABLATE 0   // diagnostic builds only: 1 skip records, 2 skip value CRC, 4 skip framing,
#endif                 // 8 skip the unit loop, 16 skip scan + finalize, 32 skip long-value folding,
                       // 64 loads only

#ifdef KVR_PROF
__device__ unsigned long long g_prof[16];
#ifdef KVR_PROF
__device__ unsigned long long g_pst[4 * 16384];   // (k_piece, per stripe: start, end, HW_ID, XCC_ID)
#endif
#define KVR_STAMP(i)                                                        \
    do {                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
        prof_acc[i] += t_ - t_last;                                         \
        t_last = t_;                                                        \
    } while (0)
#else
#define KVR_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ uint64_t uni64(uint64_t v) {   // wave-uniform value into SGPRs
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// lane l's value, l wave-uniform (v_readlane: no LDS traffic, unlike a shuffle)
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
// old with lane l set to the uniform val (v_writelane_b32: one VALU instruction, no compare/select)
__device__ __forceinline__ uint32_t wl32(uint32_t old, uint32_t val, uint32_t l) {
    val = __builtin_amdgcn_readfirstlane(val);
    asm("" : "+s"(val));   // (an SGPR even when val is a known constant: v_writelane takes no literal)
    asm("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(val), "{m0}"(l));   // lane select through m0
    return old;
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {   // (readlane returns int: widen as unsigned)
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
}

// DPP move (no LDS): CTRL = row_shr:d (0x110 + d), row_bcast:15 (0x142), row_bcast:31 (0x143),
// wave_shr:1 (0x138), wave_shl:1 (0x130); lanes without a source read 0
template <int CTRL, int ROWS = 0xF, bool BC = true>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, BC);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {   // (every lane gets the maximum)
    v = __builtin_elementwise_max(v, dpp<0x111>(v));
    v = __builtin_elementwise_max(v, dpp<0x112>(v));
    v = __builtin_elementwise_max(v, dpp<0x114>(v));
    v = __builtin_elementwise_max(v, dpp<0x118>(v));
    v = __builtin_elementwise_max(v, dpp<0x142, 0xA, false>(v));
    v = __builtin_elementwise_max(v, dpp<0x143, 0xC, false>(v));
    return rl32(v, 63);
}

__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {   // inclusive prefix sum over the lanes
    v += dpp<0x111>(v);
    v += dpp<0x112>(v);
    v += dpp<0x114>(v);
    v += dpp<0x118>(v);
    v += dpp<0x142, 0xA, false>(v);
    v += dpp<0x143, 0xC, false>(v);
    return v;
}

// Record-start candidates of a lane's unit w (SWAR over its 32 registers): byte b of word i is one
// when it is an opcode byte (0x00 / 0x01) and the byte 4 on -- the top byte of the key length that
// would follow -- does not exceed the top byte of rem (the segment bytes left from the tile start;
// a necessary condition for a valid record, engine.rs:96-107).  cm[g] bit 8 b + j: byte b of word
// 8 g + j, i.e. unit offset 32 g + 4 j + b.  (The unit's last word is not bounded by its next.)
__device__ __forceinline__ void cand_masks(const uint32_t (&w)[UW], int64_t rem, uint32_t (&cm)[4]) {
    const int32_t rc = rem > 0x7FFFFFFFll ? 0x7FFFFFFF : (int32_t)rem;
    const uint32_t addT = (0x7Fu - ((uint32_t)rc >> 24)) * 0x01010101u;
    cm[0] = cm[1] = cm[2] = cm[3] = 0u;
#pragma unroll
    for (int i = 0; i < UW; ++i) {
        // bit 7 of a byte: the byte is 0x00 / 0x01 (no carry leaves a byte: (b & 0x7E) + 0x7F <= 0xFD)
        uint32_t z = ~(((w[i] & 0x7E7E7E7Eu) + 0x7F7F7F7Fu) | w[i] | 0x7F7F7F7Fu);
        if (i + 1 < UW) {                              // bytes above the bound set their 0x80 bit
            const uint32_t x = w[i + 1];
            z &= ~((((x & 0x7F7F7F7Fu) + addT) | x));
        }
        cm[i >> 3] |= z >> (7 - (i & 7));
    }
}
// The candidate rounds' filter (cheaper, not a necessary condition): the opcode byte and the byte 4
// on (the key length's top byte) are both 0x00 / 0x01, i.e. (w | x) & 0xFE is a zero byte: four
// VALU a word, the accumulation two words at a time.  A record whose key is 32 MiB or longer is not
// a candidate, so the chain stops there and the exact loop walks it.  Same layout as cand_masks.
__device__ __forceinline__ void cand_masks_fast(const uint32_t (&w)[UW], uint32_t (&cm)[4]) {
    cm[0] = cm[1] = cm[2] = cm[3] = 0u;
    uint32_t z[UW];
#pragma unroll
    for (int i = 0; i < UW; ++i) {
        const uint32_t x = i + 1 < UW ? w[i + 1] : 0u;   // (the unit's last word: its opcode bytes only)
        const uint32_t v = (w[i] | x) & 0xFEFEFEFEu;                   // (one v_bitop3 each)
        const uint32_t t = ((w[i] | x) & 0x7E7E7E7Eu) + 0x7F7F7F7Fu;
        z[i] = ~(t | v | 0x7F7F7F7Fu);   // bit 7 of a byte: (w | x) & 0xFE is zero there
    }
#pragma unroll
    for (int i = 0; i < UW; i += 2)
        cm[i >> 3] |= (z[i] >> (7 - (i & 7))) | (z[i + 1] >> (7 - ((i + 1) & 7)));
}
// keep only the candidates at unit offsets below lim (any lim; <= 0 clears all)
__device__ __forceinline__ void mask_from(uint32_t (&cm)[4], int32_t lim) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        uint32_t mk = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {   // offsets 32 g + 4 j + b < lim  <=>  j < ceil((lim - 32 g - b) / 4)
            int32_t nj = (lim - 32 * g - b + 3) >> 2;
            nj = nj < 0 ? 0 : (nj > 8 ? 8 : nj);
            mk |= ((1u << nj) - 1u) << (8 * b);
        }
        cm[g] &= mk;
    }
}

// ---------------------------------------------------------------------------------------
// CRC primitives
// ---------------------------------------------------------------------------------------
// Row b of Smem::C2 (64 dwords):
//   [0, 32):  dword 8 t + r = table t (t = 0: one byte, t = k: a byte then k zero bytes) for byte
//             b, replica r < 8 -- the slice-by-4 set
//   [32, 64): table 0, replica lane & 31 (single-byte steps: a half-wave's 32 lanes in 32 banks)
// A slice-by-4 step x = c ^ w needs T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3].  Lane group
// g = (lane >> 3) & 3 takes table (g + i) & 3 in its i-th lookup and replica lane & 7, so the 32
// lanes of a half-wave hit 32 distinct banks in every lookup; the group's byte order is absorbed
// by rotating x left by 8 g first (one v_alignbit), which keeps the four selectors uniform.
struct Crc {
    const uint8_t *t;   // Smem::C2
    uint32_t L;         // byte 0: T0 copy, 128 + 4 (lane & 31)
    uint32_t L4;        // byte i: 4 (8 ((g + i) & 3) + (lane & 7)), this lane's i-th slice-by-4 lookup
#if KVR_PSEL
    uint32_t sel[4];    // lookup i's v_perm selector: byte 0 = L4's byte i, byte 1 = x's byte 3 - ((g + i) & 3)
#else
    uint32_t rot;       // (32 - 8 g) & 31: x rotated right by this = x rotated left by 8 g
#endif
};
// the C2 entry (dword) of LDS row b, column d: which table it holds (the staging loops)
__host__ __device__ constexpr int c2_table(int d) { return d < 32 ? (d >> 3) : 0; }
__device__ __forceinline__ void crc_init(Crc &K, const uint32_t *C2, uint32_t lane) {
    const uint32_t g = (lane >> 3) & 3u, r = lane & 7u, r32 = lane & 31u;
    K.t = reinterpret_cast<const uint8_t *>(C2);
    K.L = 128u + 4u * r32;
    K.L4 = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) K.L4 |= (4u * (8u * ((g + i) & 3u) + r)) << (8 * i);
#if KVR_PSEL
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) K.sel[i] = 0x0C0C0000u | ((7u - ((g + i) & 3u)) << 8) | i;
#else
    K.rot = (32u - 8u * g) & 31u;
#endif
}
// the byte order a lookup selector expects: x itself (KVR_PSEL) or x rotated left by 8 g
__device__ __forceinline__ uint32_t crc_rot(uint32_t x, const Crc &k) {
#if KVR_PSEL
    (void)k;
    return x;
#else
    return __builtin_amdgcn_alignbit(x, x, k.rot);
#endif
}
__device__ __forceinline__ uint32_t crc_sel(const Crc &k, uint32_t i) {
#if KVR_PSEL
    return k.sel[i];
#else
    (void)k;
    return 0x0C0C0000u | ((7u - i) << 8) | i;
#endif
}
// v_perm_b32 builds the LDS address: byte 1 = a byte of x, byte 0 = this lane's table copy
constexpr uint32_t SEL_T0_B0 = 0x0C0C0400u;
__device__ __forceinline__ uint32_t tget(const Crc &k, uint32_t x, uint32_t sel) {
    return *reinterpret_cast<const uint32_t *>(k.t + __builtin_amdgcn_perm(x, k.L, sel));
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {   // one VALU op
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));   // a ^ b ^ c
    return r;
}
// lookup i of a slice-by-4 step on xr = x rotated left by 8 g: byte 1 = xr byte 3 - i, which
// is x byte 3 - ((g + i) & 3), the byte table (g + i) & 3 takes
__device__ __forceinline__ uint32_t s4get(const Crc &k, uint32_t xr, uint32_t i) {
    return *reinterpret_cast<const uint32_t *>(k.t + __builtin_amdgcn_perm(xr, k.L4, crc_sel(k, i)));
}
// (the four lookups are issued before any is used: the empty asm keeps the scheduler from
// serialising them; it is not volatile, so independent chains still interleave around it)
__device__ __forceinline__ uint32_t crc4(uint32_t c, uint32_t w, const Crc &k) {
    const uint32_t x = c ^ w, xr = crc_rot(x, k);
    uint32_t a0 = s4get(k, xr, 0), a1 = s4get(k, xr, 1), a2 = s4get(k, xr, 2), a3 = s4get(k, xr, 3);
    asm("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    return xor3(a0, a1, a2) ^ a3;
}
__device__ __forceinline__ uint32_t bitop3_xandn(uint32_t a, uint32_t b, uint32_t c) {   // one v_bitop3
    return a ^ (b & ~c);
}
// the lookups of one slice-by-4 step for two chains' inputs xa, xb, all issued together: the
// step's result is ta ^ a3 (tb ^ b3), and the next step's input that ^ the next word, one v_bitop3
__device__ __forceinline__ void look4x2(uint32_t xa, uint32_t xb, const Crc &k, uint32_t &ta, uint32_t &a3, uint32_t &tb,
                                        uint32_t &b3) {
    const uint32_t ra = crc_rot(xa, k), rb = crc_rot(xb, k);
    uint32_t a0 = s4get(k, ra, 0), a1 = s4get(k, ra, 1), a2 = s4get(k, ra, 2), a3_ = s4get(k, ra, 3);
    uint32_t b0 = s4get(k, rb, 0), b1 = s4get(k, rb, 1), b2 = s4get(k, rb, 2), b3_ = s4get(k, rb, 3);
    asm("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3_), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3_));
    ta = xor3(a0, a1, a2);
    a3 = a3_;
    tb = xor3(b0, b1, b2);
    b3 = b3_;
}
__device__ __forceinline__ uint32_t crc1(uint32_t c, uint32_t b, const Crc &k) {
    const uint32_t x = c ^ b;
    return (x >> 8) ^ tget(k, x, SEL_T0_B0);
}

// register state v times a constant K (nibble tables; every lane reads table i at once, so the
// 16 entries sit in 16 banks and equal indices broadcast: conflict free).  For a per-lane constant,
// kmul_col below.  The eight lookups
// are independent: the empty asm makes the scheduler issue them all before the first use.
__device__ __forceinline__ uint32_t xor8(uint32_t *t) {
    asm("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]));
    return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
}
// (the nibbles are split into two byte planes first: each index is then one byte extract)
__device__ __forceinline__ uint32_t kmul(uint32_t v, const uint32_t *K) {
    uint32_t pl[2] = {v & 0x0F0F0F0Fu, (v >> 4) & 0x0F0F0F0Fu};
    asm("" : "+v"(pl[0]), "+v"(pl[1]));   // keep the planes (no re-fusion into nibble shifts)
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = K[i * 16 + ((pl[i & 1] >> (8 * (i >> 1))) & 255u)];
    return xor8(t);
}
// v times the constant in column k (per lane) of a [i][n][k] table of 64 columns (KR, KQL) at
// byte OFF >= 64 KiB of Smem, rows of PITCH dwords: entry (i, n, k) sits at OFF + (16 i + n) 4 PITCH
// + 4 k.  PITCH 64: the address is one v_perm_b32 (byte 0 = 4 k and byte 2 = 1, the 64-KiB bit,
// from L4k; byte 1 = i << 4 | n from a plane, each plane byte carrying its lookup's i above the
// nibble), and the ds_read immediate is OFF - 64 KiB.  A lookup's bank is then k mod 32 whatever
// the nibble, so lanes that share a column (the pieces of different values pushed the same
// distance, KR) conflict; PITCH 66 puts entry (n, k) in bank 2 n + k: one v_perm (the row byte)
// and one v_mad_u32_u24 a lookup.
template <uint32_t OFF, int PITCH = 64, class SM = Smem>
__device__ __forceinline__ uint32_t kmul_col(uint32_t v, const SM &S, uint32_t k4) {
    const uint32_t L4k = k4 | 0x10000u;
    // plane 0: nibbles i = 0, 2, 4, 6 (byte j: i = 2j), plane 1: i = 1, 3, 5, 7
    uint32_t pl[2] = {(v & 0x0F0F0F0Fu) | 0x60402000u, ((v >> 4) & 0x0F0F0F0Fu) | 0x70503010u};
    asm("" : "+v"(pl[0]), "+v"(pl[1]));   // keep the planes (no re-fusion into nibble shifts)
    const uint8_t *tb = reinterpret_cast<const uint8_t *>(&S);
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t a;
        if constexpr (PITCH == 64) {
            a = __builtin_amdgcn_perm(pl[i & 1], L4k, 0x0C020000u | ((4u + (uint32_t)(i >> 1)) << 8));
        } else {
            const uint32_t row = __builtin_amdgcn_perm(0u, pl[i & 1], 0x0C0C0C00u | (uint32_t)(i >> 1));
            a = __umul24(row, 4u * (uint32_t)PITCH) + L4k;
        }
        t[i] = *reinterpret_cast<const uint32_t *>(tb + (OFF - 65536u) + a);
    }
    return xor8(t);
}

// ---------------------------------------------------------------------------------------
// Segment reads relative to a tile's first byte (offset o = segment position lo + o), through a
// buffer resource that ends at the segment's last 16-B word (words past it read as 0).  Used
// for what is not in the registers: the candidates' decode windows, key and value bytes of the
// records, headers past the tile end, the stripe's entry search.  Offsets the resource cannot
// reach (before the tile, or past 2^31) go through plain loads; callers stay inside the segment.
// ---------------------------------------------------------------------------------------
struct TileSeg {
    __amdgpu_buffer_rsrc_t rs;
    int64_t lo;           // segment position of offset 0
    uint64_t len;         // segment length
    const uint8_t *seg;   // segment byte 0
    int64_t lim;          // the resource covers offsets [0, lim)

    __device__ __forceinline__ uint32_t b8(int64_t o) const {
        if (o >= 0 && o < lim) return __builtin_amdgcn_raw_buffer_load_b8(rs, (int)o, 0, 0);
        return seg[lo + o];
    }
    __device__ __forceinline__ uint32_t w32a(int o) const {   // 4-aligned, 0 <= o < lim
        return __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
    }
    __device__ __forceinline__ uint32_t u32(int64_t o) const {   // any alignment; o .. o+3 in the segment
        if (o >= 0 && o + 8 <= lim) {
            const int a = (int)o & ~3;
            return __builtin_amdgcn_alignbyte(w32a(a + 4), w32a(a), (uint32_t)o & 3u);
        }
        return b8(o) | (b8(o + 1) << 8) | (b8(o + 2) << 16) | (b8(o + 3) << 24);
    }
};

// raw CRC register (from ~0) over the n <= 4 NW bytes of a span whose aligned words are r[0..NW]
// (sh = the span's start mod 4), and in *bad the 0x80 bits of those bytes; nw (wave-uniform) >=
// the words any lane needs
template <int NW>
__device__ __forceinline__ uint32_t crc_words(const uint32_t (&r)[NW + 1], const Crc &K, uint32_t sh, uint32_t n,
                                              uint32_t nw, uint32_t *bad) {
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
// the same when n is one length for every lane of the call (wave-uniform, n <= 4 NW): whole words
// need no byte masks, so a word is an align, a CRC step and an or (the usual case: every key of a
// store has one length)
template <int NW>
__device__ __forceinline__ uint32_t crc_words_u(const uint32_t (&r)[NW + 1], const Crc &K, uint32_t sh, uint32_t n,
                                                uint32_t *bad) {
    uint32_t c = ~0u, bd = 0;
    const uint32_t nf = n >> 2, rb = n & 3u;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if ((uint32_t)i < nf) {
            const uint32_t kw = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
            bd |= kw & 0x80808080u;
            c = crc4(c, kw, K);
        }
    }
    if (rb) {
        uint32_t kw = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i)
            if ((uint32_t)i == nf) kw = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
        bd |= kw & ((1u << (8u * rb)) - 1u) & 0x80808080u;
        for (uint32_t b = 0; b < rb; ++b) c = crc1(c, (kw >> (8u * b)) & 255u, K);
    }
    *bad = bd;
    return c;
}

// the same over segment bytes [o, o + n) loaded here (o >= 0, o + 4 NW + 4 <= lim)
template <int NW>
__device__ __forceinline__ uint32_t crc_span(const TileSeg &ts, const Crc &K, int o, uint32_t n, uint32_t nw,
                                             uint32_t *bad) {
    const int a = o & ~3;
    uint32_t r[NW + 1];
#pragma unroll
    for (int i = 0; i <= NW; ++i) r[i] = (uint32_t)i <= nw ? ts.w32a(a + 4 * i) : 0u;
    return crc_words<NW>(r, K, (uint32_t)o & 3u, n, nw, bad);
}

// CRC register update over segment bytes [o, o + n) (any length; the general path)
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

// ---------------------------------------------------------------------------------------
// UTF-8 validation with Rust's Utf8Error semantics (engine.rs:114, String::from_utf8).
// Returns true if valid, else *vu = valid_up_to and *el = error_len (0 = incomplete).
// ---------------------------------------------------------------------------------------
template <class TS>
__device__ inline bool utf8_check(const TS &ts, int64_t p, uint64_t n, uint64_t *vu, uint32_t *el) {
    uint64_t i = 0;
#pragma unroll 1
    while (i < n) {
        const int64_t q = p + (int64_t)i;
        if (n - i >= 4 && q >= 0 && q + 8 <= ts.lim) {   // ASCII fast path, 4 bytes at a time
            if ((ts.u32(q) & 0x80808080u) == 0) { i += 4; continue; }
        }
        const uint32_t b = ts.b8(q);
        if (b < 0x80u) { ++i; continue; }
        const uint64_t start = i;
        int width = 0;
        if (b >= 0xC2u && b <= 0xDFu) width = 2;
        else if (b >= 0xE0u && b <= 0xEFu) width = 3;
        else if (b >= 0xF0u && b <= 0xF4u) width = 4;
        *vu = start;
        if (width == 0) { *el = 1; return false; }
        if (++i >= n) { *el = 0; return false; }
        const uint32_t c1 = ts.b8(p + (int64_t)i);
        bool ok1;
        if (width == 2) ok1 = (c1 & 0xC0u) == 0x80u;
        else if (width == 3)
            ok1 = (b == 0xE0u && c1 >= 0xA0u && c1 <= 0xBFu) || (b >= 0xE1u && b <= 0xECu && c1 >= 0x80u && c1 <= 0xBFu) ||
                  (b == 0xEDu && c1 >= 0x80u && c1 <= 0x9Fu) || (b >= 0xEEu && c1 >= 0x80u && c1 <= 0xBFu);
        else
            ok1 = (b == 0xF0u && c1 >= 0x90u && c1 <= 0xBFu) || (b >= 0xF1u && b <= 0xF3u && c1 >= 0x80u && c1 <= 0xBFu) ||
                  (b == 0xF4u && c1 >= 0x80u && c1 <= 0x8Fu);
        if (!ok1) { *el = 1; return false; }
        for (int k = 2; k < width; ++k) {
            if (++i >= n) { *el = 0; return false; }
            if ((ts.b8(p + (int64_t)i) & 0xC0u) != 0x80u) { *el = (uint32_t)k; return false; }
        }
        ++i;
    }
    return true;
}

// ---------------------------------------------------------------------------------------
// the stripe's entry: its first plausible record start (k_link verifies it)
// ---------------------------------------------------------------------------------------
// End of the record at o (engine.rs framing, exact), or -1 if the framing is broken there:
// opcode outside {0,1} or a field running past the segment end.  o inside the segment.
template <class TS>
__device__ inline int64_t next_rec(const TS &ts, int64_t o) {
    const int64_t rem = (int64_t)ts.len - ts.lo;          // segment end, tile-relative
    const uint32_t op = ts.b8(o);
    if (op > 1u || rem - o < 5) return -1;
    const int64_t e = o + 5 + (int64_t)ts.u32(o + 1);
    if (e > rem) return -1;
    if (op == 1u) return e;
    if (rem - e < 4) return -1;
    const int64_t e2 = e + 4 + (int64_t)ts.u32(e);
    return e2 > rem ? -1 : e2;
}

// Could the first min(klen, 16) key bytes begin a valid UTF-8 string without NUL?  Keys are
// String (engine.rs:114): a candidate whose "key" is random value bytes fails the UTF-8 test,
// and one that starts a few bytes before a true header ([0][len LE] makes an in-range length
// whose "key" is the zero bytes of the true length) fails the NUL test.  Heuristic only: a true
// record rejected here (a key holding NUL) is found again by the stripe link check and the
// exact re-walk, so results never depend on it.
template <class TS>
__device__ inline bool key_prefix_ok(const TS &ts, int64_t ok, uint32_t klen) {
    const int m = klen > 16u ? 16 : (int)klen;
    int i = 0;
    #pragma unroll 1
    while (i < m) {
        const uint32_t b = ts.b8(ok + i);
        if (b == 0u) return false;
        if (b < 0x80u) { ++i; continue; }
        int w;
        uint32_t c_lo = 0x80u, c_hi = 0xBFu;
        if (b >= 0xC2u && b <= 0xDFu) w = 2;
        else if (b >= 0xE0u && b <= 0xEFu) { w = 3; if (b == 0xE0u) c_lo = 0xA0u; if (b == 0xEDu) c_hi = 0x9Fu; }
        else if (b >= 0xF0u && b <= 0xF4u) { w = 4; if (b == 0xF0u) c_lo = 0x90u; if (b == 0xF4u) c_hi = 0x8Fu; }
        else return false;
        if (i + 1 >= m) return true;
        const uint32_t c1 = ts.b8(ok + i + 1);
        if (c1 < c_lo || c1 > c_hi) return false;
        for (int k = 2; k < w; ++k) {
            if (i + k >= m) return true;
            if ((ts.b8(ok + i + k) & 0xC0u) != 0x80u) return false;
        }
        i += w;
    }
    return true;
}

// key_prefix_ok over the key bytes held in registers: byte i of the key is byte 5 + i of the
// little-endian window x[0..5] (x starts at the record).  The same UTF-8 prefix rules as a
// state machine unrolled over the 16 bytes (need: continuation bytes still due, [clo, chi]: the
// range of the next one), so no byte waits on the previous one's load.
__device__ __forceinline__ bool key_prefix_ok_r(const uint32_t (&x)[6], uint32_t klen) {
    const uint32_t m = klen > 16u ? 16u : klen;
    uint32_t need = 0, clo = 0x80u, chi = 0xBFu;
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t b = (x[(5 + i) >> 2] >> (8 * ((5 + i) & 3))) & 255u;
        const bool act = (uint32_t)i < m;
        const bool lead2 = b >= 0xC2u && b <= 0xDFu, lead3 = b >= 0xE0u && b <= 0xEFu,
                   lead4 = b >= 0xF0u && b <= 0xF4u;
        const bool bad_lead = b == 0u || (b >= 0x80u && !lead2 && !lead3 && !lead4);
        const bool bad_cont = b < clo || b > chi;
        bad = bad || (act && (need == 0u ? bad_lead : bad_cont));
        const uint32_t n_need = need != 0u ? need - 1u : (lead2 ? 1u : lead3 ? 2u : lead4 ? 3u : 0u);
        const uint32_t n_lo = need == 0u && b == 0xE0u ? 0xA0u : need == 0u && b == 0xF0u ? 0x90u : 0x80u;
        const uint32_t n_hi = need == 0u && b == 0xEDu ? 0x9Fu : need == 0u && b == 0xF4u ? 0x8Fu : 0xBFu;
        need = n_need; clo = n_lo; chi = n_hi;
    }
    return !bad;
}

template <class TS>
__device__ inline bool plausible(const TS &ts, int64_t o) {
    const int64_t rem = (int64_t)ts.len - ts.lo;
    // the near tests first (header and key bytes sit in the tile's lines): inside a long value
    // nearly every candidate fails them, before next_rec reads at the far value length.  Inside
    // the resource the header and 16 key bytes arrive as one window of independent loads.
    if (o >= 0 && o + 32 <= ts.lim) {
        const int a = (int)o & ~3;
        const uint32_t sh = (uint32_t)o & 3u;
        uint32_t r[7], x[6];
#pragma unroll
        for (int i = 0; i < 7; ++i) r[i] = ts.w32a(a + 4 * i);
#pragma unroll
        for (int i = 0; i < 6; ++i) x[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], sh);
        const uint32_t op = x[0] & 255u;
        const uint32_t klen = (x[0] >> 8) | (x[1] << 24);
        if (op > 1u || rem - o < 5 || (int64_t)klen > rem - o - 5) return false;
        if (!key_prefix_ok_r(x, klen)) return false;
    } else {
        const uint32_t op = ts.b8(o);
        if (op > 1u || rem - o < 5) return false;
        const uint32_t klen = ts.u32(o + 1);
        if ((int64_t)klen > rem - o - 5) return false;
        if (!key_prefix_ok(ts, o + 5, klen)) return false;
    }
    const int64_t nx = next_rec(ts, o);
    if (nx < 0) return false;
    if (nx == rem) return true;
    if (ts.b8(nx) > 1u || rem - nx < 5) return false;
    return nx + 5 + (int64_t)ts.u32(nx + 1) <= rem;
}

// ---------------------------------------------------------------------------------------
// records
// ---------------------------------------------------------------------------------------
// the first min(klen, 16) key bytes as four little-endian words, zero padded (the fold's key
// prefix, kvr_compact.hip FoldEnt::key), from the key words x[0..4] that start sh bytes into x[0]
__device__ __forceinline__ uint4 key_prefix_words(const uint32_t *x, uint32_t sh, uint32_t klen) {
    uint32_t k[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t v = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
        const uint32_t n = klen > 4u * j ? klen - 4u * j : 0u;   // key bytes in this word
        k[j] = n >= 4u ? v : (v & ((1u << (8u * n)) - 1u));
    }
    return make_uint4(k[0], k[1], k[2], k[3]);
}
// the same from the segment bytes at tile offset kb (o >= 0 inside the tile's resource, or any
// segment position through single-byte reads)
__device__ inline uint4 key_prefix_mem(const TileSeg &ts, int64_t kb, uint32_t klen) {
    if (kb >= 0 && kb + 24 <= ts.lim) {
        const int a = (int)kb & ~3;
        uint32_t x[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = ts.w32a(a + 4 * i);
        return key_prefix_words(x, (uint32_t)kb & 3u, klen);
    }
    uint32_t k[4] = {0u, 0u, 0u, 0u};
    const uint32_t m = klen < 16u ? klen : 16u;
    for (uint32_t i = 0; i < m; ++i) k[i >> 2] |= ts.b8(kb + (int64_t)i) << (8u * (i & 3u));
    return make_uint4(k[0], k[1], k[2], k[3]);
}

struct RecRes {          // one record's outcome on the general path
    uint32_t err, kind;  // record index of an error (N32: none) and its KVR_E_* kind
    uint64_t aux;
};

// parse + emit the record at tile offset o with every engine.rs check, in engine.rs order
// (its value, if longer than SMALL, was folded by the framing)
__device__ inline RecRes do_record(const TileSeg &ts, const Crc &K, int64_t o, uint32_t j, uint32_t slot, uint32_t seg,
                                   kvr_tuple *pool, uint4 *kpool) {
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
    pool[slot] = t;
    if (kpool) kpool[slot] = key_prefix_mem(ts, kb, (uint32_t)klen);
    return ro;
}

// the value CRC a record's own lane computes: a value of at most SMALL bytes, or one inside a
// single unit (longer values crossing a unit boundary are folded into the unit CRC phase)
__device__ __forceinline__ uint32_t short_value_crc(const TileSeg &ts, const Crc &K, int vb, uint32_t vlen) {
    uint32_t vbad;
    if (vlen <= (uint32_t)SMALL) {
        if (vb + 4 * VALW + 8 <= ts.lim) return ~crc_span<VALW>(ts, K, vb, vlen, (uint32_t)VALW, &vbad);
        return ~crc_long(ts, ~0u, vb, vlen, K);
    }
    if ((vb >> SC_LOG) == ((vb + (int)vlen - 1) >> SC_LOG)) {   // inside one unit
        if (vb + 4 * UW + 8 <= ts.lim) return ~crc_span<UW>(ts, K, vb, vlen, (uint32_t)UW, &vbad);
        return ~crc_long(ts, ~0u, vb, vlen, K);
    }
    return 0u;
}

// this lane's 128-B unit of tile k: eight 16-B raw buffer loads through a per-tile resource whose
// range is the 16-B words touching the segment, so words outside it read as 0 in hardware
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// (quads [Q0, Q1) of the unit: the whole unit, or one half while the other is still in use)
template <int Q0 = 0, int Q1 = UW / 4>
__device__ __forceinline__ void load_unit(const uint8_t *abase, int64_t d0, uint64_t len, uint32_t k, int lane,
                                          uint32_t *r) {
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
#pragma unroll
    for (int i = Q0; i < Q1; ++i) {
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16 * i, 0, 0);
        r[4 * i] = a.x; r[4 * i + 1] = a.y; r[4 * i + 2] = a.z; r[4 * i + 3] = a.w;
    }
}

// the reads of tile k relative to its first byte (see TileSeg)
__device__ __forceinline__ TileSeg tile_seg(const uint8_t *abase, const uint8_t *seg, int64_t d0, uint64_t len,
                                            uint32_t k) {
    TileSeg ts;
    const int64_t t0 = (int64_t)k * TILE;
    const int64_t endw = (d0 + (int64_t)len + 15) & ~(int64_t)15;
    int64_t lim = endw - t0;
    lim = lim > 0x7FFFFF00ll ? 0x7FFFFF00ll : lim;
    const uint64_t b = (uint64_t)(abase + t0);
    const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)b), bhi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    ts.rs = __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)bhi << 32) | blo), (short)0,
                                              __builtin_amdgcn_readfirstlane((int)lim), 0x00020000);
    ts.lo = t0 - d0;
    ts.len = len;
    ts.seg = seg;
    ts.lim = lim;
    return ts;
}

// ---------------------------------------------------------------------------------------
// the piece mode (uniform_run in replay_body)
// ---------------------------------------------------------------------------------------
// a lane's 128-B piece at byte offset o of the resource: 16-B loads from the dword that holds its
// first byte, and the dword after them (byte-unaligned 16-B loads run at half the rate: tools/
// piece_probe.hip); piece_align shifts the words into place once they have landed.  Offsets past the
// resource read 0.
#ifndef KVR_PAUX   // k_piece's piece loads: cache policy bits (2: nt, streamed past the caches; A/B knob)
#define KVR_PAUX 0
#endif
__device__ __forceinline__ void load_piece(__amdgpu_buffer_rsrc_t rs, int o, uint32_t (&w)[UW + 1]) {
    const int a = o & ~3;
#pragma unroll
    for (int i = 0; i < UW / 4; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, a + 16 * i, 0, KVR_PAUX);
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
    w[UW] = __builtin_amdgcn_raw_buffer_load_b32(rs, a + 4 * UW, 0, KVR_PAUX);
}
__device__ __forceinline__ void piece_align(uint32_t (&w)[UW + 1], int o) {
    const uint32_t sh = (uint32_t)o & 3u;
    if (__ballot(sh != 0u) == 0ull) return;   // (every lane's piece starts on a dword)
#pragma unroll
    for (int i = 0; i < UW; ++i) w[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}
// the raw CRC register (from 0) of the lane's 128 B: two slice-by-4 chains over words 0-15 and
// 16-31 (no value boundary inside), the first pushed through the second's 64 bytes.  On lanes with
// `on` (a value's first piece) the bytes before byte zb (wave-uniform, < SC) are not part of the value:
// leading zeros leave a register of 0 unchanged, so such a lane restarts its chain at word zb / 4 with
// that word's leading bytes masked (the uniform step index makes the restart one select), and the
// chain over words 0-15 contributes nothing when the restart is in the second half.
template <class SM>
__device__ __forceinline__ uint32_t piece_raw(const uint32_t (&w)[UW + 1], const Crc &K, const SM &S, bool on,
                                              uint32_t zb) {
    constexpr int H = UW / 2;
    const uint32_t zw = zb >> 2, pm = ~0u << (8u * (zb & 3u));
    uint32_t xa = w[0], xb = w[H], ca = 0, cb = 0;
#pragma unroll
    for (int kk = 0; kk < H; ++kk) {
        if (zb != 0u && zw == (uint32_t)kk) xa = on ? (w[kk] & pm) : xa;
        if (zb != 0u && zw == (uint32_t)(kk + H)) xb = on ? (w[kk + H] & pm) : xb;
        uint32_t ta, a3, tb, b3;
        look4x2(xa, xb, K, ta, a3, tb, b3);
        if (kk + 1 < H) {
            xa = xor3(ta, a3, w[kk + 1]);
            xb = xor3(tb, b3, w[kk + 1 + H]);
        } else {
            ca = ta ^ a3;
            cb = tb ^ b3;
        }
    }
    if (zw >= (uint32_t)H) ca = on ? 0u : ca;
    return kmul(ca, S.KQ2) ^ cb;
}
// piece_raw with four chains of eight words (half the dependent LDS steps of two chains of sixteen),
// combined as c0 x^(8*96) ^ c1 x^(8*64) ^ c2 x^(8*32) ^ c3
template <class SM>
__device__ __forceinline__ uint32_t piece_raw4(const uint32_t (&w)[UW + 1], const Crc &K, const SM &S) {
    constexpr int Q = UW / 4;
    uint32_t x0 = w[0], x1 = w[Q], x2 = w[2 * Q], x3 = w[3 * Q], c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int kk = 0; kk < Q; ++kk) {
        uint32_t t0, a0, t1, a1, t2, a2, t3, a3;
        look4x2(x0, x1, K, t0, a0, t1, a1);
        look4x2(x2, x3, K, t2, a2, t3, a3);
        if (kk + 1 < Q) {
            x0 = xor3(t0, a0, w[kk + 1]);
            x1 = xor3(t1, a1, w[kk + 1 + Q]);
            x2 = xor3(t2, a2, w[kk + 1 + 2 * Q]);
            x3 = xor3(t3, a3, w[kk + 1 + 3 * Q]);
        } else {
            c0 = t0 ^ a0; c1 = t1 ^ a1; c2 = t2 ^ a2; c3 = t3 ^ a3;
        }
    }
    return xor3(kmul(c0, S.KQ4 + 128), kmul(c1, S.KQ2), kmul(c2, S.KQ4)) ^ c3;
}
// segmented inclusive XOR scan over the lanes (DPP only): fm all ones starts a segment
__device__ __forceinline__ uint32_t seg_xscan(uint32_t v, uint32_t fm) {
    uint32_t ov;
    ov = dpp<0x111>(v); v = bitop3_xandn(v, ov, fm); fm |= dpp<0x111>(fm);
    ov = dpp<0x112>(v); v = bitop3_xandn(v, ov, fm); fm |= dpp<0x112>(fm);
    ov = dpp<0x114>(v); v = bitop3_xandn(v, ov, fm); fm |= dpp<0x114>(fm);
    ov = dpp<0x118>(v); v = bitop3_xandn(v, ov, fm); fm |= dpp<0x118>(fm);
    ov = dpp<0x142, 0xA, false>(v); v = bitop3_xandn(v, ov, fm); fm |= dpp<0x142, 0xA, false>(fm);
    return bitop3_xandn(v, dpp<0x143, 0xC, false>(v), fm);
}
// a buffer resource over segment bytes [pos, len) (at most 2^31 - 256 of them; none past len)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seg_rsrc(const uint8_t *seg, uint64_t pos, uint64_t len) {
    const uint64_t n = pos < len ? len - pos : 0ull;
    const int nr = n > 0x7FFFFF00ull ? 0x7FFFFF00 : (int)n;
    const uint64_t b = (uint64_t)(seg + pos);
    const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)b), bhi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)bhi << 32) | blo), (short)0,
                                             __builtin_amdgcn_readfirstlane(nr), 0x00020000);
}
// the same over the dwords that hold segment bytes [pos, len): byte pos is at offset adj (0 .. 3) of
// the resource, so that an offset o + adj with o a multiple of 4 from pos is a dword-aligned address,
// and the dword holding byte len - 1 is read whole (the range check is per dword: a dword that
// crosses the end would read 0; its bytes past len are never used)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seg_rsrc_a(const uint8_t *seg, uint64_t pos, uint64_t len,
                                                             uint32_t &adj) {
    adj = (uint32_t)((uint64_t)(seg + pos) & 3u);
    const uint64_t end = ((uint64_t)(seg + len) + 3u) & ~3ull;   // (the dword holding byte len - 1 ends here)
    return seg_rsrc(seg, pos - adj, end - (uint64_t)seg);
}

// ---------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------
// The stripe's entry in tile [lo, lo + TILE): its first plausible record start, or NONE (k_link
// verifies it).  Candidate op bytes (0x00 / 0x01) come straight from the registers, kept only when the
// top byte of the key length after them (byte b of the next word) does not exceed the top byte of the
// segment bytes left: a necessary condition, word-wide (SWAR).  plausible() (memory reads, the exact
// tests) runs on the survivors alone, one per lane and round, so the lanes' dependent loads run side
// by side; a lane keeps its lowest plausible start, and lanes above the lowest lane holding one stop
// (unit positions grow with the lane).  [o0, o1): this lane's unit offsets inside the segment.
__device__ inline uint64_t find_entry(const uint32_t (&w)[UW], const TileSeg &ts, int64_t lo, int64_t rem, int o0, int o1,
                                      int lane) {
    const int us = lane * SC;
    uint32_t cm[4];
    cand_masks(w, rem, cm);
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
    return fnd == 0ull ? NONE : (uint64_t)(lo + (int64_t)rl32((uint32_t)cand, (int)__builtin_ctzll(fnd)));
}

// the CRC and multiply tables, global -> LDS (every workgroup of k_replay, k_rewalk and k_piece)
template <int NT = RT>
__device__ __forceinline__ void stage_tables(Smem &S, const Tables &tb, int tid) {
    for (int i = tid; i < 256 * 64; i += NT) S.C2[i] = tb.crc8[c2_table(i & 63) * 256 + (i >> 6)];
    for (int i = tid; i < 8 * 16 * KR_PITCH; i += NT) {
        const int row = i / KR_PITCH, kk = i - row * KR_PITCH;   // row = 16 i + n
        S.KR[i] = kk < 64 ? tb.kmul[((KSET_R + kk) * 8 + (row >> 4)) * 16 + (row & 15)] : 0u;
    }
    for (int i = tid; i < 8 * 16 * KQL_PITCH; i += NT) {
        const int row = i / KQL_PITCH, q = i - row * KQL_PITCH;   // row = 16 i + n
        S.KQL[i] = q < NQ ? tb.kmul[((KSET_Q + q) * 8 + (row >> 4)) * 16 + (row & 15)] : 0u;
    }
    for (int i = tid; i < 2 * 8 * 16; i += NT) S.KQ2[i] = tb.kmul[(KSET_Q + (i < 128 ? SC / 8 : SC / 4)) * 8 * 16 + (i & 127)];
    for (int i = tid; i < 2 * 8 * 16; i += NT) S.KQ4[i] = tb.kmul[(KSET_Q + (i < 128 ? SC / 16 : 3 * SC / 16)) * 8 * 16 + (i & 127)];
    if (tid < NIX) S.IX[tid] = tb.initx[tid];
}

template <int NT>
__device__ __forceinline__ void stage_tables_p(SmemP &S, const Tables &tb, int tid) {
    for (int i = tid; i < 256 * 64; i += NT) S.C2[i] = tb.crc8[c2_table(i & 63) * 256 + (i >> 6)];
    for (int i = tid; i < 8 * 16 * KR_PITCH; i += NT) {
        const int row = i / KR_PITCH, kk = i - row * KR_PITCH;   // row = 16 i + n
        S.KR[i] = kk < 64 ? tb.kmul[((KSET_R + kk) * 8 + (row >> 4)) * 16 + (row & 15)] : 0u;
    }
    for (int i = tid; i < 2 * 8 * 16; i += NT) S.KQ2[i] = tb.kmul[(KSET_Q + (i < 128 ? SC / 8 : SC / 4)) * 8 * 16 + (i & 127)];
    for (int i = tid; i < 2 * 8 * 16; i += NT) S.KQ4[i] = tb.kmul[(KSET_Q + (i < 128 ? SC / 16 : 3 * SC / 16)) * 8 * 16 + (i & 127)];
    if (tid < NIX) S.IX[tid] = tb.initx[tid];
}

// REDO: the re-walk pass (k_rewalk) over k_link's list, with the walk-on into later stripes; the
// first pass (k_replay) walks every stripe once.  NT threads a workgroup, one stripe a wave.
template <bool REDO, int NT = RT>
__device__ __forceinline__ void replay_body(const SegDesc *__restrict__ segs,
                                            const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                            StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                            kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                            Tables tb, const RedoEnt *__restrict__ redo,
                                            const LinkResult *__restrict__ link, uint32_t pool_chunk,
                                            uint4 *__restrict__ kpool, uint32_t *__restrict__ scnt,
                                            const PieceHand *__restrict__ hand) {
    constexpr bool redo_mode = REDO;
    __shared__ Smem S;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (!REDO && hand) {   // after k_piece: a workgroup whose stripes it all finished has nothing to do
        const uint32_t g = blockIdx.x * (NT / 64) + (uint32_t)wv;
        if (!__syncthreads_or(g < n_stripes && !hand[g].done)) return;
    }
    stage_tables<NT>(S, tb, tid);
    if (tid == 0) { S.BAL[0] = 0u; S.BAL[1] = 0u; }
    __syncthreads();   // the only workgroup barrier: from here on every wave is on its own
    uint32_t *const MK = S.MK[wv];   // this wave's long-value marks

    Crc K;
    crc_init(K, S.C2, (uint32_t)lane);
    // the stripe index is wave-uniform: say so, so that the whole stripe state lives in SGPRs
    const uint32_t gw = blockIdx.x * (NT / 64) + (uint32_t)__builtin_amdgcn_readfirstlane(wv);
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
    // this wave's pool chunk.  Pool slots are 32-bit (the host keeps the pool under 2^32 - 2^16
    // tuples) and every slot a wave writes was claimed: a claim past pool_cap (the host then grows
    // the pool and runs again) is served from the slack the host allocates behind pool_cap, so no
    // store needs a bound check
    uint32_t chunk_base = 0, chunk_left = 0;
    // A re-walk (redo pass) walks on into the stripes after its own while their speculated entry
    // disagrees with the chain it carries, so a run of wrong speculations (a value holding a whole
    // segment image, say) costs one pass rather than one pass per stripe (see the end of the loop)
#pragma unroll 1
    for (;;) {
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
    const bool trapped = entry != NONE && (int64_t)entry < (int64_t)sd.t_begin * TILE - d0;
    if (trapped) {   // bug trap: k_link never does this
        stop = 2;
        stripe_entry = NONE;
        if (lane == 0) atomicOr(&ctr->overflow, 4u);
    }
    uint64_t err_pos = NONE, err_aux = 0;
    uint32_t err_kind = 0, total = 0;
    // (fast_skip bits 16 on: the records of the tile k_piece handed back that it emitted, the last ones
    // claimed (chunk_base - that count on); bits 0-15: tiles left to the scalar hop loop)
    uint32_t stride = 0, fast_skip = 0;           // lane-parallel framing: the last record length
    uint32_t run_first = N32;                     // the stripe's first pool slot, while its tuples are one run
    bool run_contig = true;                       // (no second chunk claimed after its first tuple)
    uint32_t carry = 0, c_state = 0;              // 1: a long value crosses the tile start (c_state: its register);
    uint64_t c_vb = 0, c_ve = 0;                  // 2: pending (its value starts in a later tile)
    uint32_t c_slot = 0;

    uint32_t w[UW];     // this lane's unit of the tile (the next tile's load is issued as soon as the
    bool loaded = false;   // CRC phase is done with these registers, see the end of the loop body)
    uint32_t k = sd.t_begin;
    if (!REDO && hand) {   // k_piece went first: it finished the stripe, or hands it back from tile h.k on
        const PieceHand h = hand[si];
        if (h.done) break;
        entry = h.entry;
        search = entry == NONE;
        stripe_entry = h.stripe_entry;
        k = h.k;
        fast_skip = h.ahead << 16;
        stride = h.stride;
        total = h.total;
        chunk_base = h.chunk_base;
        chunk_left = h.chunk_left;
        run_first = h.run_first;
        run_contig = h.run_contig != 0u;
    }
#ifdef KVR_PROF
    unsigned long long t_last = __builtin_amdgcn_s_memtime();
    unsigned long long prof_acc[16] = {};
    const unsigned long long rrt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // progress balance (KVR_RBAL): as k_piece's, over the stripe's tiles; a wave more than
    // KVR_PBAL_D / 4096 of its stripe behind the workgroup's mean runs one priority up
    bool rbal_up = false;
    const uint32_t rb_t0 = sd.t_begin, rb_n = sd.t_end > sd.t_begin ? sd.t_end - sd.t_begin : 1u;
    const uint64_t rb_scale = (4096ull << 32) / rb_n;
    uint32_t rb_own = 0;
    const bool rb_on = KVR_RBAL && !REDO;
    if (rb_on && lane == 0) atomicAdd(&S.BAL[1], 1u);
    for (;; ++k) {
        if (rb_on) {
            const uint32_t kd = k > rb_t0 ? k - rb_t0 : 0u;
            const uint32_t pn = (uint32_t)(((uint64_t)(kd < rb_n ? kd : rb_n) * rb_scale) >> 32);
            uint32_t sum = 0, cnt = 1;
            if (lane == 0) {
                sum = atomicAdd(&S.BAL[0], pn - rb_own) + (pn - rb_own);
                cnt = S.BAL[1];
            }
            rb_own = pn;
            sum = uni32(sum);
            cnt = uni32(cnt);
            const int32_t d = (int32_t)(pn * cnt - sum), dl = (int32_t)(KVR_PBAL_D * cnt);
            rbal_up = d < -dl;
            if (KVR_RBAL == 2) {   // (the phases at one priority: four levels from the progress alone)
                if (d < -dl) __builtin_amdgcn_s_setprio(3);
                else if (d < 0) __builtin_amdgcn_s_setprio(2);
                else if (d < dl) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            } else {
                KVR_SETPRIO(0);
            }
        }
        if (KVR_TOPWAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        KVR_STAMP(5);
        const bool in_stripe = k < sd.t_end;
        if (stop || (!in_stripe && !carry) || k >= sg.n_tiles) break;
        if (!loaded) {
            load_unit(abase, d0, len, k, lane, w);
            if (KVR_TOPWAIT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        loaded = false;
        if (KVR_ABLATE & 64) {   // loads only (FETCH_SIZE calibration on a known byte count)
            uint32_t x = 0;
#pragma unroll
            for (int i = 0; i < UW; ++i) x ^= w[i];
            if (x == 0x9E3779B9u && lane == 0) atomicOr(&ctr->overflow, 8u);   // keeps the loads alive
            carry = 0;
            continue;
        }

        const int64_t lo = (int64_t)k * TILE - d0;      // segment position of tile byte 0
        const uint64_t vlo = lo < 0 ? 0ull : (uint64_t)lo;
        const uint64_t vhi = (uint64_t)(lo + TILE) > len ? len : (uint64_t)(lo + TILE);
        const int64_t rem = (int64_t)len - lo;          // segment bytes from tile byte 0 on
        const int64_t vlo_r = (int64_t)vlo - lo, vhi_r = (int64_t)vhi - lo;
        const TileSeg ts = tile_seg(abase, sg.base, d0, len, k);
        const int us = lane * SC, ue = us + SC;
        // the little-endian u64 at tile offset o (uniform, 0 <= o, o + 8 <= TILE): out of the
        // lanes' registers (uniform register index + readlane), no memory access
        auto tword = [&](int j) -> uint32_t { return rl32(w[j & (UW - 1)], j >> 5); };
        auto tu64 = [&](int o) -> uint64_t {
            const int j = o >> 2;
            return ((((uint64_t)tword(j + 1)) << 32) | tword(j)) >> (8u * (uint32_t)(o & 3));
        };

        KVR_STAMP(0);
        // ---- F + R. framing and records -------------------------------------------------------
        if (in_stripe && search) {   // the stripe's entry: the first plausible record start
            const uint64_t mn = find_entry(w, ts, lo, rem, us > (int)vlo_r ? us : (int)vlo_r, ue < (int)vhi_r ? ue : (int)vhi_r, lane);
            if (mn != NONE) { entry = mn; search = false; stripe_entry = mn; }
        }
        const bool walk = in_stripe && !search && entry < vhi;
        uint64_t tile_exit = entry;
        // the long values touching this tile, folded into every unit's view as they are found
        // (per-lane flags as 32-bit values: a per-lane bool lives in an SGPR lane mask)
        int32_t vx = 0;                      // a long value crosses the end of this unit: its end
                                             // (tile-relative, clamped to FAR; 0: none)
        int32_t a_off = -1;                  // ... starting inside the unit at a_off
        uint32_t vx_carry = 0;               // ... the value carried in from the previous tile
        int32_t m = 0;                       // a long value ends inside this unit, at m (1 .. SC)
        uint32_t m_ref = 0;                  // ... its tuple: a slot (m_abs) or a record index of the tile
        uint32_t m_abs = 0;
        bool any_long = false;               // (uniform) some long value touches the tile
        bool out = false;                    // (uniform) a value crosses the tile end
        uint64_t out_ve = 0;
        uint32_t out_ref = 0;
        bool out_abs = false;
        auto consider = [&](int32_t vb, uint64_t ve_abs, uint32_t ref, bool is_abs, bool from_carry) {
            const int64_t v64 = (int64_t)ve_abs - lo;
            const int32_t ver = v64 > FAR ? FAR : (int32_t)v64;
            if (vb < ue && ver > ue) { vx = ver; a_off = vb >= us ? vb - us : -1; vx_carry = from_carry ? 1u : 0u; }
            if (vb < us && ver > us && ver <= ue) { m = ver - us; m_ref = ref; m_abs = is_abs ? 1u : 0u; }
            if (ver > TILE) { out = true; out_ve = ve_abs; out_ref = ref; out_abs = is_abs; }
            any_long = true;
        };
        uint32_t n_carry = 0;
        uint64_t n_vb = 0, n_ve = 0;         // the next tile's carry
        uint32_t n_ref = 0;                  // (a slot, or a record index)
        bool n_abs = true;
        if (carry == 1u) consider(-FAR, c_ve, c_slot, true, true);
        if (carry == 2u) {                   // a value whose record started in an earlier tile
            if ((int64_t)c_vb - lo < TILE) consider((int32_t)((int64_t)c_vb - lo), c_ve, c_slot, true, false);
            else { n_carry = 2; n_vb = c_vb; n_ve = c_ve; n_ref = c_slot; }   // still further on
        }
        // pool slots: the tile's records take at most two runs, [b1, b1 + c1) then [b2, ...)
        // (the tile k_piece handed back: its first `ahead` records were emitted, the last slots claimed)
        const uint32_t ahead = fast_skip >> 16;
        fast_skip &= 0xFFFFu;
        uint32_t b1 = chunk_base - ahead, b2 = 0;
        uint32_t c1 = N32;
        uint32_t nrec = ahead, err_rec = N32;   // records emitted; index of the tile's first error
        // claim pool slots for nb more records of the tile (one run: a fresh chunk holds any
        // tile's rest); returns the first slot
        auto claim = [&](uint32_t nb) -> uint32_t {
            if (nb > chunk_left) {
                const uint32_t cm = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
                unsigned long long bb = 0;
                if (lane == 0) {
                    bb = atomicAdd(&ctr->pool_cursor, (unsigned long long)cm);
                    if (bb + cm > pool_cap) {   // past the pool: flag it, write into the slack
                        atomicOr(&ctr->overflow, 1u);
                        bb = pool_cap;
                    }
                }
                chunk_base = uni32((uint32_t)bb);
                chunk_left = cm;
                if (nrec) { b2 = chunk_base; c1 = nrec; }   // the tile's second run
                if (run_first != N32) run_contig = false;
            }
            if (run_first == N32 && nb) run_first = chunk_base;
            if (nrec == 0) b1 = chunk_base;
            const uint32_t s0 = chunk_base;
            chunk_base += nb;
            chunk_left -= nb;
            return s0;
        };
        // a batch's long values crossing a unit boundary: each marks its first unit with
        // (rank + 1) << 6 | its lane (lmark; rank order = position order); one DPP prefix max over
        // the units finds, for every unit, the last one starting at or before it (and, shifted by
        // one lane, before it); two ds_bpermute fetch that record's value span from its lane.  Long
        // values are disjoint and in order, so these are the only candidates.  rank: the record's
        // index within the tile's records so far, per lane.
        auto fold_views = [&](uint32_t lmark, int32_t rvb, int32_t re2, uint32_t rank) {
            uint32_t pm = lmark;
            pm = __builtin_elementwise_max(pm, dpp<0x111>(pm));
            pm = __builtin_elementwise_max(pm, dpp<0x112>(pm));
            pm = __builtin_elementwise_max(pm, dpp<0x114>(pm));
            pm = __builtin_elementwise_max(pm, dpp<0x118>(pm));
            pm = __builtin_elementwise_max(pm, dpp<0x142, 0xA, false>(pm));
            pm = __builtin_elementwise_max(pm, dpp<0x143, 0xC, false>(pm));
            const uint32_t pp = dpp<0x138>(pm);   // wave_shr:1: the marks before this unit
            const int ic = 4 * (int)(pm & 63u), ip = 4 * (int)(pp & 63u);   // (the marks' lanes)
            const int32_t vbc = __builtin_amdgcn_ds_bpermute(ic, rvb), e2c = __builtin_amdgcn_ds_bpermute(ic, re2);
            const int32_t e2p = __builtin_amdgcn_ds_bpermute(ip, re2);
            const uint32_t rkp = (uint32_t)__builtin_amdgcn_ds_bpermute(ip, (int)rank);
            const bool cx = pm != 0u && e2c > ue;
            vx = cx ? e2c : vx;
            a_off = cx ? (vbc >= us ? vbc - us : -1) : a_off;
            vx_carry = cx ? 0u : vx_carry;
            const bool cmn = pp != 0u && e2p > us && e2p <= ue;
            m = cmn ? e2p - us : m;
            m_ref = cmn ? rkp : m_ref;
            m_abs = cmn ? 0u : m_abs;
            // a value crossing the last unit's end runs past the tile (ue = TILE there)
            const uint32_t e63 = rl32(cx ? (uint32_t)e2c : 0u, 63);
            if (e63 != 0u) {
                out = true; out_ve = (uint64_t)(lo + (int32_t)e63);
                out_ref = rl32((uint32_t)__builtin_amdgcn_ds_bpermute(ic, (int)rank), 63); out_abs = false;
            }
            any_long = true;
        };
        // fold_views for a round of n records of one length Ls, all SETs with one value length vu >
        // SC (so every value crosses a unit boundary): record j's value is [vb0 + j Ls, + vu), so a
        // unit finds the last value starting before its end (and before its start) by a division,
        // with no marks in LDS and no lane permutes
        auto fold_uniform = [&](int32_t vb0, int32_t Ls, uint32_t n, int32_t vu, uint32_t nbase) {
            const float invL = 1.0f / (float)Ls;
            auto below = [&](int32_t X) -> uint32_t {   // records with vb0 + j Ls < X (at most n)
                const int32_t t = X - vb0 - 1;
                int32_t q = (int32_t)((float)(t < 0 ? 0 : t) * invL);   // floor(t / Ls), then corrected
                q += (q + 1) * Ls <= t ? 1 : 0;
                q -= q * Ls > t ? 1 : 0;
                const uint32_t c = t < 0 ? 0u : (uint32_t)q + 1u;
                return c < n ? c : n;
            };
            const uint32_t nc = below(ue), np = below(us);
            const int32_t vbc = vb0 + ((int32_t)nc - 1) * Ls, e2c = vbc + vu;
            const bool cx = nc != 0u && e2c > ue;
            vx = cx ? e2c : vx;
            a_off = cx ? (vbc >= us ? vbc - us : -1) : a_off;
            vx_carry = cx ? 0u : vx_carry;
            const int32_t e2p = vb0 + ((int32_t)np - 1) * Ls + vu;
            const bool cmn = np != 0u && e2p > us && e2p <= ue;
            m = cmn ? e2p - us : m;
            m_ref = cmn ? nbase + np - 1u : m_ref;
            m_abs = cmn ? 0u : m_abs;
            // a value crossing the last unit's end runs past the tile (ue = TILE there)
            const uint32_t e63 = rl32(cx ? (uint32_t)e2c : 0u, 63);
            if (e63 != 0u) {
                out = true; out_ve = (uint64_t)(lo + (int32_t)e63);
                out_ref = nbase + rl32(nc, 63) - 1u; out_abs = false;
            }
            any_long = true;
        };
#if KVR_LANEFRAME
        // ---- lane-parallel framing ---------------------------------------------------------------
        // decode(c): the record that would start at tile offset c (per lane; act: the lane takes
        // part), from a window of the segment bytes: opcode, key length, value length, every
        // engine.rs framing check, and where its successor starts.  The value-length field is read
        // out of the window for the key length of lane kl (one length for every key is the usual
        // case); a lane with another key length reads it from memory (vmem) or leaves its
        // successor unknown (nx = UNK, resolved when the chain reaches it).
        struct Dec {
            uint32_t win[WINW];
            uint32_t s, op, klen, vlen, vb, nx;
            bool ok;
        };
        constexpr uint32_t UNK = 0xFFFFFFFEu;
        const int32_t vhiT = (int32_t)vhi_r, remT = (int32_t)rem;   // (used only when !huge)
        auto decode = [&](int32_t c, bool act, int kl, bool vmem, int32_t cend) -> Dec {
            Dec d;
            const int32_t a = c & ~3;
            d.s = (uint32_t)c & 3u;
            // (a lane that takes no part reads past the resource, which yields 0 with no memory
            // access: the loads need no exec mask, so no branch around each of them)
            const int32_t ao = act ? a : (int32_t)0x7FFFFF00;
#pragma unroll
            for (int i = 0; i < WINW; ++i) d.win[i] = ts.w32a(ao + 4 * i);
            const uint32_t x0 = __builtin_amdgcn_alignbyte(d.win[1], d.win[0], d.s);
            const uint32_t x1 = __builtin_amdgcn_alignbyte(d.win[2], d.win[1], d.s);
            d.op = x0 & 255u;
            d.klen = (x0 >> 8) | (x1 << 24);
            // engine.rs framing checks, tile-relative in 32 bits (rem < 2^31)
            const uint32_t room = (uint32_t)(remT - c);
            bool ok = act && d.op <= 1u && c < cend && room >= 5u && d.klen <= room - 5u;
            const uint32_t e = (uint32_t)c + 5u + (ok ? d.klen : 0u);   // < 2^31
            const bool need_v = ok && d.op == 0u;
            ok = ok && (!need_v || (uint32_t)remT - e >= 4u);
            const uint32_t ku = rl32(d.klen, kl);
            d.vlen = 0;
            bool vdone = false;
            {
                const uint32_t dd = 5u + ku, B0 = dd >> 2;
                if (B0 >= 1u && B0 <= (uint32_t)(WINW - 3)) {
                    uint32_t wa = 0, wb = 0, wc = 0;
#pragma unroll
                    for (int bb = 1; bb <= WINW - 3; ++bb)
                        if (B0 == (uint32_t)bb) { wa = d.win[bb]; wb = d.win[bb + 1]; wc = d.win[bb + 2]; }
                    const uint32_t oo = d.s + (dd & 3u);
                    const bool cy = oo >= 4u;
                    d.vlen = __builtin_amdgcn_alignbyte(cy ? wc : wb, cy ? wb : wa, oo & 3u);
                    vdone = d.klen == ku;
                }
            }
            bool unk = false;
            if (need_v && ok && !vdone) {
                if (vmem) d.vlen = ts.u32((int64_t)e);
                else unk = true;
            }
            d.vb = e + 4u;
            ok = ok && (!need_v || unk || d.vlen <= (uint32_t)remT - d.vb);
            d.ok = ok;
            d.nx = unk ? UNK : (d.op == 1u ? e : d.vb + d.vlen);
            return d;
        };
        // emit: the records of a framing round.  Lane j with `on` emits record nrec + rk (rk: its
        // rank on the chain, rank order = position order); lead / lastl: the lanes of the round's
        // first and last records.  strided: record j starts at cur0 + j L (the stride round), so the
        // long values of a round of equal SETs fold into the units by arithmetic.
        // (it calls no other lambda: the caller claims the pool slots and runs the long-value
        // fold it asks for, so no closure object has to live in memory)
        struct Fold { uint32_t lmark; int kind; };   // kind 0: none, 1: fold_uniform, 2: fold_views
        auto emit = [&](const Dec &d, int32_t c, bool on, uint32_t rk, uint32_t n_on, int lead, int lastl,
                        bool strided, uint32_t slot0) -> Fold {
            if (KVR_REC_PRIO != KVR_HOP_PRIO) KVR_SETPRIO(KVR_REC_PRIO);
            const uint32_t klen = d.klen, op = d.op, vlen = d.vlen, vb = d.vb, s = d.s;
            Fold fo{0u, 0};
            // one key length for the batch (the first record's, ku): no per-lane byte masks
            const uint32_t ku = rl32(klen, lead);
            const bool kuni = __ballot(on && klen != ku) == 0ull && ku <= 4u * KEYW;
            const uint32_t kmx = kuni ? ku : wave_max(on ? klen : 0u);
            uint32_t rerr = N32, rkind = 0;
            uint64_t raux = 0;
            if (on && !(KVR_ABLATE & 1)) {
                const uint32_t kc = kmx > 4u * KEYW ? 4u * KEYW : kmx;
                const uint32_t nw = (kc + 3u) >> 2;   // key words of the longest key
                uint32_t kr[KEYW + 1];
#pragma unroll
                for (int i = 0; i <= KEYW; ++i) kr[i] = s == 3u ? d.win[i + 2] : d.win[i + 1];
                const int kb = c + 5;
                uint32_t cc = ~0u, bad = 0x80u;
                if (kuni) cc = crc_words_u<KEYW>(kr, K, (s + 1u) & 3u, ku, &bad);
                else if (klen <= 4u * KEYW) cc = crc_words<KEYW>(kr, K, (s + 1u) & 3u, klen, nw, &bad);
                if (bad != 0u) {              // non-ASCII or long key: the full UTF-8 check
                    uint64_t vu = 0;
                    uint32_t el = 0;
                    if (!utf8_check(ts, kb, klen, &vu, &el)) {   // engine.rs:114
                        rerr = nrec + rk; rkind = KVR_E_UTF8; raux = vu | ((uint64_t)el << 32);
                    } else {
                        cc = crc_long(ts, ~0u, kb, klen, K);
                    }
                }
                if (rerr == N32) {
                    kvr_tuple t;
                    t.rec_off = (uint64_t)(lo + c);
                    t.seg_idx = sd.seg;
                    t.key_len = klen;
                    t.val_len = op == 0u ? vlen : 0u;
                    t.crc32 = op == 0u ? short_value_crc(ts, K, (int)vb, vlen) : 0u;
                    t.key_tag = ~cc;
                    t.op = (uint8_t)op;
                    t.flags = 0;
                    t.reserved = 0;
                    pool[slot0 + rk] = t;
                    // the key prefix for the fold (only calls that fold ask for it)
                    if (kpool) kpool[slot0 + rk] = key_prefix_words(kr, (s + 1u) & 3u, klen);
                }
            }
            // long values crossing a unit boundary: marked at their first unit (a scatter through
            // this wave's LDS row; the mark carries the rank, so the prefix max finds the latest,
            // and the lane), then folded into every unit's view
            const bool lv = on && op == 0u && vlen > (uint32_t)SMALL && ((vb ^ (vb + vlen - 1u)) >> SC_LOG) != 0u;
            const uint64_t lvm = __ballot(lv);
            // a round of SETs of one key and one value length (longer than a unit)
            const uint32_t vu = rl32(vlen, lead);
            const bool vuni = KVR_UNIFOLD && strided && vu > (uint32_t)SC &&
                              __ballot(on && (op != 0u || vlen != vu || klen != ku)) == 0ull;
            if (lvm && !(KVR_ABLATE & 32)) {
                uint32_t lmark = 0;
                if (!vuni) {
                    MK[lane] = 0u;
                    __builtin_amdgcn_wave_barrier();
                    if (lv && vb < (uint32_t)TILE) MK[vb >> SC_LOG] = ((rk + 1u) << 6) | (uint32_t)lane;
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    lmark = MK[lane];
                }
                // a long value starting past the tile end (only the last record's): carried
                if ((lvm >> lastl) & 1ull) {
                    const uint32_t vbl = rl32(vb, lastl);
                    if (vbl >= (uint32_t)TILE) {
                        n_carry = 2; n_vb = (uint64_t)(lo + (int64_t)vbl);
                        n_ve = (uint64_t)(lo + (int64_t)vbl + rl32(vlen, lastl));
                        n_ref = nrec + n_on - 1u;
                        n_abs = false;
                    }
                }
                fo.lmark = lmark;
                fo.kind = vuni ? 1 : 2;
            } else if (lvm) {
                any_long = true;
            }
            // the first error of the batch (lowest record index)
            if (__ballot(rerr != N32)) {
                const uint32_t mn = ~wave_max(~rerr);
                const int el = (int)__builtin_ctzll(__ballot(rerr == mn));
                err_rec = mn;
                err_kind = rl32(rkind, el);
                err_aux = rl64(raux, el);
                err_pos = (uint64_t)(lo + (int64_t)(int32_t)rl32((uint32_t)c, el));
            }
            if (KVR_REC_PRIO != KVR_HOP_PRIO) KVR_SETPRIO(KVR_HOP_PRIO);
            return fo;
        };
#endif
        if (walk) {
            // positions are tile-relative, in 32 bits unless the segment runs more than 2 GiB past
            // the tile (then the 64-bit copy of the exact hop loop takes the whole tile)
            const bool huge = rem > 0x7FFFFFFFll;
            int64_t p = (int64_t)entry - lo;
            bool broke = false;              // the chain broke at the last record walked
            if (KVR_ABLATE & 4) p = vhi_r;
            if (KVR_HOP_PRIO) KVR_SETPRIO(KVR_HOP_PRIO);
#if KVR_LANEFRAME
            bool round_broke = false;        // a lane-parallel round ended on a broken record
            if (!huge && p < vhi_r && fast_skip == 0u) {
                // ---- stride prediction, verified ---------------------------------------------------
                // Lane j decodes the record that would start at cur + j L (L = the last record's
                // length).  Lane 0's position is exact; lane j's is exact if records 0 .. j-1 were
                // valid and L long.  The first lane whose record is broken or whose successor is not
                // the next prediction ends the round (record f): the records up to f are the exact
                // chain, and f's own successor is exact.  A store of equal-sized records takes every
                // record of the tile in one round.  One round a tile (a loop here made the compiler
                // spill and reload much of the stripe state every tile): a round that found fewer than
                // three records hands the next tiles to the candidate round.
                int32_t cur = (int32_t)p;
                uint32_t L = stride;
                do {
                    const bool one = L == 0u || L >= (uint32_t)TILE;   // no usable stride: lane 0 only
                    const int32_t c = cur + (one ? 0 : lane * (int32_t)L);
                    const bool act = lane == 0 || (!one && c < vhiT);
                    const Dec d = decode(c, act, 0, true, vhiT);
                    KVR_STAMP(1);
                    // the first lane whose record is broken or whose successor is not the next
                    // prediction (the last active lane's successor is unconstrained)
                    const int n = (int)__builtin_popcountll(__ballot(act));
                    const bool mis = act && (!d.ok || (lane < n - 1 && d.nx != (uint32_t)(c + (int32_t)L)));
                    const uint64_t mm = __ballot(mis);
                    const int f = mm ? (int)__builtin_ctzll(mm) : n - 1;   // the round's last chain record
                    const bool okf = rl32(d.ok ? 1u : 0u, f) != 0u;
                    const uint32_t n_on = okf ? (uint32_t)f + 1u : (uint32_t)f;   // records on the chain
                    const uint32_t cf = rl32((uint32_t)c, f);
                    if (n_on) {
                        const uint32_t slot0 = claim(n_on);
                        const Fold fo = emit(d, c, (uint32_t)lane < n_on, (uint32_t)lane, n_on, 0, (int)n_on - 1, !one, slot0);
                        if (fo.kind == 1) {
                            fold_uniform(cur + 9 + (int32_t)rl32(d.klen, 0), (int32_t)L, n_on, (int32_t)rl32(d.vlen, 0), nrec);
                        } else if (fo.kind == 2) {
                            fold_views(fo.lmark, (int32_t)d.vb, (int32_t)(d.vb + d.vlen), nrec + (uint32_t)lane);
                        }
                        nrec = err_rec != N32 ? err_rec : nrec + n_on;
                    }
                    KVR_STAMP(6);
                    if (!okf) { cur = (int32_t)cf; round_broke = true; break; }   // the exact loop reports it
                    const uint32_t nf = rl32(d.nx, f);
                    L = nf - cf;                               // record f's length predicts the next tile
                    cur = (int32_t)nf;
                    if (err_rec != N32) break;
                    if (!one && n_on < 3u && cur < vhiT) {      // lengths vary: candidate rounds for a while
                        fast_skip = KVR_FAST_BACKOFF;
                        break;
                    }
                } while (0);
                stride = L;
                p = cur;
            } else if (fast_skip) {
                --fast_skip;
            }
#if KVR_CANDFRAME
            if (!huge && p < vhi_r && err_rec == N32 && !round_broke) {
                // ---- candidate chain: records of varying lengths, lane-parallel ----------------------
                // Every byte of [p, vhi) that can start a record of a key shorter than 32 MiB (an opcode
                // byte 0x00 / 0x01 with a key length whose top byte is 0x00 / 0x01: SWAR over the
                // registers, cand_masks_fast) is a candidate.  A window takes the candidates of the units from p's on, as many
                // whole units as fit 64: they go to one lane each (a scatter through this wave's LDS
                // row) and are decoded there with their successor.  The chain from p then follows the
                // candidates by lane matches (a ballot per record), which ranks the records: rank
                // order is position order.  A window ends where its units end (the next one starts at
                // the chain's position); a position that is not a candidate (a broken record, or a key
                // of 32 MiB or more) is left with the rest of the tile to the exact loop, and so is a
                // unit holding more than 64 candidates.
                uint32_t cm[4];
                cand_masks_fast(w, cm);
                if (vhiT < TILE) mask_from(cm, vhiT - us);   // the segment's last tile: nothing past its end
                const uint32_t cnt_u = (uint32_t)(__builtin_popcount(cm[0]) + __builtin_popcount(cm[1]) +
                                                  __builtin_popcount(cm[2]) + __builtin_popcount(cm[3]));
                KVR_STAMP(7);
                bool go = true;
#pragma unroll 1
                while (go && p < vhi_r && err_rec == N32) {
                    const int32_t p0 = (int32_t)p;
                    const uint32_t cnt = ue <= p0 ? 0u : cnt_u;       // units wholly before p hold none
                    const uint32_t inc = wave_incl_add(cnt);
                    const bool fits = inc <= 64u;                     // (inc grows with the lane)
                    const uint64_t fm = __ballot(!fits);
                    const int fl = fm ? (int)__builtin_ctzll(fm) : 64;   // the first lane whose unit does not fit
                    if (fl <= (p0 >> SC_LOG)) break;                  // p's unit alone holds more than 64
                    const uint32_t tot = rl32(inc, fl - 1);
                    const int32_t cover = fl * SC;                    // the window's units end here
                    if (tot == 0u) break;                             // p is no candidate: a broken record
                    // lane l's candidates (when its units fit) to slots [ex, ex + cnt) of the row (any
                    // order within a unit)
                    uint32_t ex = inc - cnt;
                    uint32_t m0 = cm[0], m1 = cm[1], m2 = cm[2], m3 = cm[3];
                    if (!fits || ue <= p0) { m0 = 0u; m1 = 0u; m2 = 0u; m3 = 0u; }
#pragma unroll 1
                    while (__ballot((m0 | m1 | m2 | m3) != 0u)) {
                        if ((m0 | m1 | m2 | m3) != 0u) {
                            const int q = m0 ? 0 : m1 ? 1 : m2 ? 2 : 3;
                            const uint32_t mb = q == 0 ? m0 : q == 1 ? m1 : q == 2 ? m2 : m3;
                            const uint32_t nb2 = mb & (mb - 1u);
                            m0 = q == 0 ? nb2 : m0; m1 = q == 1 ? nb2 : m1; m2 = q == 2 ? nb2 : m2; m3 = q == 3 ? nb2 : m3;
                            const int t = __builtin_ctz(mb);
                            MK[ex] = (uint32_t)(us + 32 * q + 4 * (t & 7) + (t >> 3));
                            ++ex;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const int32_t c = lane < (int)tot ? (int32_t)MK[lane] : -1;
                    const bool act = c >= p0 && c < vhiT;
                    const uint64_t at0 = __ballot(act && c == p0);
                    Dec d = decode(act ? c : p0, act, at0 ? (int)__builtin_ctzll(at0) : 0, false, vhiT);
                    const uint32_t nxp = act && d.ok ? d.nx : N32;
                    const int32_t wend = cover < vhiT ? cover : vhiT;
                    // each candidate's successor slot (KVR_SUCC): the row slots of the successor's unit
                    // come from that unit's lane by one ds_bpermute (start | count << 8), and the few
                    // slots are compared in parallel; -1 when none holds it (or the successor lies past
                    // the window, or is unknown)
                    int32_t sl = -1;
                    if (KVR_SUCC) {
                        const uint32_t rng = (fits && cnt) ? ((inc - cnt) | (cnt << 8)) : 0u;
                        const bool want = nxp < (uint32_t)wend;   // (UNK and N32 are past any window)
                        const uint32_t r2 =
                            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4u * (want ? nxp >> SC_LOG : 0u)), (int)rng);
                        const uint32_t s0 = r2 & 255u, sc = want ? (r2 >> 8) : 0u;
                        const uint32_t mx = wave_max(sc);
#pragma unroll 1
                        for (uint32_t t = 0; t < mx; ++t) {
                            const uint32_t pos = t < sc ? MK[(s0 + t) & 63u] : N32;
                            sl = (sl < 0 && pos == nxp) ? (int32_t)(s0 + t) : sl;
                        }
                    }
                    KVR_STAMP(11);
                    // the chain from p through the window's candidates
                    uint32_t rk = N32, vl = d.vlen;
                    int32_t cur = p0;
                    uint32_t nb = 0;
                    int lead = 0, lastl = 0;
                    int j = at0 ? (int)__builtin_ctzll(at0) : -1;   // the lane holding cur (-1: look it up)
#pragma unroll 1
                    while (cur < wend) {
                        if (j < 0) {
                            const uint64_t mm = __ballot(c == cur);
                            if (mm == 0ull) { go = false; break; }   // not a candidate: a broken record
                            j = (int)__builtin_ctzll(mm);
                        }
                        uint32_t nxj = rl32(nxp, j);
                        int jn = (int)rl32((uint32_t)sl, j);
                        if (nxj == UNK) {                      // another key length: its value length
                            const int32_t e = cur + 5 + (int32_t)rl32(d.klen, j);
                            const uint32_t vj = e + 8 <= TILE ? (uint32_t)tu64(e) : uni32(ts.u32(e));
                            nxj = vj <= (uint32_t)(remT - e - 4) ? (uint32_t)(e + 4) + vj : N32;
                            vl = wl32(vl, vj, (uint32_t)j);
                            jn = -1;
                        }
                        if (nxj == N32) { go = false; break; }   // a broken record: the exact loop reports it
                        rk = wl32(rk, nb, (uint32_t)j);
                        lead = nb == 0u ? j : lead;
                        lastl = j;
                        ++nb;
                        cur = (int32_t)nxj;
                        j = jn;
                    }
                    d.vlen = vl;
                    KVR_STAMP(12);
                    if (nb) {
                        const uint32_t slot0 = claim(nb);
                        const Fold fo = emit(d, c, rk != N32, rk, nb, lead, lastl, false, slot0);
                        if (fo.kind) fold_views(fo.lmark, (int32_t)d.vb, (int32_t)(d.vb + d.vlen), nrec + rk);
                        nrec = err_rec != N32 ? err_rec : nrec + nb;
                        if (go) stride = (uint32_t)(cur - (int32_t)rl32((uint32_t)c, lastl));
                    }
                    p = cur;
                    if (nb == 0u) go = false;
                    KVR_STAMP(13);
                }
            }
#endif
#endif
            // ---- the exact scalar hop loop: anything the lane-parallel framing left -----------
            // (entered only when the lane-parallel round left part of the tile: the loop's spill and
            // reload code then stays off the common path)
            if (p < vhi_r && err_rec == N32) {
            int64_t lastq = -1;              // the last record start it walked (its length is the next stride)
#pragma unroll 1
            while (p < vhi_r && !broke && err_rec == N32) {
                // exact hops; lane j keeps record nrec + j (per-lane selects)
                uint32_t nb = 0, kmx = 0, kmn = N32;   // the batch's longest and shortest key
                int32_t myrec = -1;
                uint32_t my_op = 0, my_klen = 0, my_vlen = 0;
                uint32_t lmark = 0, bl = 0;
                auto hops = [&](auto q) -> decltype(q) {
                    using T = decltype(q);
                    using U = std::make_unsigned_t<T>;
                    const T remT = (T)rem, vhiT = (T)vhi_r;
#pragma unroll 1
                    while (q < vhiT && nb < 64u) {
                        uint32_t op, klen;
                        if (q + 8 <= TILE) {
                            const uint64_t x = tu64((int)q);
                            op = (uint32_t)x & 255u;
                            klen = (uint32_t)(x >> 8);
                        } else {                     // the header crosses the tile end
                            op = uni32(ts.b8(q));
                            klen = remT - q >= 5 ? uni32(ts.u32(q + 1)) : 0u;
                        }
                        const bool me = lane == (int)nb;
                        lastq = (int64_t)q;
                        myrec = me ? (int32_t)q : myrec;
                        my_op = me ? op : my_op;
                        my_klen = me ? klen : my_klen;
                        ++nb;
                        if (op > 1u || remT - q < 5 || (U)klen > (U)(remT - q - 5)) { broke = true; break; }
                        kmx = klen > kmx ? klen : kmx;
                        kmn = klen < kmn ? klen : kmn;
                        const T e = q + 5 + (T)klen;
                        if (op == 1u) { q = e; continue; }
                        if (remT - e < 4) { broke = true; break; }
                        const uint32_t vlen = e + 8 <= TILE ? (uint32_t)tu64((int)e) : uni32(ts.u32(e));
                        my_vlen = lane == (int)nb - 1 ? vlen : my_vlen;
                        const T vb = e + 4;
                        if ((U)vlen > (U)(remT - vb)) { broke = true; break; }
                        const T e2 = vb + (T)vlen;
                        // a value longer than SMALL that crosses a unit boundary: fold it into every
                        // unit's view (one inside a single unit is CRC'd by its record's lane)
                        if (vlen > (uint32_t)SMALL && (vb >> SC_LOG) != ((e2 - 1) >> SC_LOG)) {
                            const uint64_t idx = nrec + nb - 1;
                            if (KVR_ABLATE & 32) any_long = true;
                            else if (vb < TILE) {
                                // (a 64-bit walk: the value may end more than 2^31 bytes on, so it
                                // is folded on the spot with its 64-bit end, not batched in 32 bits)
                                if constexpr (sizeof(T) == 8) consider((int32_t)vb, (uint64_t)(lo + e2), idx, false, false);
                                else { lmark = wl32(lmark, (nb << 6) | (nb - 1u), (uint32_t)vb >> SC_LOG); bl = 1; }
                            }
                            else { n_carry = 2; n_vb = (uint64_t)(lo + vb); n_ve = (uint64_t)(lo + e2); n_ref = idx; n_abs = false; }
                        }
                        q = e2;
                    }
                    return q;
                };
                if (huge) p = hops((int64_t)p);
                else p = hops((int32_t)p);
                if (bl) {
                    // lane j holds batch record j: its value [rvb, re2) (tile-relative)
                    const int32_t rvb = myrec + 9 + (int32_t)my_klen, re2 = rvb + (int32_t)my_vlen;
                    fold_views(lmark, rvb, re2, nrec + (uint32_t)lane);
                }
                const uint32_t slot = claim(nb) + (uint32_t)lane;
                // the batch's records: lane j emits record nrec + j
                uint32_t rerr = N32, rkind = 0;
                uint64_t raux = 0;
                const uint32_t j = nrec + (uint32_t)lane;
                if (KVR_REC_PRIO != KVR_HOP_PRIO) KVR_SETPRIO(KVR_REC_PRIO);
                if (!(KVR_ABLATE & 1) && myrec >= 0) {
                    if (broke && lane == (int)nb - 1) {   // the record that broke the chain: every check
                        const RecRes r = do_record(ts, K, myrec, j, slot, sd.seg, pool, kpool);
                        rerr = r.err; rkind = r.kind; raux = r.aux;
                        if (r.err == N32) { rerr = j; rkind = KVR_E_VAL; }   // defensive: a break is an error
                    } else {
                        const uint32_t kc = kmx > 4u * KEYW ? 4u * KEYW : kmx;
                        const uint32_t nw = (kc + 3u) >> 2;   // key words of the longest fast-path key
                        const int kb = myrec + 5;
                        const uint32_t klen = my_klen;
                        uint32_t c = ~0u, bad = 0x80u;
                        if (kmn == kmx && kmx <= 4u * KEYW && kb + 4 * KEYW + 8 <= ts.lim) {   // one key length
                            const int a = kb & ~3;
                            uint32_t r[KEYW + 1];
#pragma unroll
                            for (int i = 0; i <= KEYW; ++i) r[i] = (uint32_t)i <= nw ? ts.w32a(a + 4 * i) : 0u;
                            c = crc_words_u<KEYW>(r, K, (uint32_t)kb & 3u, kmx, &bad);
                        } else if (klen <= 4u * KEYW && kb + 4 * KEYW + 8 <= ts.lim) {
                            c = crc_span<KEYW>(ts, K, kb, klen, nw, &bad);
                        }
                        if (bad != 0u) {              // non-ASCII or long key: the full UTF-8 check
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
                            t.val_len = my_op == 0u ? my_vlen : 0u;
                            t.crc32 = my_op == 0u ? short_value_crc(ts, K, kb + (int)klen + 4, my_vlen) : 0u;
                            t.key_tag = ~c;
                            t.op = (uint8_t)my_op;
                            t.flags = 0;
                            t.reserved = 0;
                            pool[slot] = t;
                            if (kpool) kpool[slot] = key_prefix_mem(ts, kb, klen);
                        }
                    }
                }
                // first error of the batch (lowest record index)
                if (__ballot(rerr != N32)) {
                    const int el = (int)__builtin_ctzll(__ballot(rerr != N32));
                    err_rec = rl32(rerr, el);
                    err_kind = rl32(rkind, el);
                    err_aux = rl64(raux, el);
                    err_pos = (uint64_t)(lo + (int64_t)(int32_t)rl32((uint32_t)myrec, el));
                }
                nrec = err_rec != N32 ? err_rec : nrec + nb;
                if (KVR_REC_PRIO != KVR_HOP_PRIO) KVR_SETPRIO(KVR_HOP_PRIO);
            }
            if (lastq >= 0 && !broke && !huge) stride = (uint32_t)(p - lastq);
            }
            if (KVR_HOP_PRIO) KVR_SETPRIO(0);
            tile_exit = broke ? ERRP : (uint64_t)(lo + p);
        }
        // the tile's result record, stored ahead of the next tile's load, so that the wait for that
        // load at the loop top does not also wait for this store's ack
        auto tile_result = [&]() {
            if (c1 == N32) c1 = nrec;
            if (in_stripe && lane == 0) {
                TileRes tr;
                tr.pool_off = nrec ? (uint64_t)b1 : 0ull;
                tr.pool_off2 = b2;
                tr.count = nrec;
                tr.count1 = c1 < nrec ? c1 : nrec;
                tres[sg.tile0 + k] = tr;
            }
        };
        // a record index of this tile -> its pool slot
        auto slot_of = [&](uint32_t ref, bool is_abs) -> uint32_t {
            return is_abs ? ref : (ref < c1 ? b1 + ref : b2 + (ref - c1));
        };
        tile_result();
        if (n_carry == 2u && !n_abs) n_ref = slot_of(n_ref, false);
        // the stripe goes on past this tile (a value running past its end is carried on)
        const bool need_next = err_pos == NONE && k + 1 < sg.n_tiles && (k + 1 < sd.t_end || n_carry || out);
        KVR_STAMP(2);
        // the word of a value end's partial tail, for the finalize (its latency runs under the unit loop)
        uint32_t wm = 0;
        if (!(KVR_ABLATE & 2) && any_long && m != 0 && m < SC) wm = ts.w32a(us + 4 * (m >> 2));
        // ---- C. CRC of long values --------------------------------------------------------
        if (!(KVR_ABLATE & 2) && any_long) {
            KVR_STAMP(8);
            // the unit's two halves, words 0..15 (A) and 16..31 (B), CRC'd as independent chains
            // from a zero register, with the snapshot of the raw CRC of the unit's first 4 qm
            // bytes (the value ending here) and the restart at the value starting here (a)
            constexpr int H = UW / 2;
            const int qm = m >> 2;
            const int qa = (vx && a_off >= 0) ? (a_off >> 2) : -1;
            const uint32_t amask = ~0u << (8 * (a_off & 3));
            // (one compare per step: q & 15 picks the step, a loop-invariant lane mask the chain)
            const int qh = qm & (H - 1), qah = qa >= 0 ? (qa & (H - 1)) : -1;
            const bool mb = qm >= H, ab = qa >= H;
            // The chains carry the step input x = register ^ word rather than the register: the
            // lookups' XOR and the next word go into one v_bitop3.  A snapshot takes x at the value
            // end's word (the register there is x ^ that word, wm, loaded before the loop), and a
            // restart replaces x by the masked word: x = w & amask.
            uint32_t ca = 0, cb = 0, sn = 0;
            if (KVR_ABLATE & 8) {
                ca = w[0]; cb = w[1];
            } else if (!__ballot(m != 0 || qa >= 0)) {
                uint32_t xa = w[0], xb = w[H];
#pragma unroll
                for (int kk = 0; kk < H; ++kk) {
                    uint32_t ta, a3, tb, b3;
                    look4x2(xa, xb, K, ta, a3, tb, b3);
                    if (kk + 1 < H) {
                        xa = xor3(ta, a3, w[kk + 1]);
                        xb = xor3(tb, b3, w[kk + 1 + H]);
                    } else {
                        ca = ta ^ a3;
                        cb = tb ^ b3;
                    }
                }
            } else {
                uint32_t xa = (qah == 0 && !ab) ? (w[0] & amask) : w[0];
                uint32_t xb = (qah == 0 && ab) ? (w[H] & amask) : w[H];
                uint32_t snx = 0;
#pragma unroll
                for (int kk = 0; kk < H; ++kk) {
                    snx = kk == qh ? (mb ? xb : xa) : snx;
                    uint32_t ta, a3, tb, b3;
                    look4x2(xa, xb, K, ta, a3, tb, b3);
                    if (kk + 1 < H) {
                        xa = xor3(ta, a3, w[kk + 1]);
                        xb = xor3(tb, b3, w[kk + 1 + H]);
                        const bool r = kk + 1 == qah;
                        xa = (r && !ab) ? (w[kk + 1] & amask) : xa;
                        xb = (r && ab) ? (w[kk + 1 + H] & amask) : xb;
                    } else {
                        ca = ta ^ a3;
                        cb = tb ^ b3;
                    }
                }
                sn = qm == UW ? cb : (snx ^ wm);
            }
            // the unit loop was the tile registers' last reader: the next tile's load is issued
            // here and its latency runs under the scan and the finalize (a speculative tile's, after
            // the scan, behind its windows)
            if (need_next && !loaded) {
                load_unit(abase, d0, len, k + 1, lane, w);
                loaded = true;
            }
            // the piece of the value crossing the unit end: A pushed through B's bytes, then B
            // (A does not count when that value starts in B's half); the raw CRC of the first
            // 4 qm bytes: A's snapshot, or all of A pushed through 4 (qm - H) bytes, then B's
            if (KVR_FIN_PRIO) KVR_SETPRIO(KVR_FIN_PRIO);
            const uint32_t pa = kmul(ca, S.KQ2);
            const uint32_t c = qa >= H ? cb : (pa ^ cb);
            KVR_STAMP(9);
            uint32_t v = 0, fm = N32;            // segment start fm (all ones): no inflow from the previous unit
            if (vx) {
                if (a_off >= 0) v = c ^ S.IX[SC - a_off];
                else if (lane == 0 && vx_carry) v = c ^ kmul(c_state, S.KQ2 + 128);   // carried register across unit 0
                else { v = c; fm = 0u; }
            }
            // every piece pushed straight to where it is consumed (the unit before the one the
            // value ends in, or lane 63 for a value running past the tile): one multiply by
            // x^(8 SC d), then a segmented XOR scan (DPP only) sums each value's pieces there
            // (state at the end of unit l = f ? v : state(l-1) * x^(8*SC) ^ v)
            if (!(KVR_ABLATE & 16)) {
                const int32_t ce = vx > TILE ? 63 : ((vx - 1) >> SC_LOG) - 1;   // (vx = 0: v = 0)
                const int32_t dd = ce - lane;
                // (a lane with no push reads the broadcast entry of a zero register: its lookups add no
                // distinct address to column 0's bank)
                const uint32_t t_ = kmul_col<KR_OFF, KR_PITCH>(dd > 0 ? v : 0u, S, dd > 0 ? 4u * (uint32_t)(dd - 1) : 0u);
                v = dd > 0 ? t_ : v;
                // (a lane without a source reads 0 from the DPP move -- row_shr past the row start,
                // the rows a broadcast skips -- which adds nothing and starts no segment, so no lane
                // test is needed: v ^= inflow unless a segment starts here, fm |= the inflow's fm)
#define KVR_XSCAN_STEP(CTRL, RM, BC)                                         \
            {                                                                \
                const uint32_t ov = dpp<CTRL, RM, BC>(v);                    \
                v = bitop3_xandn(v, ov, fm);                                 \
                fm |= dpp<CTRL, RM, BC>(fm);                                 \
            }
                KVR_XSCAN_STEP(0x111, 0xF, true)
                KVR_XSCAN_STEP(0x112, 0xF, true)
                KVR_XSCAN_STEP(0x114, 0xF, true)
                KVR_XSCAN_STEP(0x118, 0xF, true)
                KVR_XSCAN_STEP(0x142, 0xA, false)
#undef KVR_XSCAN_STEP
                v = bitop3_xandn(v, dpp<0x143, 0xC, false>(v), fm);
            }
            KVR_STAMP(10);
            uint32_t sin = dpp<0x138>(v);        // wave_shr:1: the state at this unit's start
            if (lane == 0) sin = c_state;
            // the value ending in this unit at m: its register is sin * x^(8m) ^ raw[0, m), and
            // raw[0, 4 qm) is A's snapshot, or all of A pushed through 4 (qm - H) bytes ^ B's: so
            // (base * x^(8*4q) ^ sn) with base = sin, q = qm, or base = sin * x^(8*4H) ^ A, q = qm - H
            // (one per-lane multiply); then the r = m & 3 bytes past 4 qm, by linearity one chain
            if (!(KVR_ABLATE & 16) && m != 0) {
                const int r = m & 3;
                const uint32_t base = mb ? (kmul(sin, S.KQ2) ^ ca) : sin;
                uint32_t t = kmul_col<KQL_OFF, KQL_PITCH>(base, S, 4u * (uint32_t)(mb ? qm - H : qm)) ^ sn;
                for (int b = 0; b < r; ++b) t = crc1(t, (wm >> (8 * b)) & 255u, K);
                pool[slot_of(m_ref, m_abs)].crc32 = ~t;
            }
            if (out) {                           // the value running past the tile: hand over its register
                n_carry = 1;
                c_state = rl32(v, 63);
                n_ve = out_ve;
                n_ref = slot_of(out_ref, out_abs);
            }
        }

        if (KVR_FIN_PRIO) KVR_SETPRIO(0);
        // the tile's registers are dead from here on: the next tile's load overlaps the rest
        if (!loaded && err_pos == NONE && k + 1 < sg.n_tiles && (k + 1 < sd.t_end || n_carry)) {
            load_unit(abase, d0, len, k + 1, lane, w);
            loaded = true;
        }
        KVR_STAMP(3);
        // ---- bookkeeping ------------------------------------------------------------------
        if (in_stripe) {
            total += nrec;
            if (walk) entry = tile_exit;
        }
        carry = n_carry;
        c_vb = n_vb; c_ve = n_ve; c_slot = n_ref;
        if (err_pos != NONE) stop = 1;
        else if (walk && tile_exit == ERRP) {   // defensive: a broken chain must have reported
            stop = 1; err_pos = entry; err_kind = KVR_E_VAL;
        }
        KVR_STAMP(4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain an unused next-tile load
    if (rb_on) {   // out of the mean
        if (lane == 0) { atomicSub(&S.BAL[0], rb_own); atomicSub(&S.BAL[1], 1u); }
        __builtin_amdgcn_s_setprio(0);
    }
#ifdef KVR_PROF
    if (lane == 0) {
        for (int i = 0; i < 16; ++i) atomicAdd(&g_prof[i], prof_acc[i]);
        if (!REDO && !hand && si < 16384u) {   // (per stripe, as k_piece's: k_replay alone, KVR_NO_PIECE)
            g_pst[4 * si] = rrt0;
            g_pst[4 * si + 1] = __builtin_amdgcn_s_memrealtime();
            g_pst[4 * si + 2] = __builtin_amdgcn_s_getreg(0xF804);
            g_pst[4 * si + 3] = __builtin_amdgcn_s_getreg(0xF814);
        }
    }
#endif
    // tiles of the stripe that were never reached (error stop / pass-through) hold no tuples
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
        r.owned = redo_mode ? 1u : 0u;
        r.pool_run = run_contig && run_first != N32 ? (uint64_t)run_first : NONE;
        r.pad = 0;
        sres[si] = r;
        if (scnt) scnt[si] = total;   // (dense, for k_compact_s's own stripe offsets)
    }
    // ---- redo pass: walk on into the next stripe of the segment --------------------------------
    // while its speculated result (last pass) disagrees with the chain position this walk reached,
    // `entry` (the walked exit, or the imposed entry a pass-through stripe keeps), as k_link would
    // find; a stripe listed for its own re-walk in this pass (owned bit 0) is left to its wave
    if (!REDO || err_pos != NONE || trapped) break;
    const uint32_t nx = si + 1;
    if (nx >= n_stripes || entry == NONE) break;
    const StripeDesc nd = stripes[nx];
    if (nd.seg != sd.seg) break;
    const StripeRes nr = sres[nx];        // (no other wave writes it in this pass)
    if (nr.owned & 1u) break;
    const int64_t nhi_i = (int64_t)nd.t_end * TILE - d0;
    const uint64_t n_hi = (uint64_t)nhi_i > len ? len : (uint64_t)nhi_i;
    if (nr.entry == NONE ? entry >= n_hi : nr.entry == entry) break;   // consistent: the chain joins
    si = nx;
    forced = entry;
    }
}

__global__ __launch_bounds__(RT) void k_replay(const SegDesc *__restrict__ segs,
                                               const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                               StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                               kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                               Tables tb, uint32_t pool_chunk, uint4 *__restrict__ kpool,
                                               uint32_t *__restrict__ scnt, const PieceHand *__restrict__ hand) {
    replay_body<false>(segs, stripes, n_stripes, sres, tres, pool, pool_cap, ctr, tb, nullptr, nullptr, pool_chunk, kpool,
                       scnt, hand);
}

// (half the workgroup of k_replay: two waves a SIMD, so the REDO body's state fits 256 VGPRs unspilled;
// the fallback re-walks few stripes, occupancy does not matter there)
__global__ __launch_bounds__(RT_REWALK) void k_rewalk(const SegDesc *__restrict__ segs,
                                               const StripeDesc *__restrict__ stripes, uint32_t n_stripes,
                                               StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                               kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                               Tables tb, const RedoEnt *__restrict__ redo,
                                               const LinkResult *__restrict__ link, uint32_t pool_chunk,
                                               uint4 *__restrict__ kpool) {
    replay_body<true, RT_REWALK>(segs, stripes, n_stripes, sres, tres, pool, pool_cap, ctr, tb, redo, link, pool_chunk, kpool,
                      nullptr, nullptr);
}


// k_piece's check before a run: records 1 .. KVR_PCHECK - 1 after the one at Pe (those starting
// before s_hi) are SETs of key length ku and value length vu that fit the segment, one lane each
// (out of line: inlined, its registers changed the allocation of the step loop, cfg2 +8 %)
__device__ __attribute__((noinline)) bool run_heads_equal(const uint8_t *base, uint64_t len, uint64_t Pe, uint32_t L,
                                                          uint32_t ku, uint32_t vu, uint64_t s_hi, int lane) {
    const uint64_t pj = Pe + (uint64_t)lane * L;
    bool bad = false;
    if (lane > 0 && lane < KVR_PCHECK && pj < s_hi) {
        if (pj + L > len) {
            bad = true;
        } else {
            const __amdgpu_buffer_rsrc_t rj = seg_rsrc(base, pj, len);
            const uint32_t a = __builtin_amdgcn_raw_buffer_load_b32(rj, 0, 0, 0);   // (unaligned)
            const uint32_t b = __builtin_amdgcn_raw_buffer_load_b32(rj, 4, 0, 0);
            const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rj, 5 + (int)ku, 0, 0);
            bad = (a & 255u) != 0u || ((a >> 8) | (b << 24)) != ku || v != vu;
        }
    }
    return __ballot(bad) == 0ull;
}

// ---------------------------------------------------------------------------------------
// k_piece: the piece mode, first over every stripe.
// ---------------------------------------------------------------------------------------
// A stripe that starts with a run of SETs of one key length ku and one value length vu >= KVR_UMIN
// is replayed value-aligned: every value is cut into P = ceil(vu / 128) pieces that end at its last
// byte (the first holds r = vu - 128 (P - 1) bytes behind 128 - r masked ones); lane l of a step CRCs
// piece 64 s + l of the run from a zero register, pushes it by x^(8 128 d) to the lane that completes
// the value (or carries it on, lane 63), and a segmented XOR scan sums each value there.  No value
// boundary falls inside a lane's bytes: no snapshot, restart or finalize (~400 VALU per 8 KiB,
// profiles/r06/final_pmc_cfg2.txt).  A record's 48-B header window is loaded in the step its value
// completes and waits in the wave's LDS row; groups of completed records are verified against the
// prediction (opcode, key length, value length, segment end, UTF-8 key) and emitted with their value
// CRCs, the run's first pool chunk in run form (PieceRun + 8 B a record).  The first record not as
// predicted ends the run, and the stripe is handed to k_replay's tile loop at that record (PieceHand);
// so is a stripe that does not start with such a record, or whose entry the search has not found in
// its first tiles.
// k_piece's workgroup (KVR_PNT threads: 16 waves, four per SIMD at up to 128 VGPRs; 512 = 8 waves at
// up to 256, each wave then taking two stripes one after the other) and the piece buffers a wave keeps
// (KVR_PNB: the step being worked on and KVR_PNB - 1 loading behind it).  A workgroup takes the WPB
// stripes k_replay's workgroup of the same index takes (profiles/r06/ab_piece_layouts.txt: 16 waves x 2
// buffers is the fastest that fits; 8 waves x 3 buffers and 16 x 1 were slower).
#ifndef KVR_PNT
#define KVR_PNT 1024
#endif
#ifndef KVR_PNB
#define KVR_PNB 2
#endif
#ifndef KVR_PRUNFORM   // 1: a run's first pool chunk in run form (PieceRun, 8 B a record: the tuples' writes,
#define KVR_PRUNFORM 1     // mixed into k_piece's read stream, cost it 0.05-0.15 ms on cfg2)
#endif
#ifndef KVR_PWIDE   // 1: a flush writes its tuples as whole 128-B lines (0: one tuple a lane, two 16-B halves)
#define KVR_PWIDE 0
#endif
#ifndef KVR_PWEARLY   // 1: a step's windows are loaded before its next pieces and CRC (their lines are still in
#define KVR_PWEARLY 0    // L2 from the pieces; 0: after the CRC, no window registers across it)
#endif
#ifndef KVR_PWROW   // 1: the header windows of a group wait in the wave's LDS row (0: in registers)
#define KVR_PWROW 1
#endif
#ifndef KVR_PWDMA   // 1 (with KVR_PWROW): a step's header windows go straight from memory into the wave's LDS
#define KVR_PWDMA 1     // row (buffer_load ... lds: no registers), issued before the step's next pieces while
#endif                  // their lines are still in L2 from the step's own pieces (0: through registers, after the CRC)
#ifndef KVR_PWDMA_AFTER   // 1: the DMA windows after the next pieces, before the CRC (timing A/B; the flush
#define KVR_PWDMA_AFTER 0     // then waits vmcnt(0))
#endif
#ifndef KVR_PWDMA_VMC   // the flush's wait for its windows: 9 (the pieces issued behind them stay in flight) or 0
#define KVR_PWDMA_VMC (KVR_PWDMA_AFTER ? 0 : 9)
#endif
constexpr int PNT = KVR_PNT, PNB = KVR_PNB, PSPW = WPB / (PNT / 64);
static_assert(PNT / 64 <= KVR_PWMAX, "one LDS window row per wave");
static_assert(PSPW * (PNT / 64) == WPB && PNB >= 1 && PNB <= 3, "k_piece layout");

// one stripe of k_piece (the kernel below): j = the wave's j-th stripe (progress balance)
template <int NB>
__device__ __forceinline__ void piece_stripe(const uint32_t si, const uint32_t j, SmemP &S, const Crc &K, const int lane,
                                             const int wv,
                                             const SegDesc *__restrict__ segs, const StripeDesc *__restrict__ stripes,
                                             StripeRes *__restrict__ sres, TileRes *__restrict__ tres,
                                             kvr_tuple *__restrict__ pool, uint64_t pool_cap, Counters *ctr,
                                             uint32_t pool_chunk, uint4 *__restrict__ kpool, uint32_t *__restrict__ scnt,
                                             PieceHand *__restrict__ hand, uint2 *__restrict__ pcrc,
                                             PieceRun *__restrict__ prun) {
    uint32_t *const bal = S.BAL;   // [0] the progress of the waves in their step loop, [1] their number
    if (prun && lane == 0) prun[si] = PieceRun{0ull, 0u, 0u, 0u, 0u, 0u, 0u};   // (no run form yet)
#ifdef KVR_PROF
    // (diagnostic build: cycles per phase into g_prof 0-5, 8-9, counts in 6-7, s_memrealtime 12-14;
    // tools/prof_phases.py)
    unsigned long long pt_last = __builtin_amdgcn_s_memtime();
    const unsigned long long prt0 = __builtin_amdgcn_s_memrealtime();   // (100 MHz: the clock's rate)
    unsigned long long pacc[10] = {};
#define KVR_PSTAMP(i)                                                       \
    do {                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();         \
        pacc[i] += t_ - pt_last;                                            \
        pt_last = t_;                                                       \
    } while (0)
#define KVR_PCOUNT(i) (pacc[i] += 1)
#define KVR_PFLUSH()                                                        \
    do {                                                                    \
        if (lane == 0) {                                                    \
            for (int i_ = 0; i_ < 10; ++i_) atomicAdd(&g_prof[i_], pacc[i_]); \
            const unsigned long long prt1 = __builtin_amdgcn_s_memrealtime(); \
            atomicAdd(&g_prof[12], prt1 - prt0);                            \
            atomicMax(&g_prof[13], prt1);                                   \
            atomicMax(&g_prof[14], ~prt0);                                 \
            if (si < 16384u) {                                              \
                g_pst[4 * si] = prt0;                                       \
                g_pst[4 * si + 1] = prt1;                                   \
                g_pst[4 * si + 2] = __builtin_amdgcn_s_getreg(0xF804);      \
                g_pst[4 * si + 3] = __builtin_amdgcn_s_getreg(0xF814);      \
            }                                                               \
        }                                                                   \
    } while (0)
#else
#define KVR_PSTAMP(i) do { } while (0)
#define KVR_PCOUNT(i) do { } while (0)
#define KVR_PFLUSH() do { } while (0)
#endif
    const StripeDesc sd = stripes[si];
    const SegDesc sg = segs[sd.seg];
    const uint64_t len = sg.len;
    const int64_t d0 = sg.d0;
    const int64_t shi_i = (int64_t)sd.t_end * TILE - d0;
    const uint64_t s_hi = (uint64_t)shi_i > len ? len : (uint64_t)shi_i;
    const uint8_t *abase = sg.base - d0;
    uint32_t w[UW + 1];
    // ---- the entry: offset 0 for a segment's first stripe, else the first plausible record start
    uint64_t entry = sd.t_begin == 0 ? 0ull : NONE;
    uint32_t k = sd.t_begin;
    if (entry == NONE) {
#pragma unroll 1
        for (; k < sd.t_end && k < sg.n_tiles && k < sd.t_begin + KVR_PSEARCH; ++k) {
            load_unit(abase, d0, len, k, lane, w);
            const int64_t lo = (int64_t)k * TILE - d0;
            const int64_t vlo_r = lo < 0 ? -lo : 0;
            const int64_t vhi_r = (lo + TILE > (int64_t)len ? (int64_t)len : lo + TILE) - lo;
            const int us = lane * SC, ue = us + SC;
            const TileSeg ts = tile_seg(abase, sg.base, d0, len, k);
            entry = find_entry(*reinterpret_cast<uint32_t(*)[UW]>(w), ts, lo, (int64_t)len - lo, us > (int)vlo_r ? us : (int)vlo_r,
                               ue < (int)vhi_r ? ue : (int)vhi_r, lane);
            if (entry != NONE) break;
        }
    }
    const uint64_t stripe_entry = (entry != NONE && entry >= s_hi) ? NONE : entry;
    // the wave's pool chunk and the stripe's run of slots
    uint32_t chunk_base = 0, chunk_left = 0, run_first = N32, total = 0;
    bool run_contig = true;
    auto tile_of = [&](uint64_t pos) -> uint32_t { return (uint32_t)((pos + (uint64_t)d0) >> 13); };
    // hand the stripe to k_replay at the record at pos (tile k_res, `ah` of its records emitted here)
    auto hand_back = [&](uint64_t pos, uint32_t k_res, uint32_t ah, uint32_t stride) {
        if (lane == 0) {
            PieceHand h;
            h.entry = pos;
            h.stripe_entry = stripe_entry;
            h.k = k_res;
            h.ahead = ah;
            h.stride = stride;
            h.total = total;
            h.chunk_base = chunk_base;
            h.chunk_left = chunk_left;
            h.run_first = run_first;
            h.run_contig = run_contig ? 1u : 0u;
            h.done = 0;
            h.pad = 0;
            hand[si] = h;
        }
    };
    // the stripe is done here (exit: the first record start at or after its end, NONE when none starts in it)
    auto finish = [&](uint64_t exit) {
        if (lane == 0) {
            StripeRes r;
            r.entry = stripe_entry;
            r.exit = stripe_entry == NONE ? NONE : exit;
            r.err_pos = NONE;
            r.err_aux = 0;
            r.err_kind = 0;
            r.count = total;
            r.forced = 0;
            r.owned = 0;
            r.pool_run = run_contig && run_first != N32 ? (uint64_t)run_first : NONE;
            r.pad = 0;
            sres[si] = r;
            if (scnt) scnt[si] = total;
            PieceHand h = {};
            h.done = 1;
            hand[si] = h;
        }
    };
    if (entry == NONE && k < sd.t_end && k < sg.n_tiles) {
        // no record start in the first KVR_PSEARCH tiles (a long value crosses them): k_replay searches
        // on from tile k (a serial walk over a 1-MiB value here held its whole launch back, cfg5)
        for (uint32_t t = sd.t_begin + (uint32_t)lane; t < k; t += 64u) {
            TileRes tr;
            tr.pool_off = 0; tr.pool_off2 = 0; tr.count = 0; tr.count1 = 0;
            tres[sg.tile0 + t] = tr;
        }
        hand_back(NONE, k, 0u, 0u);
        return;
    }
    if (entry == NONE) {   // no record starts in the stripe (or the search ran past its tiles)
        for (uint32_t t = sd.t_begin + (uint32_t)lane; t < sd.t_end; t += 64u) {
            TileRes tr;
            tr.pool_off = 0; tr.pool_off2 = 0; tr.count = 0; tr.count1 = 0;
            tres[sg.tile0 + t] = tr;
        }
        finish(NONE);
        return;
    }
    // ---- the prediction: the record at the entry
    const uint64_t Pe = entry;
    uint32_t ku = 0, vu = 0;
    bool uni = false;
    if (Pe < s_hi && Pe + 9u <= len) {
        const __amdgpu_buffer_rsrc_t rs0 = seg_rsrc(sg.base, Pe, len);
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs0, 0, 0, 0);
        ku = (a.x >> 8) | (a.y << 24);
        if ((a.x & 255u) == 0u && ku <= 4u * UKEYW && Pe + 9u + ku <= len) {
            vu = __builtin_amdgcn_raw_buffer_load_b32(rs0, 5 + (int)ku, 0, 0);   // (unaligned)
            uni = vu >= (uint32_t)KVR_UMIN && vu <= UMAXV && Pe + 9u + ku + vu <= len;
        }
        ku = uni32(ku);
        vu = uni32(vu);
        uni = __builtin_amdgcn_readfirstlane(uni ? 1 : 0) != 0;
    }
    const uint32_t L = 9u + ku + vu;
    const uint32_t P = (vu + (uint32_t)SC - 1u) >> SC_LOG, r = vu - (uint32_t)SC * (P - 1u);
    // a run shorter than KVR_PCHECK records is not worth the run's setup (a SET/DEL mix like cfg4's
    // ends most runs at the second record): the next records' headers, one lane each, before it
    if (uni && KVR_PCHECK > 1) uni = run_heads_equal(sg.base, len, Pe, L, ku, vu, s_hi, lane);
    // (a first piece's window starts 128 - r bytes before its value: inside the segment)
    if (!uni || Pe + 9u + ku + r < (uint64_t)SC || !KVR_UMODE) {
        for (uint32_t t = sd.t_begin + (uint32_t)lane; t < k; t += 64u) {   // the tiles the search passed
            TileRes tr;
            tr.pool_off = 0; tr.pool_off2 = 0; tr.count = 0; tr.count1 = 0;
            tres[sg.tile0 + t] = tr;
        }
        hand_back(Pe, k, 0u, 0u);
        return;
    }
    // ---- the run
    const uint32_t q_end = (uint32_t)((s_hi - Pe + L - 1u) / L);   // records starting in the stripe (Pe < s_hi)
    const uint64_t q_fit64 = (len - Pe) / L;                         // records ending inside the segment
    const uint32_t q_fit = q_fit64 > (uint64_t)q_end ? q_end : (uint32_t)q_fit64;
    const int32_t G = (int32_t)L - (int32_t)((uint32_t)SC * P);   // window offset per record beyond 128 P
    const uint32_t IXr = S.IX[r];                                   // ~0 * x^(8 r)
    const float invP = 1.0f / (float)P;
    const uint32_t adv_q = 64u / P, adv_p = 64u % P;                // a step: 64 = adv_q P + adv_p pieces
    const uint32_t zr = (uint32_t)SC - r;                           // masked leading bytes of a first piece
    // TileRes: tiles [t_done, ...) not yet written; the open run of slots (one chunk) starts at tile
    // seg_tile, slot seg_b, seg_n records
    uint32_t t_done = sd.t_begin, seg_tile = tile_of(Pe), seg_b = 0, seg_n = 0;
    auto close_tiles = [&](uint32_t t_to, uint32_t n_seg) {   // [t_done, t_to): the run at seg_tile, else empty
        for (uint32_t t = t_done + (uint32_t)lane; t < t_to; t += 64u) {
            const bool st = t == seg_tile && n_seg != 0u;
            TileRes tr;
            tr.pool_off = st ? (uint64_t)seg_b : 0ull;
            tr.pool_off2 = 0;
            tr.count = st ? n_seg : 0u;
            tr.count1 = tr.count;
            tres[sg.tile0 + t] = tr;
        }
    };
    // the group: records qg .. in lanes 0 .. (their header windows and value CRCs)
    uint32_t qg = 0, vcrc = 0;
    bool early = true;   // the first completed records are verified at once: a stripe that is not uniform
#if !KVR_PWROW
    uint32_t win[13], wsh = 0;   // hands back after one step's work.  (A record's window: the 13 dwords
#pragma unroll                 // from the one holding its first byte, wsh bytes in.)
    for (int i = 0; i < 13; ++i) win[i] = 0u;
#endif
    uint32_t gadj;
    __amdgpu_buffer_rsrc_t grs = seg_rsrc_a(sg.base, Pe, len, gadj);
    bool ustop = false;
    // verify and emit the group's first n records; a record not as predicted stops the run there
    auto flush = [&](uint32_t n) {
        KVR_PCOUNT(7);
        if (KVR_PABLATE & 16) {   // (diagnostic: the run's bookkeeping only)
            qg += n;
            grs = seg_rsrc_a(sg.base, Pe + (uint64_t)qg * L, len, gadj);
            return;
        }
        const uint64_t GB = Pe + (uint64_t)qg * L;
        const bool on = (uint32_t)lane < n;
        uint32_t x[12];   // the record's first 48 bytes
#if KVR_PWROW
        {   // the window from the wave's LDS row, realigned by its byte offset in the dword it was loaded
            // from (the same group base gadj as at its load: the group moves only in a flush)
            uint32_t wr[PWIN];
            if (KVR_PWDMA) {   // (the row as [3][64 lanes][4 dwords]: what the DMA loads wrote,
                               // each landed once every load issued before it has: the group's are all older)
                // (every flush runs where the last window loads it reads were followed by one step's
                // pieces, 9 loads issued unconditionally: vmcnt(9) has them landed, the pieces in flight)
                if (KVR_PWDMA_VMC == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t *const rw = &S.WROW[wv][0][0];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const uint4 v4 = reinterpret_cast<const uint4 *>(rw + 256 * i)[lane];
                    wr[4 * i] = v4.x; wr[4 * i + 1] = v4.y; wr[4 * i + 2] = v4.z; wr[4 * i + 3] = v4.w;
                }
                wr[12] = 0u;   // (bytes 48-51: past any byte the flush reads)
            } else {
#pragma unroll
                for (int i = 0; i < PWIN; ++i) wr[i] = (KVR_PABLATE & 1024) ? 0u : S.WROW[wv][i][lane];
            }
            const uint32_t wsh = ((uint32_t)lane * L + gadj) & 3u;
#pragma unroll
            for (int i = 0; i < 12; ++i) x[i] = __builtin_amdgcn_alignbyte(wr[i + 1], wr[i], wsh);
        }
#else
#pragma unroll
        for (int i = 0; i < 12; ++i) x[i] = __builtin_amdgcn_alignbyte(win[i + 1], win[i], wsh);
#endif
        const uint32_t op = x[0] & 255u, klen = (x[0] >> 8) | (x[1] << 24);
        uint32_t vl;
        {   // the value length at byte 5 + ku of the window
            const uint32_t t = 5u + ku, tw = t >> 2;
            uint32_t a = 0, b = 0;
#pragma unroll
            for (int i = 0; i < 11; ++i)
                if (tw == (uint32_t)i) { a = x[i]; b = x[i + 1]; }
            vl = __builtin_amdgcn_alignbyte(b, a, t & 3u);
        }
        // the key CRC from the window; a key with a byte >= 0x80 stops the run (k_replay runs the
        // full UTF-8 check, engine.rs:114)
        uint32_t kr[UKEYW + 1];
#pragma unroll
        for (int i = 0; i <= UKEYW; ++i) kr[i] = x[i + 1];
        uint32_t bad = 0;
        const uint32_t kc = (KVR_PABLATE & 256) ? kr[0] : crc_words_u<UKEYW>(kr, K, 1u, ku, &bad);
        const bool ok = on && (((KVR_PABLATE & 512) != 0) || (op == 0u && klen == ku && vl == vu && bad == 0u)) &&
                        qg + (uint32_t)lane < q_fit;
        const uint64_t bm = __ballot(on && !ok);
        const uint32_t f = bm ? (uint32_t)__builtin_ctzll(bm) : n;
        // slots from the wave's chunk; a fresh chunk only where a tile starts, so that every tile's
        // records stay one run (k_replay takes a handed-back tile's from chunk_base back)
        uint32_t m = f < chunk_left ? f : chunk_left;
        if (m < f && chunk_left == 0u && (qg == 0u || tile_of(GB) != tile_of(GB - L))) {
            const uint32_t tq = tile_of(GB);
            close_tiles(tq, seg_n);
            const uint32_t cmx = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
            unsigned long long bb = 0;
            if (lane == 0) {
                bb = atomicAdd(&ctr->pool_cursor, (unsigned long long)cmx);
                if (bb + cmx > pool_cap) {   // past the pool: flag it, write into the slack
                    atomicOr(&ctr->overflow, 1u);
                    bb = pool_cap;
                }
            }
            chunk_base = uni32((uint32_t)bb);
            chunk_left = cmx;
            if (run_first != N32) run_contig = false;
            t_done = tq;
            seg_tile = tq;
            seg_b = chunk_base;
            seg_n = 0;
            m = f;
        }
        if (m != 0u && run_first == N32) run_first = chunk_base;
        const uint32_t cmx_r = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
        if (KVR_PRUNFORM && prun && m != 0u && chunk_base - run_first < cmx_r && !(KVR_PABLATE & 128)) {
            // the run's first chunk: run form, the value CRC and key tag only (8 B a record; the rest
            // of the tuple follows from the run, k_compact_s writes it)
            if ((uint32_t)lane < m) pcrc[chunk_base + (uint32_t)lane] = make_uint2(vcrc, ~kc);
            if (kpool && (uint32_t)lane < m) kpool[chunk_base + (uint32_t)lane] = key_prefix_words(&x[1], 1u, ku);
        } else if (KVR_PWIDE && !(KVR_PABLATE & (128 | 2048 | 4096))) {
            // the m tuples as whole lines: store i writes tuples 32 i .. 32 i + 31, lane l the half l & 1
            // of tuple 32 i + (l >> 1) (kvr_tuple's layout: op, flags 0), its CRCs from that tuple's lane
            const uint32_t ckc = ~kc;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t t = 32u * (uint32_t)i + ((uint32_t)lane >> 1), hf = (uint32_t)lane & 1u;
                const uint32_t cv = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (int)t, (int)vcrc);
                const uint32_t ck = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (int)t, (int)ckc);
                if (32u * (uint32_t)i < m) {
                    const uint64_t ro = GB + (uint64_t)t * L;
                    const u32x4 v = hf ? u32x4{vu, cv, ck, 0u} : u32x4{(uint32_t)ro, (uint32_t)(ro >> 32), sd.seg, ku};
                    // ((KVR_PABLATE & 8192): diagnostic, every wave's tuples into one 256-KiB stretch of the pool)
                    // ((KVR_PABLATE & 16384): diagnostic, the k-th flush of every stripe side by side)
                    const uint32_t slot = (KVR_PABLATE & 8192)    ? ((chunk_base + t) & 8191u)
                                          : (KVR_PABLATE & 16384) ? (uint32_t)(((uint64_t)(qg >> 6) * 4096u + si) * 64u + t) % (uint32_t)(pool_cap - 64)
                                                                  : chunk_base + t;
                    if (t < m) reinterpret_cast<u32x4 *>(pool + slot)[hf] = v;
                }
            }
            if (kpool && (uint32_t)lane < m) kpool[chunk_base + (uint32_t)lane] = key_prefix_words(&x[1], 1u, ku);
        } else if ((uint32_t)lane < m && !(KVR_PABLATE & 128)) {   // the 32-B tuple as two 16-B stores (kvr_tuple's layout: op, flags 0)
            const uint64_t ro = GB + (uint64_t)lane * L;
            uint4 *const tp = reinterpret_cast<uint4 *>(pool + chunk_base + (uint32_t)lane);
            if (KVR_PABLATE & 2048) {   // (diagnostic: 8 B a record)
                reinterpret_cast<uint2 *>(pool)[chunk_base + (uint32_t)lane] = make_uint2(vcrc, ~kc);
            } else if (KVR_PABLATE & 4096) {   // (diagnostic: non-temporal stores)
                u32x4 *const tq = reinterpret_cast<u32x4 *>(tp);
                __builtin_nontemporal_store(u32x4{(uint32_t)ro, (uint32_t)(ro >> 32), sd.seg, ku}, tq);
                __builtin_nontemporal_store(u32x4{vu, vcrc, ~kc, 0u}, tq + 1);
            } else {
                tp[0] = make_uint4((uint32_t)ro, (uint32_t)(ro >> 32), sd.seg, ku);
                tp[1] = make_uint4(vu, vcrc, ~kc, 0u);
            }
            if (kpool) kpool[chunk_base + (uint32_t)lane] = key_prefix_words(&x[1], 1u, ku);
        }
        chunk_base += m;
        chunk_left -= m;
        seg_n += m;
        qg += m;
        if (m < n) ustop = true;
        grs = seg_rsrc_a(sg.base, Pe + (uint64_t)qg * L, len, gadj);
    };
    // the steps, lane 0 at piece p_s of record q_s; step s + 1's pieces are loaded before step s is
    // processed (two piece buffers)
    struct Geo {
        uint64_t B;       // lane 0's window start (uniform); the resource starts at the dword holding it
        uint32_t dq, pv;
        int32_t o;        // this lane's window in the resource (its byte offset, adj included)
        bool act;
    };
    auto geo = [&](uint32_t q_s, uint32_t p_s) -> Geo {
        Geo g;
        g.B = Pe + (uint64_t)q_s * L + 9u + ku + r - (uint64_t)SC + (uint64_t)SC * p_s;
        const uint32_t adj = (uint32_t)((uint64_t)(sg.base + g.B) & 3u);
        const uint32_t gr = p_s + (uint32_t)lane;
        g.dq = P > 64u ? (gr >= P ? 1u : 0u) : (uint32_t)(((float)gr + 0.5f) * invP);
        g.pv = gr - g.dq * P;
        g.act = g.dq < q_end - q_s;
        g.o = g.act ? lane * SC + (int32_t)g.dq * G + (int32_t)adj : 0x7FFFFF00;
        return g;
    };
    auto issue = [&](uint32_t (&x)[UW + 1], uint32_t q_s, uint32_t p_s, const Geo &g) {
        uint32_t adj;
        const __amdgpu_buffer_rsrc_t rs = seg_rsrc_a(sg.base, g.B, len, adj);
        load_piece(rs, g.o, x);
    };
    bool cont = false;
    uint32_t creg = 0;
    // a step's piece CRC (raw, from 0), with the first pieces' initial register and the value carried in
    auto crc_step = [&](uint32_t (&x)[UW + 1], const Geo &g) -> uint32_t {
        if (!(KVR_PABLATE & 8)) piece_align(x, g.o);
        const bool first = g.act && g.pv == 0u;
        // (values of whole pieces, the benchmark shapes: the chains with no restart)
        uint32_t raw;
        if (KVR_PABLATE & 1) {   // (diagnostic: no CRC; the words only kept alive)
            raw = 0;
#pragma unroll
            for (int i = 0; i <= UW; ++i) raw ^= x[i];
        } else {
            raw = zr != 0u ? piece_raw(x, K, S, first, zr) : KVR_PCHAINS == 4 ? piece_raw4(x, K, S) : piece_raw(x, K, S, false, 0u);
        }
        raw ^= first ? IXr : 0u;
        if (cont) {   // lane 0 continues the value lane 63 carried out of the last step
            const uint32_t cx = kmul(creg, S.KQ2 + 128);
            raw ^= lane == 0 ? cx : 0u;
        }
        return raw;
    };
    // Before a step's CRC (its pieces are in flight): the records whose values it completes, [qa, qb)
    // (geometry only), join the group -- after a flush of the group if they would not fit, or of the
    // run's first records (`early`) -- and their header windows are loaded, ahead of the next step's
    // pieces (so a flush waits for windows, never for pieces just issued).  A stop (ustop) ends the loop after the step.
    uint32_t qdone = 0;   // records whose values are complete (their windows loaded, their CRCs in vcrc)
    // A step's windows land in wt (every lane issues the loads, those of other lanes read past the
    // resource: no exec mask, so the wait counts stay exact) and move into win at the next step, when
    // the next step's pieces have been issued behind them: a flush then waits for windows only.
    uint32_t wt[13], wtsh = 0;
    bool wpend = false;   // (per lane: wt holds this lane's record's window)
#pragma unroll
    for (int i = 0; i < 13; ++i) wt[i] = 0u;
    auto merge_windows = [&]() {
#if KVR_PWROW
        if (!KVR_PWDMA && wpend) {   // (the lanes whose records completed: their slots of the wave's row)
#pragma unroll
            for (int i = 0; i < PWIN; ++i) S.WROW[wv][i][lane] = wt[i];
        }
        (void)wtsh;
#else
#pragma unroll
        for (int i = 0; i < 13; ++i) win[i] = wpend ? wt[i] : win[i];
        wsh = wpend ? wtsh : wsh;
#endif
        wpend = false;
    };
    // (issued on every step, a step that completes nothing reading nothing: a conditional load would
    // leave the piece waits conservative)
    auto load_windows = [&](uint32_t qa, uint32_t qb) {
        const uint32_t qj = qg + (uint32_t)lane;
        wpend = qj >= qa && qj < qb;
        const int32_t wo = lane * (int32_t)L + (int32_t)gadj, wa = wpend && !(KVR_PABLATE & 32) ? (wo & ~3) : 0x7FFFFF00;
        wtsh = (uint32_t)wo & 3u;
        if (KVR_PWDMA) {
            // LDS DMA into the wave's row: M0 = the LDS destination, lane l's 16 B land at M0 + 16 l,
            // so only the lanes whose records completed run the loads.  The compiler does not count
            // these loads: its own piece waits only grow by them (loads retire in order), and the flush
            // waits for them itself (KVR_PWDMA_VMC before it reads the row).  M0 is saved and restored
            // around them (the kernel uses it nowhere else).
            if (wpend && !(KVR_PABLATE & 64)) {
                const uint32_t rb = __builtin_amdgcn_readfirstlane(
                    (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)&S.WROW[wv][0][0]);
                // (the flush reads bytes [0, 12 + ku) of a window, realigned: 32 B for keys up to 20 B, 48 B
                // up to 36; the row's other dwords are never read)
                uint32_t m0s;
                if (ku <= 20u) {
                    asm volatile(
                        "s_mov_b32 %[sv], m0\n\t"
                        "s_mov_b32 m0, %[rb]\n\t"
                        "s_nop 0\n\t"
                        "buffer_load_dwordx4 %[o0], %[rs], 0 offen lds\n\t"
                        "s_add_u32 m0, %[rb], 0x400\n\t"
                        "s_nop 0\n\t"
                        "buffer_load_dwordx4 %[o1], %[rs], 0 offen lds\n\t"
                        "s_mov_b32 m0, %[sv]"
                        : [sv] "=&s"(m0s)
                        : [o0] "v"(wa), [o1] "v"(wa + 16), [rb] "s"(rb), [rs] "s"(grs)
                        : "memory", "scc");
                } else {
                    asm volatile(
                        "s_mov_b32 %[sv], m0\n\t"
                        "s_mov_b32 m0, %[rb]\n\t"
                        "s_nop 0\n\t"
                        "buffer_load_dwordx4 %[o0], %[rs], 0 offen lds\n\t"
                        "s_add_u32 m0, %[rb], 0x400\n\t"
                        "s_nop 0\n\t"
                        "buffer_load_dwordx4 %[o1], %[rs], 0 offen lds\n\t"
                        "s_add_u32 m0, %[rb], 0x800\n\t"
                        "s_nop 0\n\t"
                        "buffer_load_dwordx4 %[o2], %[rs], 0 offen lds\n\t"
                        "s_mov_b32 m0, %[sv]"
                        : [sv] "=&s"(m0s)
                        : [o0] "v"(wa), [o1] "v"(wa + 16), [o2] "v"(wa + 32), [rb] "s"(rb), [rs] "s"(grs)
                        : "memory", "scc");
                }
            }
            return;
        }
        if (!(KVR_PABLATE & 64)) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const u32x4 v4 = __builtin_amdgcn_raw_buffer_load_b128(grs, wa + 16 * i, 0, 0);
                wt[4 * i] = v4.x; wt[4 * i + 1] = v4.y; wt[4 * i + 2] = v4.z; wt[4 * i + 3] = v4.w;
            }
            wt[12] = __builtin_amdgcn_raw_buffer_load_b32(grs, wa + 48, 0, 0);
        }
    };
    auto pre_step = [&](uint32_t q_s, const Geo &g, uint32_t &qa, uint32_t &qb, bool load_now = true) {
        merge_windows();
        KVR_PSTAMP(8);
        if (early && qdone > qg) {
            early = false;
            flush(qdone - qg);
        }
        const uint64_t cmk = __ballot(g.act && g.pv == P - 1u);
        qa = qb = 0;
        if (cmk) {
            qa = q_s + rl32(g.dq, (int)__builtin_ctzll(cmk));
            qb = q_s + rl32(g.dq, 63 - (int)__builtin_clzll(cmk)) + 1u;
            if (qb - qg > 64u && !ustop) flush(qa - qg);   // the group is full: its records (all before qa) first
        }
        KVR_PSTAMP(4);
        if (load_now) load_windows(qa, qb);
    };
    // the step's push, scan and value CRCs (records [qa, qb) take theirs into vcrc)
    auto finish_step = [&](uint32_t raw, uint32_t q_s, uint32_t p_s, const Geo &g, uint32_t qa, uint32_t qb) {
        const bool first = g.act && g.pv == 0u;
        const bool comp = g.act && g.pv == P - 1u;
        const uint32_t dl = P - 1u - g.pv, dr = 63u - (uint32_t)lane;
        const uint32_t dd = g.act ? (dl < dr ? dl : dr) : 0u;
        uint32_t v = raw;
        if (!(KVR_PABLATE & 2)) {
            const uint32_t pushed = kmul_col<KR_OFF_P, KR_PITCH>(dd ? raw : 0u, S, dd ? 4u * (dd - 1u) : 0u);
            v = seg_xscan(dd ? pushed : raw, first ? N32 : 0u);
        }
        cont = ((__ballot(g.act && !comp) >> 63) & 1ull) != 0ull;
        creg = rl32(v, 63);
        if (qb > qa) {
            const uint32_t qj = qg + (uint32_t)lane;
            const bool in = qj >= qa && qj < qb;
            const int32_t src = (int32_t)((qj - q_s) * P + (P - 1u) - p_s);
            const uint32_t cv = (uint32_t)__builtin_amdgcn_ds_bpermute(in ? 4 * src : 0, (int)~v);
            vcrc = in ? cv : vcrc;
            qdone = qb;
        }
    };
    // the steps: lane 0 at piece p0 of record q0; the next NB - 1 steps' pieces are in flight behind
    // the one being worked on (issued before its window loads and CRC), each in buffers of its own
    uint32_t q0 = 0, p0 = 0;
    Geo g0 = geo(q0, p0);
    auto next_qp = [&](uint32_t q, uint32_t p, uint32_t &qn, uint32_t &pn) {
        qn = q + adv_q;
        pn = p + adv_p;
        if (pn >= P) { pn -= P; ++qn; }
    };
    auto geo_or_none = [&](uint32_t q, uint32_t p) -> Geo {   // (a step past the run reads nothing)
        Geo g = geo(q, p);
        if (!(q < q_end)) { g.act = false; g.o = 0x7FFFFF00; }
        return g;
    };
    // The 16 waves of a CU share its issue slots oldest first: left alone, the oldest wave of each
    // SIMD finishes its stripe in 55 % of the time of the youngest, and the CU's last quarter runs on
    // 4 waves.  A wave ahead of the mean progress (records done, 1/4096 of its PSPW runs) drops its
    // priority, one behind raises it, so the workgroup's stripes end together.
    const uint64_t pscale = (4096ull << 32) / ((uint64_t)q_end * PSPW);
    const uint32_t pbase = j * (4096u / PSPW);
    uint32_t pown = 0;
    if (KVR_PBAL && lane == 0) atomicAdd(&bal[1], 1u);
    uint32_t bstep = 0;   // (the balance runs every KVR_PBAL_EVERY steps)
    auto balance = [&](uint32_t q_now) {
        const uint32_t pn = pbase + (uint32_t)(((uint64_t)q_now * pscale) >> 32);
        uint32_t sum = 0, cnt = 1;
        if (lane == 0) {
            sum = atomicAdd(&bal[0], pn - pown) + (pn - pown);
            cnt = bal[1];
        }
        pown = pn;
        sum = uni32(sum);
        cnt = uni32(cnt);
        const int32_t d = (int32_t)(pn * cnt - sum), dl = (int32_t)(KVR_PBAL_D * cnt);
        if (d < -dl) __builtin_amdgcn_s_setprio(3);
        else if (d < 0) __builtin_amdgcn_s_setprio(2);
        else if (d < dl) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    };
    KVR_PSTAMP(0);
    if constexpr (NB == 1) {
        // one piece buffer: the next step's pieces are loaded as soon as the CRC has read this step's
        issue(w, q0, p0, g0);
#pragma unroll 1
        for (;;) {
            uint32_t qa, qb;
            pre_step(q0, g0, qa, qb);   // (a stop found here ends the loop after this step: no exit between
                                        // the window loads and the next pieces, so the waits stay exact)
            KVR_PSTAMP(9);
            const uint32_t raw = crc_step(w, g0);
            KVR_PSTAMP(1);
            KVR_PCOUNT(6);
            uint32_t q1, p1;
            next_qp(q0, p0, q1, p1);
            const bool h1 = q1 < q_end;
            Geo g1 = geo_or_none(q1, p1);
            issue(w, q1, p1, g1);   // (issued on every path, the last step's reading nothing: exact wait counts)
            KVR_PSTAMP(2);
            finish_step(raw, q0, p0, g0, qa, qb);
            if (KVR_PBAL && (++bstep & (KVR_PBAL_EVERY - 1u)) == 0u) balance(q1 < q_end ? q1 : q_end);
            KVR_PSTAMP(3);
            if (!h1 || ustop) break;
            q0 = q1; p0 = p1; g0 = g1;
        }
    } else {
        // NB buffers, a ring: step s + NB - 1 is issued into the buffer step s - 1 freed, before step
        // s's window loads and CRC (every load unconditional, a step past the run reading nothing, so
        // the waits stay exact: the CRC waits for its own pieces only).  A step in flight is only its
        // (q, p); its geometry is computed again where it is worked on (registers for the buffers).
        uint32_t wb[UW + 1], wc[UW + 1];
        uint32_t q1, p1, q2 = 0, p2 = 0;
        next_qp(q0, p0, q1, p1);
        issue(w, q0, p0, g0);
        if constexpr (NB == 3) {
            issue(wb, q1, p1, geo_or_none(q1, p1));
            next_qp(q1, p1, q2, p2);
        }
        // the step in cur; the newest in flight goes into nx
        // (the window loads and a flush come first: a flush holds many registers, and the buffer the
        // next pieces go into is free until they are issued)
        auto body = [&](uint32_t (&cur)[UW + 1], uint32_t (&nx)[UW + 1]) -> bool {
            const bool h1 = q1 < q_end;
            uint32_t qa, qb;
            pre_step(q0, g0, qa, qb, KVR_PWEARLY != 0 || (KVR_PWDMA != 0 && !KVR_PWDMA_AFTER));
            KVR_PSTAMP(9);
            if constexpr (NB == 3) issue(nx, q2, p2, geo_or_none(q2, p2));
            else issue(nx, q1, p1, geo_or_none(q1, p1));
            if (KVR_PWDMA && KVR_PWDMA_AFTER) load_windows(qa, qb);
            KVR_PSTAMP(2);
            const uint32_t raw = crc_step(cur, g0);
            KVR_PSTAMP(1);
            KVR_PCOUNT(6);
            // the windows of the records this step completes, behind the next step's pieces (their
            // registers are not held across the CRC); merged at the next step, whose CRC waits for its
            // pieces issued before them anyway
            if (!KVR_PWEARLY && !KVR_PWDMA) load_windows(qa, qb);
            finish_step(raw, q0, p0, g0, qa, qb);
            if (KVR_PBAL && (++bstep & (KVR_PBAL_EVERY - 1u)) == 0u) balance(h1 ? q1 : q_end);
            KVR_PSTAMP(3);
            if (!h1 || ustop) return true;
            q0 = q1; p0 = p1;
            if constexpr (NB == 3) {
                q1 = q2; p1 = p2;
                next_qp(q1, p1, q2, p2);
            } else {
                next_qp(q0, p0, q1, p1);
            }
            g0 = geo(q0, p0);   // (q0 < q_end here)
            return false;
        };
#pragma unroll 1
        for (;;) {
            if constexpr (NB == 3) {
                if (body(w, wc)) break;
                if (body(wb, w)) break;
                if (body(wc, wb)) break;
            } else {
                if (body(w, wb)) break;
                if (body(wb, w)) break;
            }
        }
    }
    if (KVR_PBAL) {   // out of the mean
        if (lane == 0) { atomicSub(&bal[0], pown); atomicSub(&bal[1], 1u); }
        __builtin_amdgcn_s_setprio(0);
    }
    merge_windows();
    if (!ustop && qg < qdone) flush(qdone - qg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (a prefetched step the stop left unused)
    if (!ustop && qg != q_end) ustop = true;   // (defensive: every record of the stripe completes)
    if (KVR_PRUNFORM && prun && lane == 0 && qg) {   // (the first chunk is full before another is claimed)
        const uint32_t cmx_r = pool_chunk > TILE_RECS ? pool_chunk : TILE_RECS;
        prun[si] = PieceRun{Pe, L, run_first, qg < cmx_r ? qg : cmx_r, ku, vu, sd.seg};
    }
    if (!ustop) {
        close_tiles(sd.t_end, seg_n);
        total += qg;
        if (lane == 0) atomicAdd(&ctr->piece_done, 1u);   // (the host's k_piece-or-not heuristic)
        finish(Pe + (uint64_t)q_end * L);
        KVR_PSTAMP(5);
        KVR_PFLUSH();
        return;
    }
    // hand back at record qg: its tile's records emitted here are `ah`, the last slots claimed
    const uint32_t k_res = tile_of(Pe + (uint64_t)qg * L);
    const int64_t lt = (int64_t)k_res * TILE - d0;   // the resumed tile's start
    const uint32_t qt = lt <= (int64_t)Pe ? 0u : (uint32_t)(((uint64_t)lt - Pe + L - 1u) / L);
    const uint32_t ah = qg - qt;
    close_tiles(k_res, seg_n - (seg_tile < k_res ? ah : seg_n));
    total += qg - ah;
    hand_back(Pe + (uint64_t)qg * L, k_res, ah, L);
}


__global__ __launch_bounds__(PNT) void k_piece(const SegDesc *__restrict__ segs, const StripeDesc *__restrict__ stripes,
                                               uint32_t n_stripes, StripeRes *__restrict__ sres,
                                               TileRes *__restrict__ tres, kvr_tuple *__restrict__ pool,
                                               uint64_t pool_cap, Counters *ctr, Tables tb, uint32_t pool_chunk,
                                               uint4 *__restrict__ kpool, uint32_t *__restrict__ scnt,
                                               PieceHand *__restrict__ hand, uint2 *__restrict__ pcrc,
                                               PieceRun *__restrict__ prun) {
    __shared__ SmemP S;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    stage_tables_p<PNT>(S, tb, tid);
    if (tid == 0) { S.BAL[0] = 0u; S.BAL[1] = 0u; }
    __syncthreads();
    Crc K;
    crc_init(K, S.C2, (uint32_t)lane);
    const uint32_t s0 = blockIdx.x * WPB + (uint32_t)__builtin_amdgcn_readfirstlane(wv) * PSPW;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)PSPW; ++j) {
        if (s0 + j >= n_stripes) return;
        piece_stripe<PNB>(s0 + j, j, S, K, lane, __builtin_amdgcn_readfirstlane(wv), segs, stripes, sres, tres, pool,
                          pool_cap, ctr, pool_chunk, kpool, scnt, hand, pcrc, prun);
    }
}

}  // namespace kvr
