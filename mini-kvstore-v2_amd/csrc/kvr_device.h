/*
 * kvr_device.h — device-side building blocks of the replay engine (gfx950 / CDNA4).
 *
 * Geometry:
 *   - A WAVE owns one STRIPE: a run of consecutive TILEs of one segment, walked in order, so the
 *     record chain and the CRC register of a value that spans tiles are handed from tile to
 *     tile; only the stripe's first entry is speculated (verified by k_link).
 *   - A TILE is 8 KiB; lane l holds the 128-B UNIT [128 l, 128 l + 128) in registers, prefetched
 *     one tile ahead.  The tile never goes to LDS: the framing reads headers out of the
 *     registers (readlane), records read their keys through a range-checked buffer resource.
 *   - CRC-32 (reflected 0xEDB88320, crc32fast semantics, src/volume/storage.rs:27) runs on
 *     lane-replicated slice-by-4 byte tables in LDS; register states move across units with
 *     the constants x^(8*128*d) (nibble tables), never with a variable GF(2) multiply.
 */
#ifndef KVR_DEVICE_H
#define KVR_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/kvreplay.h"

namespace kvr {

constexpr int      TILE  = 8192;           // bytes per tile (one wave: 64 lanes x 128-B units)
constexpr int      SC    = 128;            // unit: the CRC unit of one lane
constexpr int      SMALL = 64;             // values <= SMALL: CRC'd whole by their record's lane
constexpr int      NQ    = SC / 4 + 1;     // X(4q), q <= SC / 4
constexpr int      KSET_Q = 8;             // kmul sets: X(SC*2^j) j<8, then X(4q) q<=SC/4,
constexpr int      KSET_R = 8 + NQ;        //   then X(SC(k+1)) k<64 (unit-distance multipliers)
constexpr int      KMUL_SETS = 8 + NQ + 64;
constexpr int      NIX   = SC + 1;         // 0xFFFFFFFF * X(j), j <= SC
constexpr uint64_t NONE  = ~0ull;          // "no position"
constexpr uint64_t ERRP  = ~0ull - 1;      // chain ended in a framing error
constexpr uint32_t POLY  = 0xEDB88320u;
constexpr uint32_t GF_ONE = 0x80000000u;   // x^0 in the reflected representation

struct SegDesc {          // one caller segment
    const uint8_t *base;  // device pointer to byte 0
    uint64_t len;
    uint32_t d0;          // base mod 16: tiles are aligned to 16 B in the device address space
    uint32_t tile0;       // global index of the segment's first tile
    uint32_t n_tiles;
    uint32_t stripe0;     // first stripe of the segment
    uint32_t n_stripes;
    uint32_t pad;
};

struct StripeDesc {       // tiles [t_begin, t_end) of segment seg
    uint32_t seg, t_begin, t_end;
    uint32_t pad;         // 1: the segment's first stripe (k_link)
};

struct StripeRes {
    uint64_t entry;       // first record start of the stripe (NONE: no record starts in it)
    uint64_t exit;        // first record start at/after the stripe end (ERRP on error)
    uint64_t err_pos;
    uint64_t err_aux;
    uint32_t err_kind;
    uint32_t count;
    uint32_t forced;      // entry was imposed by k_link (re-walk pass)
    uint32_t owned;       // k_link, before a re-walk pass: bit 0 listed for re-walk, bit 1 inconsistent
                          // (k_replay's re-walk sets 1 on the stripes it walks)
    uint64_t pool_run;    // the stripe's tuples are pool[pool_run, + count) in order (one chunk), or NONE
    uint64_t pad;
};

struct TileRes {          // a tile's tuples in the pool: [pool_off, + count1) then [pool_off2, + count - count1)
    uint64_t pool_off;
    uint64_t pool_off2;
    uint32_t count;
    uint32_t count1;
};

struct RedoEnt { uint32_t stripe; uint32_t pad; uint64_t entry; };

struct PieceHand {        // k_piece -> k_replay, one per stripe: where the tile loop resumes
    uint64_t entry;       // its chain position (NONE: the entry search goes on from tile k)
    uint64_t stripe_entry;   // the stripe's first record start (NONE: not found yet)
    uint32_t k;           // the tile it resumes at
    uint32_t ahead;       // records starting in tile k that k_piece emitted (the wave's last claimed slots)
    uint32_t stride;      // the last record length (the stride round's prediction; 0: none)
    uint32_t total;       // records of the tiles before k
    uint32_t chunk_base, chunk_left;   // the wave's pool chunk
    uint32_t run_first, run_contig;    // the stripe's tuples so far: one run of the pool from run_first
    uint32_t done;        // 1: k_piece finished the stripe (StripeRes, scnt and every TileRes written)
    uint32_t pad;
};
static_assert(sizeof(PieceHand) == 56, "PieceHand layout");

// k_piece -> k_compact_s, one per stripe: the records of the stripe's run that k_piece left in the pool
// in run form.  Pool slots [first, first + n) hold record q = slot - first of the run, a SET at
// Pe + q L with key length ku and value length vu in segment seg; its value CRC and key tag are in
// pcrc[slot] (8 B), no 32-B tuple is written for it (k_compact_s builds the tuple)
struct PieceRun {
    uint64_t Pe;
    uint32_t L, first, n, ku, vu, seg;
};
static_assert(sizeof(PieceRun) == 32, "PieceRun layout");

struct LinkResult {
    int32_t  status;      // 0 ok, 1 corrupted, 3 unresolved (re-walk needed)
    uint32_t n_redo;
    uint32_t err_kind;
    uint32_t err_seg;
    uint64_t err_pos;
    uint64_t err_aux;
    uint32_t first_problem_seg;
    uint32_t passes;
};

struct Counters {         // device scratch, reset per call
    unsigned long long pool_cursor;
    unsigned long long total_tuples;
    unsigned long long crc_fail;
    uint32_t overflow;
    uint32_t unlinked;    // host mirror: k_compact_s (linked mode) found a stripe it cannot link alone
    uint32_t piece_done;  // stripes k_piece ran to their end (host mirror: copied by the gather / k_link)
    uint32_t pad;
};
static_assert(sizeof(Counters) + 64 <= 128, "Counters in the link + counters block");

constexpr uint32_t LC_BLOCK = 128;   // one link + counters block (LinkResult at 0, Counters at 64)

struct Tables {           // read-only tables in global memory (copied to LDS per workgroup)
    const uint32_t *crc8;   // [16][256] slice-by-16 byte tables (k_replay replicates the first 2)
    const uint32_t *kmul;   // [KMUL_SETS][8][16]: (n << 4i) * K_t (kvr_api.hip build_tables)
    const uint32_t *initx;  // [NIX]: 0xFFFFFFFF * x^(8 j)
};

// ---------------------------------------------------------------------------------------
// GF(2)[x] / P arithmetic in the reflected representation (bit 31 = x^0), as zlib's
// multmodp.  X(n) = x^(8n) mod P is "append n zero bytes" to a raw CRC register.
// ---------------------------------------------------------------------------------------
__host__ __device__ inline uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t m = (uint32_t)((int32_t)(a << i) >> 31);
        p ^= b & m;
        b = (b >> 1) ^ (POLY & (0u - (b & 1u)));
    }
    return p;
}

}  // namespace kvr
#endif
