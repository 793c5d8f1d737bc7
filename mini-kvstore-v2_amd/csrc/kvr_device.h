/*
 * kvr_device.h — device-side building blocks of the replay engine (gfx950 / CDNA4).
 *
 * Geometry:
 *   - A WAVE owns one STRIPE: a run of consecutive TILEs of one segment, walked in order, so the
 *     record chain and the CRC register of a value that spans tiles are handed from tile to
 *     tile; only the stripe's first entry is speculated (verified by k_link).
 *   - A TILE is 4 KiB; lane l holds the 64-B UNIT [64 l, 64 l + 64) in registers (prefetched one
 *     tile ahead) and copies it to the wave's LDS tile, behind which a HALO of the next 256 B
 *     arrives by LDS-DMA for headers and short fields that straddle the tile end.
 *   - CRC-32 (reflected 0xEDB88320, crc32fast semantics, src/volume/storage.rs:27) runs on
 *     lane-replicated slice-by-2 byte tables in LDS; register states move across units with
 *     the constants x^(8*64*d) (nibble tables), never with a variable GF(2) multiply.
 */
#ifndef KVR_DEVICE_H
#define KVR_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/kvreplay.h"

namespace kvr {

constexpr int      NT    = 256;            // threads per workgroup
constexpr int      TILE  = 4096;           // bytes per tile (one wave: 64 lanes x 64-B units)
constexpr int      SC    = 64;             // unit: framing sub-chunk = CRC unit per lane
constexpr int      SMALL = 64;             // values <= SMALL: CRC'd whole by their record's thread
constexpr int      HALO  = 256;            // bytes of the next tile staged behind each tile
constexpr int      KSET_Q = 8;             // kmul sets: X(64*2^j) j<8, then X(4q) q<=16,
constexpr int      KSET_R = 8 + 17;        //   then X(64(k+1)) k<32 (cross-row scan multipliers)
constexpr int      KMUL_SETS = 8 + 17 + 32;
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
    uint32_t seg, t_begin, t_end, pad;
};

struct StripeRes {
    uint64_t entry;       // first record start of the stripe (NONE: no record starts in it)
    uint64_t exit;        // first record start at/after the stripe end (ERRP on error)
    uint64_t err_pos;
    uint64_t err_aux;
    uint32_t err_kind;
    uint32_t count;
    uint32_t forced;      // entry was imposed by k_link (re-walk pass)
    uint32_t pad;
};

struct TileRes { uint64_t pool_off; uint32_t count; uint32_t pad; };

struct RedoEnt { uint32_t stripe; uint32_t pad; uint64_t entry; };

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
    uint32_t pad;
};

struct Tables {           // read-only tables in global memory (copied to LDS per workgroup)
    const uint32_t *crc8;   // [16][256] slice-by-16 byte tables (first 4 used by k_replay)
    const uint32_t *kmul;   // [KMUL_SETS][8][16]: (n << 4i) * K_t (kvr_api.hip build_tables)
    const uint32_t *initx;  // [65]: 0xFFFFFFFF * x^(8 j)
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

// ---------------------------------------------------------------------------------------
// A view of one segment with one tile (+ halo) resident in LDS.  Positions are segment
// offsets; LDS offset 0 holds segment position `lo` (lo may be negative for the first tile).
// rd8(p) needs p < len; rd32(p) needs p + 4 <= len.  Bytes outside tile + halo come from HBM.
// ---------------------------------------------------------------------------------------
struct TileView {
    const uint8_t *seg;
    const uint8_t *lds;
    uint64_t len;
    int64_t lo;

    __device__ __forceinline__ uint32_t lds_u32(int64_t off) const {   // unaligned LDS read
        const uint32_t *w = reinterpret_cast<const uint32_t *>(lds);
        const uint32_t q = (uint32_t)off >> 2, sh = (uint32_t)off & 3u;
        const uint32_t a = w[q];
        if (sh == 0) return a;
        const uint32_t b = w[q + 1];
        return __builtin_amdgcn_alignbyte(b, a, sh);
    }
    __device__ __forceinline__ uint32_t rd8(uint64_t p) const {
        const int64_t off = (int64_t)p - lo;
        if (off >= 0 && off < TILE + HALO) return lds[off];
        return seg[p];
    }
    __device__ __forceinline__ uint32_t rd32(uint64_t p) const {
        const int64_t off = (int64_t)p - lo;
        if (off >= 0 && off <= TILE + HALO - 4) return lds_u32(off);
        return (uint32_t)seg[p] | ((uint32_t)seg[p + 1] << 8) | ((uint32_t)seg[p + 2] << 16) |
               ((uint32_t)seg[p + 3] << 24);
    }
    __device__ __forceinline__ bool in_lds(uint64_t p, uint64_t n) const {
        const int64_t off = (int64_t)p - lo;
        return off >= 0 && off + (int64_t)n <= TILE + HALO;
    }
};

// End of the record at p (engine.rs framing, exact, HBM fallback), or ERRP if the framing is
// broken there: opcode outside {0,1} or a field running past the segment end.  Needs p < len.
__device__ inline uint64_t next_rec(const TileView &tv, uint64_t p) {
    const uint64_t n = tv.len;
    const uint32_t op = tv.rd8(p);
    if (op > 1u || n - p < 5) return ERRP;
    const uint64_t e = p + 5 + (uint64_t)tv.rd32(p + 1);
    if (e > n) return ERRP;
    if (op == 1u) return e;
    if (n - e < 4) return ERRP;
    const uint64_t e2 = e + 4 + (uint64_t)tv.rd32(e);
    return e2 > n ? ERRP : e2;
}

// ---------------------------------------------------------------------------------------
// UTF-8 validation with Rust's Utf8Error semantics (engine.rs:114, String::from_utf8).
// Returns true if valid, else *vu = valid_up_to and *el = error_len (0 = incomplete).
// ---------------------------------------------------------------------------------------
__device__ inline bool utf8_check(const TileView &tv, uint64_t p, uint64_t n, uint64_t *vu, uint32_t *el) {
    uint64_t i = 0;
#pragma unroll 1
    while (i < n) {
        if (n - i >= 4 && tv.in_lds(p + i, 4)) {          // ASCII fast path, 4 bytes at a time
            const uint32_t w4 = tv.lds_u32((int64_t)(p + i) - tv.lo);
            if ((w4 & 0x80808080u) == 0) { i += 4; continue; }
        }
        const uint32_t b = tv.rd8(p + i);
        if (b < 0x80u) { ++i; continue; }
        const uint64_t start = i;
        int width = 0;
        if (b >= 0xC2u && b <= 0xDFu) width = 2;
        else if (b >= 0xE0u && b <= 0xEFu) width = 3;
        else if (b >= 0xF0u && b <= 0xF4u) width = 4;
        *vu = start;
        if (width == 0) { *el = 1; return false; }
        if (++i >= n) { *el = 0; return false; }
        const uint32_t c1 = tv.rd8(p + i);
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
            if ((tv.rd8(p + i) & 0xC0u) != 0x80u) { *el = (uint32_t)k; return false; }
        }
        ++i;
    }
    return true;
}

}  // namespace kvr
#endif
