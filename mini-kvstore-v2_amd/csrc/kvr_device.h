/*
 * kvr_device.h — device-side building blocks of the replay engine (gfx950 / CDNA4).
 *
 * Geometry:
 *   - A workgroup (NT = 256 threads = 4 waves) owns one STRIPE: a run of consecutive TILEs of
 *     one segment, walked in order, so the record chain is exact inside a stripe and only the
 *     stripe's first entry is speculated (verified by k_link).
 *   - A TILE (16 KiB) is streamed HBM -> LDS by LDS-DMA, one tile ahead of the one being
 *     processed.  Its framing is walked in parallel: each thread speculates a chain through its
 *     64-B SUB-CHUNK; wave 0 stitches the 256 sub-chains by pointer jumping.
 *   - CRC-32 (reflected 0xEDB88320, crc32fast semantics, src/volume/storage.rs:27) runs on
 *     conflict-free nibble tables (32 x 16 entries: every ds_read_b32 of a wave hits one
 *     16-entry table = 16 distinct banks).  Each sub-chunk is also a CRC UNIT: its share of a
 *     long value is CRC'd independently and shifted into place with one GF(2) multiply;
 *     shares are XOR-combined (order-free), so tiles need no ordered hand-over of CRC state.
 */
#ifndef KVR_DEVICE_H
#define KVR_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/kvreplay.h"

namespace kvr {

constexpr int      NT    = 256;            // threads per workgroup
constexpr int      TILE  = 16384;          // bytes staged per tile
constexpr int      SC    = TILE / NT;      // 64: framing sub-chunk = CRC unit per thread
constexpr int      SMALL = 64;             // values <= SMALL inside the tile: CRC'd by their walker
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

struct Tables {           // read-only tables in global memory (L1/L2 resident)
    const uint32_t *crc8;   // [16][256] byte tables (generator manifest)
    const uint32_t *nib;    // [16 distances][2 nibbles][16] nibble tables
    const uint32_t *pw16;   // X(16 k), k = 0 .. TILE/16
    const uint32_t *pw1;    // X(i), i = 0 .. 16
    const uint32_t *xw;     // [8][16]: X(j * 16^i), square-free exponentiation windows
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

// X(d) for any d < 2^32 bytes from the nibble windows X(j * 16^i)
__device__ inline uint32_t gf_xpow(uint64_t d, const uint32_t *__restrict__ xw) {
    uint32_t r = GF_ONE;
    for (int i = 0; i < 8 && d; ++i, d >>= 4) {
        const uint32_t n = (uint32_t)(d & 15u);
        if (n) r = (r == GF_ONE) ? xw[i * 16 + n] : gf_mul(r, xw[i * 16 + n]);
    }
    return r;
}

// ---------------------------------------------------------------------------------------
// Nibble-table CRC.  nt[(d * 2 + h) * 16 + n] = T_d[n << 4h]: the contribution of a byte whose
// nibble h is n, at distance d bytes from the end of a 16-byte block.
// ---------------------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ uint32_t nib_word(uint32_t w, const uint32_t *__restrict__ nt) {
    const uint32_t lo4 = (w << 2) & 0x3C3C3C3Cu, hi4 = (w >> 2) & 0x3C3C3C3Cu;   // nibble * 4
    const char *b = reinterpret_cast<const char *>(nt);
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t al = (lo4 >> (8 * j)) & 0xFFu, ah = (hi4 >> (8 * j)) & 0xFFu;
        r ^= *reinterpret_cast<const uint32_t *>(b + ((D - j) * 2 + 0) * 64 + al) ^
             *reinterpret_cast<const uint32_t *>(b + ((D - j) * 2 + 1) * 64 + ah);
    }
    return r;
}

// one slice-by-16 step: register c, 16 message bytes d (little-endian dwords)
__device__ __forceinline__ uint32_t nslice16(uint32_t c, uint4 d, const uint32_t *__restrict__ nt) {
    return nib_word<15>(d.x ^ c, nt) ^ nib_word<11>(d.y, nt) ^ nib_word<7>(d.z, nt) ^ nib_word<3>(d.w, nt);
}

__device__ __forceinline__ uint32_t nbyte(uint32_t c, uint32_t b, const uint32_t *__restrict__ nt) {
    const uint32_t x = (c ^ b) & 0xFFu;
    return (c >> 8) ^ nt[x & 15u] ^ nt[16 + (x >> 4)];
}

// ---------------------------------------------------------------------------------------
// A view of one segment with one tile resident in LDS.  Positions are segment offsets;
// LDS offset 0 holds segment position `lo` (lo may be negative for the first tile).
// rd8(p) needs p < len; rd32(p) needs p + 4 <= len.  Bytes outside the tile come from HBM.
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
        if (off >= 0 && off < TILE) return lds[off];
        return seg[p];
    }
    __device__ __forceinline__ uint32_t rd32(uint64_t p) const {
        const int64_t off = (int64_t)p - lo;
        if (off >= 0 && off <= TILE - 4) return lds_u32(off);
        return (uint32_t)seg[p] | ((uint32_t)seg[p + 1] << 8) | ((uint32_t)seg[p + 2] << 16) |
               ((uint32_t)seg[p + 3] << 24);
    }
    __device__ __forceinline__ bool in_lds(uint64_t p, uint64_t n) const {
        const int64_t off = (int64_t)p - lo;
        return off >= 0 && off + (int64_t)n <= TILE;
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

// CRC register update over [p, p+n): LDS nibble slice-by-16 when resident, bytes otherwise.
__device__ inline uint32_t crc_range(const TileView &tv, uint32_t c, uint64_t p, uint64_t n,
                                     const uint32_t *__restrict__ nt) {
    if (tv.in_lds(p, n)) {
        int64_t off = (int64_t)p - tv.lo;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(tv.lds);
        while (n >= 16) {
            const uint32_t q = (uint32_t)off >> 2, sh = (uint32_t)off & 3u;
            uint4 d;
            if (sh == 0) {
                d = make_uint4(w[q], w[q + 1], w[q + 2], w[q + 3]);
            } else {
                const uint32_t a0 = w[q], a1 = w[q + 1], a2 = w[q + 2], a3 = w[q + 3], a4 = w[q + 4];
                d = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sh), __builtin_amdgcn_alignbyte(a2, a1, sh),
                               __builtin_amdgcn_alignbyte(a3, a2, sh), __builtin_amdgcn_alignbyte(a4, a3, sh));
            }
            c = nslice16(c, d, nt);
            off += 16;
            n -= 16;
        }
        while (n > 0) { c = nbyte(c, tv.lds[off], nt); ++off; --n; }
        return c;
    }
    for (uint64_t i = 0; i < n; ++i) c = nbyte(c, tv.rd8(p + i), nt);
    return c;
}

}  // namespace kvr
#endif
