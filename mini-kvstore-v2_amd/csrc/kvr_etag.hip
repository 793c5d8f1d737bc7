/*
 * kvr_etag.hip — batch ETag compute / verify: CRC-32/ISO-HDLC of many
 * blobs in one launch, the value BlobStorage::put renders as its ETag
 * (src/volume/storage.rs:27: format!("{:08x}", crc32fast::hash(data))).
 *
 * A blob is cut into 4-KiB chunks; one wave per chunk, one 64-B unit per lane:
 *   lane register  u_l = CRC register over the lane's bytes (slice-by-4 from LDS), starting at
 *                  0xFFFFFFFF for lane 0 of a blob's first chunk and at 0 everywhere else
 *   chunk register r_j = XOR_l u_l * x^(8 * bytes after lane l in the chunk)   (wave XOR reduce)
 * and one wave per blob then joins its chunks (k_etag_join):
 *   register R = (XOR_{k} r_{nch-2-k} * x^(8 k CH)) * x^(8 lastlen)  ^  r_{nch-1}
 *   crc        = R ^ 0xFFFFFFFF
 * which is the byte-serial CRC by linearity of the register update over GF(2).
 * Byte traffic: every blob byte is read once (HBM-bound); 4 B per chunk and 4 B per blob written.
 */
#pragma once

namespace kvr {

constexpr uint32_t ETAG_CH = 4096;           // chunk bytes (64 lanes x 64 B)
constexpr uint32_t ETAG_WPB = 4;             // waves per workgroup
constexpr uint32_t ETAG_NX = ETAG_CH + 1 + 64 + 1;   // XT[0..CH], XC[0..63], X(64 CH)

// chunk -> blob map: blob v owns chunks [cpre[v], cpre[v+1])
__global__ void k_etag_map(const uint64_t *__restrict__ cpre, uint64_t n, uint32_t *__restrict__ chunk_blob) {
    for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x)
        for (uint64_t c = cpre[v]; c < cpre[v + 1]; ++c) chunk_blob[c] = (uint32_t)v;
}

__device__ inline uint32_t crc_word4(const uint32_t *T, uint32_t c, uint32_t w) {
    c ^= w;
    return T[768 + (c & 255u)] ^ T[512 + ((c >> 8) & 255u)] ^ T[256 + ((c >> 16) & 255u)] ^ T[c >> 24];
}

__device__ inline uint32_t crc_byte(const uint32_t *T, uint32_t c, uint32_t b) {
    return (c >> 8) ^ T[(c ^ b) & 255u];
}

__global__ __launch_bounds__(64 * ETAG_WPB) void k_etag_chunk(const uint8_t *__restrict__ data, uint64_t data_len,
                                                             const uint64_t *__restrict__ offs,
                                                             const uint64_t *__restrict__ lens,
                                                             const uint64_t *__restrict__ cpre,
                                                             const uint32_t *__restrict__ chunk_blob, uint64_t n_chunks,
                                                             const uint32_t *__restrict__ crc_tab,
                                                             const uint32_t *__restrict__ xt,
                                                             uint32_t *__restrict__ creg) {
    __shared__ uint32_t T[1024];   // slice-by-4: T[t * 256 + b] = byte b pushed through t zero bytes
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) T[i] = crc_tab[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t c = blockIdx.x * (uint64_t)ETAG_WPB + (threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const uint32_t v = chunk_blob[c];
    const uint64_t j = c - cpre[v];
    const uint64_t len = lens[v];
    const uint64_t start = offs[v] + j * ETAG_CH;
    const uint32_t clen = (uint32_t)min<uint64_t>(ETAG_CH, len - j * ETAG_CH);
    const uint32_t u0 = lane * 64u;
    uint32_t reg = (j == 0 && lane == 0) ? 0xFFFFFFFFu : 0u;
    uint32_t after = 0;
    if (u0 < clen) {
        const uint32_t ul = min(64u, clen - u0);
        after = clen - (u0 + ul);
        const uint8_t *p = data + start + u0;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        if (ul == 64 && (a & 15u) == 0) {           // aligned full unit: 4 x 16-B loads
            const uint4 *q = reinterpret_cast<const uint4 *>(p);
            uint4 w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] = q[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                reg = crc_word4(T, reg, w[i].x);
                reg = crc_word4(T, reg, w[i].y);
                reg = crc_word4(T, reg, w[i].z);
                reg = crc_word4(T, reg, w[i].w);
            }
        } else {
            // unaligned or partial unit: dwords from the aligned-down window while it stays inside
            // the buffer, then bytes
            const uint32_t mis = (uint32_t)(a & 3u);
            const uint64_t rel = (uint64_t)(p - data);
            uint32_t k = 0;
            if (mis == 0) {
                for (; k + 4 <= ul; k += 4) reg = crc_word4(T, reg, *reinterpret_cast<const uint32_t *>(p + k));
            } else if (rel - mis + ((ul + mis + 3u) & ~3u) <= data_len && rel >= mis) {
                const uint32_t *q = reinterpret_cast<const uint32_t *>(p - mis);
                uint32_t lo = q[0];
                for (uint32_t i = 1; k + 4 <= ul; ++i, k += 4) {
                    const uint32_t hi = q[i];
                    reg = crc_word4(T, reg, __builtin_amdgcn_alignbyte(hi, lo, mis));
                    lo = hi;
                }
            }
            for (; k < ul; ++k) reg = crc_byte(T, reg, p[k]);
        }
        if (after) reg = gf_mul(reg, xt[after]);
    }
    // wave XOR reduction
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) reg ^= __shfl_xor(reg, o, 64);
    if (lane == 0) creg[c] = reg;
}

// one wave per blob: join the chunk registers, finish the CRC, verify against expected
__global__ __launch_bounds__(64 * ETAG_WPB) void k_etag_join(const uint64_t *__restrict__ lens,
                                                            const uint64_t *__restrict__ cpre, uint64_t n,
                                                            const uint32_t *__restrict__ creg,
                                                            const uint32_t *__restrict__ xt,
                                                            const uint32_t *__restrict__ expected,
                                                            uint32_t *__restrict__ out,
                                                            unsigned long long *__restrict__ n_fail) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t v = blockIdx.x * (uint64_t)ETAG_WPB + (threadIdx.x >> 6);
    if (v >= n) return;
    const uint64_t c0 = cpre[v], nch = cpre[v + 1] - c0;
    uint32_t crc = 0;
    if (nch) {
        const uint32_t *xc = xt + ETAG_CH + 1;        // XC[l] = x^(8 l CH)
        const uint32_t x64 = xt[ETAG_CH + 1 + 64];    // x^(8 * 64 CH)
        uint32_t S = 0, M = GF_ONE;
        for (uint64_t g0 = 0; g0 + 1 < nch; g0 += 64) {
            const uint64_t k = g0 + lane;
            uint32_t t = 0;
            if (k + 1 < nch) t = gf_mul(creg[c0 + (nch - 2 - k)], xc[lane]);
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) t ^= __shfl_xor(t, o, 64);
            S ^= gf_mul(t, M);
            M = gf_mul(M, x64);
        }
        const uint32_t lastlen = (uint32_t)(lens[v] - (nch - 1) * ETAG_CH);
        crc = (gf_mul(S, xt[lastlen]) ^ creg[c0 + nch - 1]) ^ 0xFFFFFFFFu;
    }
    if (lane == 0) {
        out[v] = crc;
        if (expected && expected[v] != crc) atomicAdd(n_fail, 1ull);
    }
}

}  // namespace kvr
