/*
 * kvr_etag.hip — batch ETag compute / verify: CRC-32/ISO-HDLC of many
 * blobs in one launch, the value BlobStorage::put renders as its ETag
 * (src/volume/storage.rs:27: format!("{:08x}", crc32fast::hash(data))).
 *
 * A blob is cut into 4-KiB chunks, one 64-B unit per lane; a persistent wave takes 4 chunks per
 * round and runs their CRC chains interleaved:
 *   lane register  u_l = CRC register over the lane's bytes (slice-by-4 from LDS), starting at
 *                  0xFFFFFFFF for lane 0 of a blob's first chunk and at 0 everywhere else
 *   chunk register r_j = XOR_l u_l * x^(8 * bytes after lane l in the chunk)   (wave XOR reduce;
 *                  the per-lane multiply by nibble tables in LDS for full chunks)
 * and one wave per blob then joins its chunks (k_etag_join):
 *   register R = (XOR_{k} r_{nch-2-k} * x^(8 k CH)) * x^(8 lastlen)  ^  r_{nch-1}
 *   crc        = R ^ 0xFFFFFFFF
 * which is the byte-serial CRC by linearity of the register update over GF(2).
 * Byte traffic: every blob byte is read once (HBM-bound); 4 B per chunk and 4 B per blob written.
 */
#pragma once

namespace kvr {

constexpr uint32_t ETAG_CH = 4096;           // chunk bytes (64 lanes x 64 B)
constexpr uint32_t ETAG_WPB = 16;            // waves per workgroup (96 KiB LDS: one per CU)
constexpr uint32_t ETAG_NC = 4;              // chunks per wave and round (interleaved CRC chains)
constexpr uint32_t ETAG_NX = ETAG_CH + 1 + 64 + 1;   // XT[0..CH], XC[0..63], X(64 CH); then KL
constexpr uint32_t ETAG_NKL = 64 * 128;             // KL[lane][i][n]: nibble tables of XT[CH - 64 (lane+1)]

#ifndef KVR_ETAG_DB
#define KVR_ETAG_DB 0   // 1: double-buffered rounds of ETAG_NC_DB chunks (the next round's loads in flight)
#endif
constexpr int ETAG_NC_DB = 2;

// chunk descriptors: blob v owns chunks [cpre[v], cpre[v+1]); chunk c = the j-th of its blob is
// data[start, start + clen) with start = offs[v] + j CH, packed as start | (clen - 1) << 48 |
// (j == 0) << 63 (one load per chunk in k_etag_chunk).  One thread per chunk, v by binary search.
__global__ void k_etag_map(const uint64_t *__restrict__ cpre, uint64_t n, const uint64_t *__restrict__ offs,
                           const uint64_t *__restrict__ lens, uint64_t nch, uint64_t *__restrict__ cdesc) {
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nch; c += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = n - 1;   // the last blob with cpre[v] <= c (empty blobs own no chunk)
        while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) >> 1;
            if (cpre[mid] <= c) lo = mid; else hi = mid - 1;
        }
        const uint64_t j = c - cpre[lo];
        const uint64_t clen = min<uint64_t>(ETAG_CH, lens[lo] - j * ETAG_CH);
        cdesc[c] = (offs[lo] + j * ETAG_CH) | ((clen - 1) << 48) | ((j == 0 ? 1ull : 0ull) << 63);
    }
}
__device__ __forceinline__ void etag_desc(uint64_t d, uint64_t &start, uint32_t &clen, bool &first) {
    start = d & ((1ull << 48) - 1);
    clen = (uint32_t)((d >> 48) & 0x7FFFu) + 1u;
    first = (d >> 63) != 0;
}

// The byte tables are k_replay's (kvr_replay_kernel.hip, Crc): slice-by-4 replicated per LDS bank
// group with the rotation trick, so no lookup of a wave conflicts; crc4 / crc1 are k_replay's steps.
__device__ inline uint32_t crc_word4(const Crc &K, uint32_t c, uint32_t w) { return crc4(c, w, K); }

__device__ inline uint32_t crc_byte(const Crc &K, uint32_t c, uint32_t b) { return crc1(c, b, K); }

struct __align__(16) EtagSmem {
    uint32_t C2[256 * 64];   // byte tables (64 KiB, k_replay's Crc layout)
    uint32_t KL[64 * 128];   // [16 i + n][lane]: (n << 4 i) * x^(8 (4096 - 64 (lane + 1)))
};
static_assert(offsetof(EtagSmem, KL) == 65536, "kmul_lane's 64-KiB bit");
// v times this lane's constant: entry (i, n, lane) at KL + (16 i + n) 256 + 4 lane, the address one
// v_perm_b32 (byte 0 = 4 lane, byte 1 = i << 4 | n from a nibble plane, byte 2 = the 64-KiB bit)
__device__ __forceinline__ uint32_t kmul_lane(uint32_t v, const EtagSmem &S, uint32_t lane) {
    const uint32_t L4k = 4u * lane | 0x10000u;
    uint32_t pl[2] = {(v & 0x0F0F0F0Fu) | 0x60402000u, ((v >> 4) & 0x0F0F0F0Fu) | 0x70503010u};
    asm("" : "+v"(pl[0]), "+v"(pl[1]));
    const uint8_t *tb = reinterpret_cast<const uint8_t *>(&S);
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        t[i] = *reinterpret_cast<const uint32_t *>(
            tb + __builtin_amdgcn_perm(pl[i & 1], L4k, 0x0C020000u | ((4u + (uint32_t)(i >> 1)) << 8)));
    asm("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]));
    return (t[0] ^ t[1] ^ t[2]) ^ (t[3] ^ t[4] ^ t[5]) ^ (t[6] ^ t[7]);
}

// One chunk through the general path: any alignment, partial units, bounds-checked loads.
__device__ inline uint32_t etag_unit_general(const Crc &T, const uint8_t *data, uint64_t data_len, uint64_t start,
                                             uint32_t clen, uint32_t lane, uint32_t reg, const uint32_t *xt) {
    const uint32_t u0 = lane * 64u;
    if (u0 >= clen) return 0u;
    const uint32_t ul = min(64u, clen - u0);
    const uint32_t after = clen - (u0 + ul);
    const uint8_t *p = data + start + u0;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
    const uint64_t rel = start + u0;
    uint32_t k = 0;
    if (mis == 0) {
        for (; k + 4 <= ul; k += 4) reg = crc_word4(T, reg, *reinterpret_cast<const uint32_t *>(p + k));
    } else if (rel >= mis && rel - mis + ((ul + mis + 3u) & ~3u) <= data_len) {
        // dwords from the aligned-down window while it stays inside the buffer
        const uint32_t *q = reinterpret_cast<const uint32_t *>(p - mis);
        uint32_t w0 = q[0];
        for (uint32_t i = 1; k + 4 <= ul; ++i, k += 4) {
            const uint32_t hi = q[i];
            reg = crc_word4(T, reg, __builtin_amdgcn_alignbyte(hi, w0, mis));
            w0 = hi;
        }
    }
    for (; k < ul; ++k) reg = crc_byte(T, reg, p[k]);
    return after ? gf_mul(reg, xt[after]) : reg;
}

// Persistent: as many workgroups as are resident (occupancy query); each wave takes ETAG_NC chunks per round and runs
// their CRC chains interleaved (independent LDS lookup chains hide each other's latency).
// slice-by-4 over NC full aligned chunks whose 16-B words are w[k][0..3] (per lane), chains
// interleaved; reg[k] in: the chain's start register, out: the lane's register pushed to the chunk end
template <int NC>
__device__ __forceinline__ void etag_fast(const Crc &T, const EtagSmem &S, uint32_t lane, const uint4 (&w)[NC][4],
                                          uint32_t (&reg)[NC]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int k = 0; k < NC; ++k) reg[k] = crc_word4(T, reg[k], w[k][i].x);
#pragma unroll
        for (int k = 0; k < NC; ++k) reg[k] = crc_word4(T, reg[k], w[k][i].y);
#pragma unroll
        for (int k = 0; k < NC; ++k) reg[k] = crc_word4(T, reg[k], w[k][i].z);
#pragma unroll
        for (int k = 0; k < NC; ++k) reg[k] = crc_word4(T, reg[k], w[k][i].w);
    }
    if (lane != 63) {
#pragma unroll
        for (int k = 0; k < NC; ++k) reg[k] = kmul_lane(reg[k], S, lane);
    }
}

__global__ __launch_bounds__(64 * ETAG_WPB) void k_etag_chunk(const uint8_t *__restrict__ data, uint64_t data_len,
                                                             const uint64_t *__restrict__ cdesc, uint64_t n_chunks,
                                                             const uint32_t *__restrict__ crc_tab,
                                                             const uint32_t *__restrict__ xt,
                                                             uint32_t *__restrict__ creg) {
    // byte tables in k_replay's Smem::C2 layout (64 KiB, see Crc), then per lane the nibble tables
    // of x^(8 (4096 - 64 (lane + 1))) as columns: entry (i, n, lane) at dword (16 i + n) 64 + lane,
    // so the 32 lanes of a half-wave read 32 banks whatever their nibbles (kmul_lane)
    __shared__ EtagSmem S;
    for (uint32_t i = threadIdx.x; i < 256 * 64; i += blockDim.x) S.C2[i] = crc_tab[c2_table((int)(i & 63u)) * 256 + (i >> 6)];
    for (uint32_t i = threadIdx.x; i < 64 * 128; i += blockDim.x) S.KL[i] = xt[ETAG_NX + (i & 63u) * 128 + (i >> 6)];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t *C2 = S.C2;
    Crc T;
    crc_init(T, C2, lane);
    const uint64_t waves = (uint64_t)gridDim.x * ETAG_WPB;
    const uint64_t wave = blockIdx.x * (uint64_t)ETAG_WPB + (threadIdx.x >> 6);
    // a round's chunks: start, length, start register (0xFFFFFFFF for lane 0 of a blob's first
    // chunk), and whether all of them are full and 16-B aligned (the fast path)
    auto round_desc = [&](uint64_t base, auto &start, auto &clen, auto &reg) -> bool {
        constexpr int NC = sizeof(clen) / sizeof(clen[0]);
        bool fast = true;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            const uint64_t c = base + k;
            start[k] = 0; clen[k] = 0; reg[k] = 0;
            if (c < n_chunks) {
                bool first;
                etag_desc(cdesc[c], start[k], clen[k], first);
                reg[k] = (first && lane == 0) ? 0xFFFFFFFFu : 0u;
            }
            fast = fast && clen[k] == ETAG_CH && ((reinterpret_cast<uintptr_t>(data) + start[k]) & 15u) == 0;
        }
        return fast;
    };
    auto finish = [&](uint64_t base, auto &reg) {
        constexpr int NC = sizeof(reg) / sizeof(reg[0]);
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            uint32_t r = reg[k];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) r ^= __shfl_xor(r, o, 64);
            if (lane == 0 && base + k < n_chunks) creg[base + k] = r;
        }
    };
#if KVR_ETAG_DB
    // double-buffered: the next round's descriptors and 16-B words are loaded before this round's
    // chains run, so every wave keeps a round of loads in flight while it computes
    constexpr int NC = ETAG_NC_DB;
    uint64_t base = wave * NC;
    uint64_t st[NC];
    uint32_t cl[NC], rg[NC];
    bool fast = base < n_chunks && round_desc(base, st, cl, rg);
    uint4 wa[NC][4];
    if (fast) {
#pragma unroll
        for (int k = 0; k < NC; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i) wa[k][i] = reinterpret_cast<const uint4 *>(data + st[k] + lane * 64u)[i];
    }
    for (; base < n_chunks; base += waves * NC) {
        const uint64_t nbase = base + waves * NC;
        uint64_t nst[NC];
        uint32_t ncl[NC], nrg[NC];
        const bool nfast = nbase < n_chunks && round_desc(nbase, nst, ncl, nrg);
        uint4 wb[NC][4];
        if (nfast) {
#pragma unroll
            for (int k = 0; k < NC; ++k)
#pragma unroll
                for (int i = 0; i < 4; ++i) wb[k][i] = reinterpret_cast<const uint4 *>(data + nst[k] + lane * 64u)[i];
        }
        if (fast) {
            etag_fast<NC>(T, S, lane, wa, rg);
        } else {
#pragma unroll 1
            for (int k = 0; k < NC; ++k)
                if (cl[k]) rg[k] = etag_unit_general(T, data, data_len, st[k], cl[k], lane, rg[k], xt);
        }
        finish(base, rg);
        fast = nfast;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            st[k] = nst[k]; cl[k] = ncl[k]; rg[k] = nrg[k];
#pragma unroll
            for (int i = 0; i < 4; ++i) wa[k][i] = wb[k][i];
        }
    }
#else
    for (uint64_t base = wave * ETAG_NC; base < n_chunks; base += waves * ETAG_NC) {
        uint64_t start[ETAG_NC];
        uint32_t clen[ETAG_NC], reg[ETAG_NC];
        const bool fast = round_desc(base, start, clen, reg);
        if (fast) {   // ETAG_NC full aligned chunks: 4 x 16-B loads per lane and chunk, chains interleaved
            uint4 w[ETAG_NC][4];
#pragma unroll
            for (int k = 0; k < ETAG_NC; ++k) {
                const uint4 *q = reinterpret_cast<const uint4 *>(data + start[k] + lane * 64u);
#pragma unroll
                for (int i = 0; i < 4; ++i) w[k][i] = q[i];
            }
            etag_fast<ETAG_NC>(T, S, lane, w, reg);
        } else {
#pragma unroll 1
            for (int k = 0; k < ETAG_NC; ++k)
                if (clen[k]) reg[k] = etag_unit_general(T, data, data_len, start[k], clen[k], lane, reg[k], xt);
        }
        finish(base, reg);
    }
#endif
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
