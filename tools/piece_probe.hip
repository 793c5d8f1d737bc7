// Load-structure probe for the uniform-record piece mode of k_replay (diagnostic, not shipped).
//
// 1. Correctness: a 16-B raw buffer load at every byte offset 0..15 (the piece windows start at any
//    byte) against the bytes themselves.
// 2. Throughput over 4 GiB, 16 waves per workgroup, one workgroup per CU (k_replay's LDS pins it),
//    a wave walking a stripe of "steps" of 64 pieces:
//      tile      lane l reads [128 l, +128) of an 8-KiB tile (k_replay's unit layout)
//      piece-u   lane l reads the 128-B piece of a 1049-B record stream (cfg2's shape: 8 pieces
//                per record, 25 B of header and key between values) with byte-unaligned 16-B loads
//      piece-a   the same with 4-B aligned 16-B loads plus one dword, realigned by v_alignbyte
//    depth 1: one step in flight; depth 2: the next step's loads issued before this step's work.
//    DELAY dependent-free VALU per step stand in for the CRC.
// Build: hipcc --offload-arch=gfx950 -O3 -o piece_probe piece_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int RT = 1024;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_align(const uint8_t *buf, uint32_t *out) {
    const int lane = threadIdx.x;   // 16 lanes: offset = lane
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)0, 4096, 0x00020000);
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, lane, 0, 0);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * lane, 0, 0);
    out[8 * lane + 0] = a.x; out[8 * lane + 1] = a.y; out[8 * lane + 2] = a.z; out[8 * lane + 3] = a.w;
    out[8 * lane + 4] = b.x; out[8 * lane + 5] = b.y; out[8 * lane + 6] = b.z; out[8 * lane + 7] = b.w;
}

__device__ __forceinline__ uint32_t spin(uint32_t x, uint32_t y, int n) {
#pragma unroll 1
    for (int i = 0; i < n; i += 8) {
        asm volatile("v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %0\n v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %0\n"
                     "v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %0\n v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %0"
                     : "+v"(x), "+v"(y));
    }
    return x ^ y;
}

// PAT 0 tile, 1 piece-u, 2 piece-a
template <int PAT>
__device__ __forceinline__ void load_step(__amdgpu_buffer_rsrc_t rs, int off, uint32_t (&w)[33]) {
    if (PAT == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * i, 0, 0);
            w[4 * i] = a.x; w[4 * i + 1] = a.y; w[4 * i + 2] = a.z; w[4 * i + 3] = a.w;
        }
    } else {
        const int a0 = PAT == 2 ? (off & ~3) : off;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, a0 + 16 * i, 0, 0);
            w[4 * i] = a.x; w[4 * i + 1] = a.y; w[4 * i + 2] = a.z; w[4 * i + 3] = a.w;
        }
        if (PAT == 2) w[32] = __builtin_amdgcn_raw_buffer_load_b32(rs, a0 + 128, 0, 0);
    }
}

template <int PAT>
__device__ __forceinline__ uint32_t fold(const uint32_t (&w)[33], int off) {
    uint32_t x = 0;
    if (PAT == 2) {
        const uint32_t sh = (uint32_t)off & 3u;
#pragma unroll
        for (int i = 0; i < 32; ++i) x ^= __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) x ^= w[i];
    }
    return x;
}

// the 52-B header windows k_piece loads beside its pieces: 3 dwordx4 + 1 dword a step, WIN lanes
// reading (1049-B records apart), the others out of the resource (WMASK 0) or exec-masked off (1)
// (loaded in one step, consumed at the next: the wait for them never covers the pieces issued after)
template <int WIN, int WMASK>
__device__ __forceinline__ void windows(__amdgpu_buffer_rsrc_t rs, int lane, uint32_t (&wv)[13]) {
    if (WIN < 0) return;
    const int o = lane < WIN ? lane * 1049 + 3 : 0x7FFFFF00;
    if (WMASK && lane >= WIN) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (o & ~3) + 16 * i, 0, 0);
        wv[4 * i] = v.x; wv[4 * i + 1] = v.y; wv[4 * i + 2] = v.z; wv[4 * i + 3] = v.w;
    }
    wv[12] = __builtin_amdgcn_raw_buffer_load_b32(rs, (o & ~3) + 48, 0, 0);
}
__device__ __forceinline__ uint32_t wfold(uint32_t (&wv)[13]) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 13; ++i) x ^= wv[i];
    return x;
}

template <int PAT, int DEPTH, int NT = RT, int WIN = -1, int WMASK = 0>
__global__ __launch_bounds__(NT) void k_pat(const uint8_t *__restrict__ buf, uint64_t bytes_per_stripe,
                                            uint32_t n_stripes, int delay, uint32_t *sink) {
    __shared__ uint32_t pin[130 * 1024 / 4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) pin[0] = 0;
    const uint32_t si = blockIdx.x * (NT / 64) + __builtin_amdgcn_readfirstlane(wv);
    if (si >= n_stripes) return;
    const uint8_t *p = buf + (uint64_t)si * bytes_per_stripe;
    // a step: 64 pieces.  tile: 8 KiB.  piece: 8 records of 1049 B (8 pieces each)
    const uint32_t step_bytes = PAT == 0 ? 8192u : 8u * 1049u;
    const int off = PAT == 0 ? 128 * lane : (lane >> 3) * 1049 + 25 + 128 * (lane & 7);
    const uint64_t n_steps = (bytes_per_stripe - 1100) / step_bytes;
    uint32_t acc = 0;
    uint32_t a[33], b[33], c[33], wn[13] = {};
    auto rsrc = [&](uint64_t s) {   // (a step past the stripe re-reads the last one: never out of the buffer)
        s = s < n_steps ? s : n_steps - 1;
        return __builtin_amdgcn_make_buffer_rsrc((void *)(p + s * step_bytes), (short)0, (int)(step_bytes + 1100), 0x00020000);
    };
    load_step<PAT>(rsrc(0), off, a);
    if (DEPTH == 3) {   // three buffers: two steps in flight while one is worked on
        load_step<PAT>(rsrc(1), off, b);
#pragma unroll 1
        for (uint64_t s = 0; s < n_steps; s += 3) {
            load_step<PAT>(rsrc(s + 2), off, c);
            asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
            acc ^= spin(fold<PAT>(a, off), acc, delay);
            load_step<PAT>(rsrc(s + 3), off, a);
            asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
            acc ^= spin(fold<PAT>(b, off), acc, delay);
            load_step<PAT>(rsrc(s + 4), off, b);
            asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
            acc ^= spin(fold<PAT>(c, off), acc, delay);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (acc == 0x12345678u) sink[threadIdx.x] = acc + pin[0];
        return;
    }
#pragma unroll 1
    for (uint64_t s = 0; s < n_steps; s += 2) {
        if (DEPTH == 2) {
            load_step<PAT>(rsrc(s + 1), off, b);
            if (PAT == 2) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        acc ^= wfold(wn);
        windows<WIN, WMASK>(rsrc(s), lane, wn);
        acc ^= spin(fold<PAT>(a, off), acc, delay);
        if (DEPTH == 1) load_step<PAT>(rsrc(s + 1), off, b);
        if (DEPTH == 2) {
            load_step<PAT>(rsrc(s + 2), off, a);
            if (PAT == 2) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        acc ^= wfold(wn);
        windows<WIN, WMASK>(rsrc(s + 1), lane, wn);
        acc ^= spin(fold<PAT>(b, off), acc, delay);
        if (DEPTH == 1) load_step<PAT>(rsrc(s + 2), off, a);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc + pin[0];
}

template <int PAT, int DEPTH, int NT = RT, int WIN = -1, int WMASK = 0>
static void run(const uint8_t *d, uint64_t bytes, int cus, int delay, uint32_t *sink) {
    const uint32_t n_stripes = cus * (NT / 64);
    const uint64_t bps = bytes / n_stripes;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e9f;
    for (int it = 0; it < 6; ++it) {
        CK(hipEventRecord(e0));
        k_pat<PAT, DEPTH, NT, WIN, WMASK><<<cus, NT>>>(d, bps, n_stripes, delay, sink);
        const hipError_t le = hipGetLastError();
        if (le != hipSuccess) { printf("launch: %s\n", hipGetErrorString(le)); return; }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
    }
    const char *nm[] = {"tile", "piece-u", "piece-a"};
    printf("%-8s waves %2d depth %d win %2d mask %d delay %4d VALU: %.3f ms  %7.1f GB/s\n", nm[PAT], NT / 64, DEPTH, WIN, WMASK,
           delay, best, bytes / best / 1e6);
}

int main(int argc, char **argv) {
    const bool calib = argc > 1 && strcmp(argv[1], "calib") == 0;   // (tools/pmc_traffic.py: piece-a only)
    // 1. correctness of unaligned 16-B buffer loads
    uint8_t *d8; uint32_t *dout;
    CK(hipMalloc(&d8, 4096)); CK(hipMalloc(&dout, 16 * 8 * 4));
    std::vector<uint8_t> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 37 + 11);
    hipMemcpy(d8, h.data(), 4096, hipMemcpyHostToDevice);
    k_align<<<1, 16>>>(d8, dout);
    std::vector<uint32_t> o(16 * 8);
    hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
    int bad_u = 0, bad_4 = 0;
    for (int l = 0; l < 16; ++l) {
        uint32_t e[4], f[4];
        memcpy(e, h.data() + l, 16);
        memcpy(f, h.data() + 4 * l, 16);
        for (int i = 0; i < 4; ++i) { bad_u += o[8 * l + i] != e[i]; bad_4 += o[8 * l + 4 + i] != f[i]; }
    }
    printf("unaligned raw_buffer_load_b128: %s (%d bad words); dword-aligned: %s (%d bad)\n",
           bad_u ? "WRONG" : "exact", bad_u, bad_4 ? "WRONG" : "exact", bad_4);
    // 2. throughput
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t bytes = 4ull << 30;
    uint8_t *d; uint32_t *sink;
    if (hipMalloc(&d, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    CK(hipMalloc(&sink, RT * 4));
    CK(hipMemset(d, 1, bytes));
    if (calib) {   // the byte count FETCH_SIZE is calibrated against: every step's 8 records, once
        const uint32_t n_stripes = cus * 16;
        const uint64_t bps = bytes / n_stripes, n_steps = (bps - 1100) / (8u * 1049u);
        run<2, 2>(d, bytes, cus, 0, sink);
        printf("calib_bytes_per_dispatch=%llu\n", (unsigned long long)(n_stripes * n_steps * 8u * 1049u));
        return 0;
    }
    if (argc > 1 && strcmp(argv[1], "win") == 0) {   // the header-window loads beside the pieces (round 6)
        for (int delay : {0, 512}) {
            run<2, 1>(d, bytes, cus, delay, sink);
            run<2, 1, RT, 0, 0>(d, bytes, cus, delay, sink);
            run<2, 1, RT, 8, 0>(d, bytes, cus, delay, sink);
            run<2, 1, RT, 8, 1>(d, bytes, cus, delay, sink);
            run<2, 1, RT, 64, 0>(d, bytes, cus, delay, sink);
            run<2, 2>(d, bytes, cus, delay, sink);
            run<2, 2, RT, 0, 0>(d, bytes, cus, delay, sink);
            run<2, 2, RT, 8, 0>(d, bytes, cus, delay, sink);
            run<2, 2, RT, 8, 1>(d, bytes, cus, delay, sink);
            run<2, 2, RT, 64, 0>(d, bytes, cus, delay, sink);
        }
        return 0;
    }
    if (argc > 1 && strcmp(argv[1], "waves") == 0) {   // waves per CU x pieces in flight (round 6)
        for (int delay : {256, 512, 1024, 1536}) {
            run<2, 1>(d, bytes, cus, delay, sink);
            run<2, 2>(d, bytes, cus, delay, sink);
            run<2, 2, 768>(d, bytes, cus, delay, sink);
            run<2, 3, 768>(d, bytes, cus, delay, sink);
            run<2, 2, 512>(d, bytes, cus, delay, sink);
            run<2, 3, 512>(d, bytes, cus, delay, sink);
        }
        return 0;
    }
    for (int delay : {0, 256, 512}) {
        run<0, 1>(d, bytes, cus, delay, sink);
        run<1, 1>(d, bytes, cus, delay, sink);
        run<2, 1>(d, bytes, cus, delay, sink);
        run<0, 2>(d, bytes, cus, delay, sink);
        run<1, 2>(d, bytes, cus, delay, sink);
        run<2, 2>(d, bytes, cus, delay, sink);
    }
    return 0;
}
