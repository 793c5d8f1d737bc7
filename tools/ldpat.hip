// Load-structure microbenchmark for k_replay's tile loop (diagnostic, not shipped).
//
// Each wave walks a stripe of consecutive 8-KiB tiles, 16 waves per workgroup and one workgroup
// per CU (an LDS allocation the size of k_replay's pins the occupancy), like k_replay.  Per tile
// the wave loads the tile into 32 VGPRs per lane, waits, XOR-folds it (kept alive) and optionally
// spins for DELAY VALU instructions, standing in for the tile's compute.  Variants:
//   pattern 0  lane l holds bytes [128 l, 128 l + 128): instruction i reads 16 B at 128 l + 16 i
//              (k_replay's unit layout: 64 distinct lines per instruction)
//   pattern 1  instruction i reads the contiguous KiB [1024 i, 1024 i + 1024): 16 B at 1024 i + 16 l
//   depth 1    one tile in flight: the next load is issued after this tile's compute
//   depth 2    the next tile's load is issued before this tile's compute (64 VGPRs of tile data)
// Prints GB/s for each (pattern, depth, delay).  Build: hipcc --offload-arch=gfx950 -O3 -o ldpat ldpat.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int RT = 1024, TILE = 8192;

template <int PAT>
__device__ __forceinline__ void load_tile(const uint8_t *base, int lane, uint32_t (&w)[32]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int off = PAT == 0 ? (128 * lane + 16 * i) : (1024 * i + 16 * lane);
        const uint4 v = *reinterpret_cast<const uint4 *>(base + off);
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
}

__device__ __forceinline__ uint32_t spin(uint32_t x, int n) {
#pragma unroll 1
    for (int i = 0; i < n; i += 8) {
        asm volatile("v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n"
                     "v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0"
                     : "+v"(x));
    }
    return x;
}

// VALU issue rate: n instructions per lane as 4 independent dependent chains (ILP 4), or one chain
template <int ILP>
__global__ __launch_bounds__(RT) void k_valu(uint32_t *sink, int n) {
    __shared__ uint32_t pin[100 * 1024 / 4];
    uint32_t a = threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u;
    if (threadIdx.x == 0) pin[0] = 0;
#pragma unroll 1
    for (int i = 0; i < n; i += 8) {
        if (ILP == 4)
            asm volatile("v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %1, %1, %1, %1\n v_xad_u32 %2, %2, %2, %2\n v_xad_u32 %3, %3, %3, %3\n"
                         "v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %1, %1, %1, %1\n v_xad_u32 %2, %2, %2, %2\n v_xad_u32 %3, %3, %3, %3"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        else if (ILP == 2)
            asm volatile("v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %0\n v_xor_b32 %2, %2, %3\n v_xor_b32 %3, %3, %2\n"
                         "v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %0\n v_xor_b32 %2, %2, %3\n v_xor_b32 %3, %3, %2"
                         : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        else
            asm volatile("v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n"
                         "v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0\n v_xad_u32 %0, %0, %0, %0"
                         : "+v"(a));
    }
    if ((a ^ b ^ c ^ d) == 0x12345678u) sink[threadIdx.x] = a + pin[0];
}

template <int PAT, int DEPTH>
__global__ __launch_bounds__(RT) void k_pat(const uint8_t *__restrict__ buf, uint64_t tiles_per_stripe,
                                            uint32_t n_stripes, int delay, uint32_t *sink) {
    __shared__ uint32_t pin[100 * 1024 / 4];   // k_replay-sized LDS: one workgroup per CU
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) pin[0] = 0;
    const uint32_t si = blockIdx.x * (RT / 64) + wv;
    if (si >= n_stripes) return;
    const uint8_t *p = buf + (uint64_t)si * tiles_per_stripe * TILE;
    uint32_t acc = 0;
    uint32_t a[32], b[32];
    load_tile<PAT>(p, lane, a);
#pragma unroll 1
    for (uint64_t k = 0; k < tiles_per_stripe; ++k) {
        if (DEPTH == 2 && k + 1 < tiles_per_stripe) load_tile<PAT>(p + (k + 1) * TILE, lane, b);
        if (DEPTH == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) x ^= a[i];
        acc ^= spin(x, delay);
        if (DEPTH == 2) {
#pragma unroll
            for (int i = 0; i < 32; ++i) a[i] = b[i];
        } else if (k + 1 < tiles_per_stripe) {
            load_tile<PAT>(p + (k + 1) * TILE, lane, a);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 0x12345678u) sink[threadIdx.x] = acc + pin[0];
}

int main(int argc, char **argv) {
    const uint64_t bytes = 4ull << 30;
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    uint8_t *buf;
    uint32_t *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4096 * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 0x5A, bytes);
    const uint32_t n_stripes = (uint32_t)ncu * (RT / 64);
    const uint64_t tps = bytes / TILE / n_stripes;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("cus=%d stripes=%u tiles/stripe=%llu bytes=%llu\n", ncu, n_stripes, (unsigned long long)tps,
           (unsigned long long)(tps * n_stripes * TILE));
    {   // VALU issue: 16 waves per CU, 1<<16 instructions per lane
        const int n = 1 << 16;
        for (int ilp : {1, 2, 4}) {
            auto run = [&]() {
                if (ilp == 1) hipLaunchKernelGGL((k_valu<1>), dim3(ncu), dim3(RT), 0, 0, sink, n);
                if (ilp == 2) hipLaunchKernelGGL((k_valu<2>), dim3(ncu), dim3(RT), 0, 0, sink, n);
                if (ilp == 4) hipLaunchKernelGGL((k_valu<4>), dim3(ncu), dim3(RT), 0, 0, sink, n);
            };
            run();
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            hipEventRecord(e0);
            run();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // per SIMD: 4 waves x n instructions; cycles at the measured clock below
            int khz = 0;
            hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
            const double cyc = ms * 1e-3 * khz * 1e3;
            printf("valu ilp %d (%s): %.3f ms, %.2f cycles per wave64 VALU per SIMD at %d MHz\n", ilp,
                   ilp == 2 ? "v_xor_b32 pairs" : "v_xad_u32", ms, cyc / (4.0 * n), khz / 1000);
            fflush(stdout);
        }
    }
    const int delays[] = {0, 256, 512, 1024, 2048};
    for (int pat = 0; pat < 2; ++pat)
        for (int depth = 1; depth <= 2; ++depth)
            for (int d : delays) {
                auto launch = [&]() {
                    dim3 g(ncu), t(RT);
                    if (pat == 0 && depth == 1) hipLaunchKernelGGL((k_pat<0, 1>), g, t, 0, 0, buf, tps, n_stripes, d, sink);
                    if (pat == 0 && depth == 2) hipLaunchKernelGGL((k_pat<0, 2>), g, t, 0, 0, buf, tps, n_stripes, d, sink);
                    if (pat == 1 && depth == 1) hipLaunchKernelGGL((k_pat<1, 1>), g, t, 0, 0, buf, tps, n_stripes, d, sink);
                    if (pat == 1 && depth == 2) hipLaunchKernelGGL((k_pat<1, 2>), g, t, 0, 0, buf, tps, n_stripes, d, sink);
                };
                launch();
                if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
                float best = 1e9f;
                for (int r = 0; r < 5; ++r) {
                    hipEventRecord(e0);
                    launch();
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms = 0;
                    hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best) best = ms;
                }
                const double gb = (double)(tps * n_stripes * TILE) / 1e9;
                printf("pattern %d depth %d delay %5d VALU: %.3f ms  %7.1f GB/s\n", pat, depth, d, best, gb / best * 1e3);
                fflush(stdout);
            }
    return 0;
}
