// Store-pattern micro-benchmark of the full-layout sweep (k_sweep_fwd, round 6; diagnostic only).
// C2 full geometry: volume [1024][1024][1024] fp32 = 4.29 GB.  A workgroup owns (band of TH rows, 16-column
// tile, chunk of S = 176 owned volume columns) as sweep_grid(owned) lays it out for C2 (3 compute waves of 64
// diagonal lanes + 1 loader wave); per step it writes its 16 rows x S floats (16 segments of 704 bytes, one
// per camera column of the tile, 4 KB apart), nothing computed, one barrier per step.  Variants: dword vs
// 16-byte stores, nt vs default policy, waves per workgroup.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, rem = nb % 8, x = b % 8, i = b / 8;
    return x < rem ? x * (q + 1) + i : rem * (q + 1) + (x - rem) * q + i;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}

template <bool X4, int AUX>
__global__ __launch_bounds__(256) void k_full(float* out, int64_t H, int64_t W, int S, int nChunk, int nTile, int TH,
                                              int NC) {
    extern __shared__ float pad[];
    if (threadIdx.x == 1000) pad[0] = 0.f;
    const int64_t bid = xcd_remap(blockIdx.x, gridDim.x);
    const int chunk = (int)(bid % nChunk);
    const int64_t rest = bid / nChunk;
    const int wt = (int)(rest % nTile), band = (int)(rest / nTile);
    const int64_t u0 = (int64_t)wt * 16, h0 = (int64_t)band * TH, h1 = h0 + TH < H ? h0 + TH : H;
    const int cb = chunk * S, ce = cb + S < W ? cb + S : (int)W;
    const int tid = threadIdx.x;
    if (tid >= NC) {  // the loader wave: barriers only
        for (int64_t t = h0; t < h1; ++t) __syncthreads();
        return;
    }
    for (int64_t t = h0; t < h1; ++t) {
        float* base = out + (t * W + u0) * W;
        const auto r = rsrc(base, 0x7FFFFFF0u);
        if constexpr (X4) {
            const int gpr = S / 4;
            for (int q = tid; q < 16 * gpr; q += NC) {
                const int m = q / gpr, c = cb + 4 * (q % gpr);
                const bool ok = c < ce;
                const i32x4 v = {q, m, c, (int)t};
                __builtin_amdgcn_raw_buffer_store_b128(v, r, ok ? (uint32_t)((m * W + c) * 4) : 0x80000000u, 0u, AUX);
            }
        } else {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int c = cb + tid;
                __builtin_amdgcn_raw_buffer_store_b32((unsigned)m, r, c < ce ? (uint32_t)((m * W + c) * 4) : 0x80000000u,
                                                      0u, AUX);
            }
        }
        __syncthreads();
    }
}

int main() {
    const int64_t H = 1024, W = 1024;
    const int64_t n = H * W * W;
    float* out;
    if (hipMalloc(&out, n * 4 + 4096) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto time = [&](const char* name, auto launch) {
        for (int r = 0; r < 30; ++r) launch();
        (void)hipDeviceSynchronize();
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            for (int r = 0; r < 10; ++r) launch();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            ms /= 10;
            best = ms < best ? ms : best;
        }
        printf("%-60s %8.4f ms  %7.1f GB/s\n", name, best, n * 4 / best / 1e6);
        fflush(stdout);
    };
    char nm[128];
    for (int TH : {64, 32, 128}) {
        const int S = 176, NC = 192, nChunk = (int)((W + S - 1) / S), nTile = (int)(W / 16);
        const int nBand = (int)((H + TH - 1) / TH);
        const dim3 grid(nChunk * nTile * nBand), blk(NC + 64);
        // dynamic LDS as the kernel's (49.7 KB at C2: 3 workgroups per CU)
        snprintf(nm, sizeof nm, "full S%d TH%d dword nt (the kernel's pattern at TH64)", S, TH);
        time(nm, [&] { hipLaunchKernelGGL((k_full<false, 2>), grid, blk, 50000, 0, out, H, W, S, nChunk, nTile, TH, NC); });
        snprintf(nm, sizeof nm, "full S%d TH%d dword default", S, TH);
        time(nm, [&] { hipLaunchKernelGGL((k_full<false, 0>), grid, blk, 50000, 0, out, H, W, S, nChunk, nTile, TH, NC); });
        snprintf(nm, sizeof nm, "full S%d TH%d x4 nt", S, TH);
        time(nm, [&] { hipLaunchKernelGGL((k_full<true, 2>), grid, blk, 50000, 0, out, H, W, S, nChunk, nTile, TH, NC); });
    }
    return 0;
}
