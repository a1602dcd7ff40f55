// Store-path microbenchmark shaped like the forward sweep (diagnostic only):
// 6144 workgroups of 192 lanes, 64 row steps each, one barrier per step, per step a
// dummy fp64 compute of WORK dependent-FMA rounds and then the step's volume tile
// (16 camera columns x 192 diagonals of a 1024^3 full volume) stored as
//   V=1: one dword per lane per column (16 wave stores, the sweep's pattern)
//   V=4: the same bytes as dwordx4 (4 consecutive floats per lane, 4 wave stores)
// ALIGN=1 rounds segment starts to 16 B (best case for V=4).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, rem = nb % 8, x = b % 8, i = b / 8;
    return x < rem ? x * (q + 1) + i : rem * (q + 1) + (x - rem) * q + i;
}

template <int V, int ALIGN>
__global__ __launch_bounds__(192) void k_sim(float* out, int W, int work, int nchunk, int ntile) {
    const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
    const int chunk = (int)(b % nchunk);
    const int64_t rest = b / nchunk;
    const int tile = (int)(rest % ntile);
    const int band = (int)(rest / ntile);
    const int tid = threadIdx.x;
    const int u0 = tile * 16;
    double a0 = tid * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7FFFFFF0, 0x00020000);
    for (int s = 0; s < 64; ++s) {
        const int64_t h = (int64_t)band * 64 + s;
        for (int i = 0; i < work; ++i) {
            a0 = fma(a0, 0.999, 1e-3); a1 = fma(a1, 0.999, 1e-3);
            a2 = fma(a2, 0.999, 1e-3); a3 = fma(a3, 0.999, 1e-3);
        }
        const float v = (float)(a0 + a1 + a2 + a3);
        // descriptor-relative byte offsets inside rows h*W + u0 .. +15 (fits 31 bits per step)
        const auto rrow = __builtin_amdgcn_make_buffer_rsrc(out + (h * W + u0) * (int64_t)W, 0, 0x7FFFFFF0, 0x00020000);
        if constexpr (V == 3) {
            // overlapping chunks: chunk c stores columns [c*176, c*176+176) of every row
            // (64-B aligned, one owner per sector); lane l holds column c*176 - 15 + m + l
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int col = chunk * 176 - 15 + m + tid;
                const bool ok = col >= chunk * 176 && col < chunk * 176 + 176 && col < W;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v + m), rrow,
                                                      ok ? (uint32_t)((m * W + col) * 4) : 0x80000000u, 0, 0);
            }
        } else if constexpr (V == 2) {
            // segment [c0, c0+192) with c0 misaligned; stores issued on the 64-B grid
            // (4 wave stores per row, head/tail lanes masked)
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int c0 = chunk * 192 + m - 15, a0 = c0 & ~15;
                // 208 aligned columns [a0, a0+208) cover the segment; 3 waves x 64 lanes + wave 0 again
                {
                    const int col = a0 + tid;
                    const bool ok = col >= c0 && col < c0 + 192 && col >= 0 && col < W;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v + m), rrow,
                                                          ok ? (uint32_t)((m * W + col) * 4) : 0x80000000u, 0, 0);
                }
                if (tid < 64) {
                    const int col = a0 + 192 + tid;
                    const bool ok = col < c0 + 192 && col < W;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v + m), rrow,
                                                          ok ? (uint32_t)((m * W + col) * 4) : 0x80000000u, 0, 0);
                }
            }
        } else if constexpr (V == 1) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                int col = chunk * 192 + tid + m - 15;
                if (ALIGN) col = chunk * 192 + tid;
                const uint32_t off = (col >= 0 && col < W) ? (uint32_t)((m * W + col) * 4) : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v + m), rrow, off, 0, 0);
            }
        } else {
            // 48 lanes per column row (768 B), 4 rows per instruction
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = q * 4 + tid / 48, j = tid % 48;
                int col = chunk * 192 + 4 * j + m - 15;
                if (ALIGN) col = chunk * 192 + 4 * j;
                const uint32_t off = (col >= 0 && col + 3 < W) ? (uint32_t)((m * W + col) * 4) : 0x80000000u;
                const float4 w = make_float4(v, v + 1, v + 2, v + 3);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, w), rrow, off, 0, 0);
            }
        }
        __syncthreads();
    }
    (void)rs;
}

int main() {
    const int W = 1024, H = 1024;
    const int nchunk = 6, ntile = W / 16, nband = H / 64;
    const size_t n = (size_t)H * W * W;
    float* out;
    hipMalloc(&out, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = nchunk * ntile * nband;
    auto time = [&](const char* name, int work, auto kern) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(192), 0, 0, out, W, work, nchunk, ntile);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(192), 0, 0, out, W, work, nchunk, ntile);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        printf("%-24s work=%4d %8.3f ms %8.1f GB/s\n", name, work, ms, (double)blocks * 64 * 16 * 192 * 4 / ms / 1e6);
    };
    for (int work : {0, 32}) {
        time("dword", work, k_sim<1, 0>);
        time("dword aligned", work, k_sim<1, 1>);
        time("dword grid-aligned", work, k_sim<2, 0>);
        time("dword owned-sectors", work, k_sim<3, 0>);
        time("dwordx4", work, k_sim<4, 0>);
        time("dwordx4 aligned", work, k_sim<4, 1>);
    }
    return 0;
}
