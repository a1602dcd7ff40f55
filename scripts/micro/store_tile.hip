// Store-pattern microbenchmark for the window-layout volume (diagnostic only): C3 window
// geometry (H 2048, WO 1792, DO 257): one workgroup per (16-column tile, 64-row band)
// writes, per step (row), its contiguous 16 x DO-float block with SS dword stores per thread.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, rem = nb % 8, x = b % 8, i = b / 8;
    return x < rem ? x * (q + 1) + i : rem * (q + 1) + (x - rem) * q + i;
}
// MODE bit0: xcd remap; bit1: barrier per step; bit2: band-fastest block order; bit3: dwordx4
// MODE bit4: per step and wave, the sweep's 14 row loads (fp16 image rows, f64/f32 stats rows)
template <int MODE>
__global__ __launch_bounds__(256) void k_tile(float* out, int64_t H, int64_t WO, int64_t DO, int TH, int nTile, int nBand,
                                              const __half* img, const double* sbox, const float* ssq) {
    const int64_t bid = (MODE & 1) ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    int wt, band;
    if (MODE & 4) { band = bid % nBand; wt = bid / nBand; } else { wt = bid % nTile; band = bid / nTile; }
    const int64_t u0 = (int64_t)wt * 16;
    const int nrow = (int)min((int64_t)16, WO - u0);
    const int total = nrow * (int)DO;
    const int tid = threadIdx.x, NT = blockDim.x;
    extern __shared__ float pad[];
    if (tid == 1000) pad[0] = 0.f;  // dynamic LDS only limits occupancy
    float ring[3] = {0.f, 0.f, 0.f};
    for (int64_t t = (int64_t)band * TH; t < min(H, (int64_t)(band + 1) * TH); ++t) {
        float* blk = out + (t * WO + u0) * DO;
        float acc = 0.f;
        if (MODE & 16) {
            // MODE bit5: loads of step t + 3 (consumed 3 steps later); bit6: wave 0 only;
            // bit7: image rows only; bit8: stats rows only
            int64_t tl = (MODE & 32) ? min(t + 3, H - 1) : t;
            if (MODE & 512) tl = 7;  // bit9: stats always from row 7 (L2-resident)
            const int64_t W = 2048, l = tid & 63, w = tid >> 6;
            const int64_t rE = min(tl + 5, H - 1), rL = max(tl - 6, (int64_t)0);
            const int64_t x0 = min(u0 - 5 + 64 * w + l, W - 1), x1 = min(x0 + 64, W - 1), xc = max(u0 - 5 + (l & 15), (int64_t)0);
            const int64_t xs = min(u0 + 64 * w + l, W - 1), xs1 = min(xs + 64, W - 1);
            float v = 0.f;
            if (!(MODE & 64) || w == 0) {
                if (!(MODE & 256)) {
                    v += (float)img[rE * W + max(x0, (int64_t)0)] + (float)img[rE * W + x1] + (float)img[rL * W + max(x0, (int64_t)0)] + (float)img[rL * W + x1];
                    v += (float)img[H * W + rE * W + xc] + (float)img[H * W + rE * W + xc + 16] + (float)img[H * W + rL * W + xc] + (float)img[H * W + rL * W + xc + 16];
                }
                if (!(MODE & 128))
                    v += (float)(sbox[tl * W + xs] + sbox[tl * W + xs1] + sbox[H * W + tl * W + xc]) + ssq[tl * W + xs] + ssq[tl * W + xs1] + ssq[H * W + tl * W + xc];
            }
            if (MODE & 32) { acc = ring[2]; ring[2] = ring[1]; ring[1] = ring[0]; ring[0] = v; }
            else acc = v;
        }
        if (MODE & 8) {
            float4* b4 = (float4*)blk;
            for (int i = tid; i * 4 < total; i += NT) {
                if (i * 4 + 3 < total) b4[i] = make_float4(1.f, 2.f, 3.f, (float)t);
                else for (int j = i * 4; j < total; ++j) blk[j] = 1.f;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                const int idx = i * NT + tid;
                if (idx < total) blk[idx] = (float)t + acc;
            }
        }
        if (MODE & 2) __syncthreads();
    }
}
__global__ void k_dword(float* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t st = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += st) out[i] = 1.f;
}

int main() {
  const int64_t H = 2048, WO = 1792, DO = 257;
  const int64_t n = H * WO * DO;
  float* out; hipMalloc(&out, n * 4);
  __half* img; hipMalloc(&img, 2 * 2048 * 2048 * 2); hipMemset(img, 0, 2 * 2048 * 2048 * 2);
  double* sbox; hipMalloc(&sbox, 2 * 2048 * 2048 * 8); hipMemset(sbox, 0, 2 * 2048 * 2048 * 8);
  float* ssq; hipMalloc(&ssq, 2 * 2048 * 2048 * 4); hipMemset(ssq, 0, 2 * 2048 * 2048 * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float ms;
  auto time = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(a); for (int r = 0; r < 10; ++r) launch(); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); ms /= 10;
    printf("%-44s %8.3f ms  %8.1f GB/s\n", name, ms, n * 4 / ms / 1e6);
  };
  time("dword grid-stride", [&]{ hipLaunchKernelGGL(k_dword, dim3(8192), dim3(256), 0, 0, out, n); });
  const int nTile = (WO + 15) / 16;
  for (int TH : {64}) {
    const int nBand = (H + TH - 1) / TH;
    dim3 g(nTile * nBand);
    char nm[80];
#define RUN(M, NAME) for (int lds : {50000}) { snprintf(nm, 80, "TH=%d %s lds=%d", TH, NAME, lds); \
    time(nm, [&]{ hipLaunchKernelGGL(k_tile<M>, g, dim3(256), lds, 0, out, H, WO, DO, TH, nTile, nBand, img, sbox, ssq); }); }
    RUN(3, "xcd+barrier");
    RUN(51, "+loads prefetch3");
    RUN(307, "+loads prefetch3 stats only");
    RUN(819, "+loads prefetch3 stats only, row 7");
    RUN(563, "+loads prefetch3 all, stats row 7");
  }
  return 0;
}
