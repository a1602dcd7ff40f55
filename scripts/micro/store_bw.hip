// Store-bandwidth microbenchmark for the volume write pattern (diagnostic only).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

// (a) each wave writes 256 B contiguous per instruction (dword per lane), rows of W floats,
//     segment start offset `off` floats (misalignment), 16 rows per lane-step like the sweep.
__global__ void k_rows(float* out, int64_t W, int64_t rows, int off, int nchunk) {
  int64_t b = blockIdx.x;
  int chunk = b % nchunk; int64_t rowgrp = b / nchunk;
  int tid = threadIdx.x;
  for (int m = 0; m < 16; ++m) {
    int64_t row = rowgrp * 16 + m;
    if (row >= rows) break;
    int64_t col = (int64_t)chunk * blockDim.x + tid + off + m;   // diagonal shift like full layout
    if (col < W) out[row * W + col] = (float)m;
  }
}
// (b) float4 per lane, 1 KB per wave instruction, aligned
__global__ void k_vec4(float4* out, int64_t n4) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t st = (int64_t)gridDim.x * blockDim.x;
  for (; i < n4; i += st) out[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}
// (c) dword per lane grid-stride aligned
__global__ void k_dword(float* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t st = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += st) out[i] = 1.f;
}

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, rem = nb % 8, x = b % 8, i = b / 8;
    return x < rem ? x * (q + 1) + i : rem * (q + 1) + (x - rem) * q + i;
}
template <bool NT>
__global__ void k_rows_x(float* out, int64_t W, int64_t rows, int off, int nchunk) {
  int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  int chunk = b % nchunk; int64_t rowgrp = b / nchunk;
  int tid = threadIdx.x;
  for (int m = 0; m < 16; ++m) {
    int64_t row = rowgrp * 16 + m;
    if (row >= rows) break;
    int64_t col = (int64_t)chunk * blockDim.x + tid + off + m;
    if (col < W) { if (NT) __builtin_nontemporal_store((float)m, out + row * W + col); else out[row * W + col] = (float)m; }
  }
}
// one WG per 16-row group, 256 threads, loops over the whole row (4 KB) : contiguous 64 KB per WG
__global__ void k_rows_full(float* out, int64_t W, int64_t rows, int off) {
  int64_t rowgrp = blockIdx.x;
  int tid = threadIdx.x;
  for (int m = 0; m < 16; ++m) {
    int64_t row = rowgrp * 16 + m;
    for (int64_t c = tid + off; c < W; c += blockDim.x) out[row * W + c] = (float)m;
  }
}

int main() {
  const int64_t W = 1024, H = 1024;
  const int64_t rows = H * W;            // volume rows of W floats
  const int64_t n = rows * W;            // 1.07e9 floats = 4.3 GB
  float* out; hipMalloc(&out, n * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float ms;
  auto time = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(a); for (int r = 0; r < 5; ++r) launch(); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); ms /= 5;
    printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms, n * 4 / ms / 1e6);
  };
  time("vec4 grid-stride (1KB/wave)", [&]{ hipLaunchKernelGGL(k_vec4, dim3(8192), dim3(256), 0, 0, (float4*)out, n/4); });
  time("dword grid-stride (256B/wave)", [&]{ hipLaunchKernelGGL(k_dword, dim3(8192), dim3(256), 0, 0, out, n); });
  for (int off : {0, 7}) {
    char nm[64]; snprintf(nm, 64, "rows 256-lane chunks off=%d", off);
    int nchunk = (W + 255) / 256;
    time(nm, [&]{ hipLaunchKernelGGL(k_rows, dim3((rows / 16) * nchunk), dim3(256), 0, 0, out, W, rows, off, nchunk); });
  }
  {
    int nchunk = (W + 255) / 256;
    time("rows xcd-remap off=7", [&]{ hipLaunchKernelGGL(k_rows_x<false>, dim3((rows / 16) * nchunk), dim3(256), 0, 0, out, W, rows, 7, nchunk); });
    time("rows xcd-remap nt off=7", [&]{ hipLaunchKernelGGL(k_rows_x<true>, dim3((rows / 16) * nchunk), dim3(256), 0, 0, out, W, rows, 7, nchunk); });
    time("rows full-row per WG", [&]{ hipLaunchKernelGGL(k_rows_full, dim3(rows / 16), dim3(256), 0, 0, out, W, rows, 0); });
  }
  return 0;
}
