// Shared device/host definitions for the gfx950 ZNCC kernels.
// Compiled with -ffp-contract=off: every fused multiply-add below is an
// explicit __builtin_fmaf / fma, so the reference's nvcc contraction
// (custma/src/stereo_matching_kernel.cu:66-71 under -fmad=true) is
// reproduced exactly where the exact path needs it and nowhere else.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/custma.h"

namespace custma {

constexpr float kEps = 1e-8f;  // stereo_matching_kernel.cu:4

// Problem geometry shared by every kernel.
struct Geo {
    int64_t H, W;   // image
    int32_t k, r;   // kernel size, radius
    int32_t layout; // CUSTMA_LAYOUT_*
    int32_t D;
    int64_t WO, DO; // volume [h_hi - h_lo, WO, DO]
    int64_t h_lo, h_hi;  // volume rows = image rows [h_lo, h_hi) (row bands: the rest is halo)
    __host__ __device__ int64_t HV() const { return h_hi - h_lo; }
};

// Per-image statistics produced by the stats pass ([H*W] each).
//   mean, sq : the reference's own fp32 values (sequential sum / k^2, fma chain of
//              centred squares) -- bit-identical to what every reference thread computes.
//   box      : fp64 sum of the zero-padded k x k patch (exact for fp32 inputs up to
//              2^29 dynamic range).
//   sqt      : fp64-accurate centred second moment (box2 - box^2/k^2), rounded to fp32.
struct Stats {
    float* mean;
    float* sq;
    double* box;
    float* sqt;
};

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }

// zero-padded read (stereo_matching_kernel.cu:6-12), 64-bit indexing
template <typename T>
__device__ __forceinline__ float ldpad(const T* img, int64_t H, int64_t W, int64_t y, int64_t x) {
    return (y < 0 || y >= H || x < 0 || x >= W) ? 0.f : to_f(img[y * W + x]);
}

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Volume voxel validity and linear index for camera column w, projector column d.
__device__ __forceinline__ bool voxel_valid(const Geo& g, int64_t w, int64_t d) {
    if (w < 0 || w >= g.WO || d < 0 || d >= g.W) return false;
    if (g.layout == CUSTMA_LAYOUT_WINDOW) return d >= w && d - w <= g.D;
    return true;
}
__device__ __forceinline__ int64_t voxel_index(const Geo& g, int64_t h, int64_t w, int64_t d) {
    const int64_t s = (g.layout == CUSTMA_LAYOUT_WINDOW) ? d - w : d;
    return ((h - g.h_lo) * g.WO + w) * g.DO + s;
}

}  // namespace custma

// ---- internal launchers (one translation unit each), called from capi.hip ----
namespace custma {
hipError_t launch_stats(const void* img, int dtype, const Geo& g, Stats st, hipStream_t s);
hipError_t launch_fwd_exact(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            float* out, hipStream_t s);
hipError_t launch_fwd_fast(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                           float* out, hipStream_t s);
hipError_t launch_argmax(const float* vol, int64_t rows, int64_t n, int64_t* idx, float* best, hipStream_t s);
size_t disparity_partial_bytes(const Geo& g);
hipError_t launch_disparity(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            int64_t* idx, float* best, int32_t* n_rechecked, void* ws, hipStream_t s);
size_t backward_partial_bytes(const Geo& g);
hipError_t launch_backward(const float* grad, const void* cam, const void* proj, int dtype, const Geo& g,
                           Stats sc, Stats sp, float* dcam, float* dproj, void* ws, hipStream_t s);
bool fast_supported(int k);
}  // namespace custma
