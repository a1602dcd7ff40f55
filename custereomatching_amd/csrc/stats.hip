// Per-pixel patch statistics (one pass over each image, O(H W k^2), tiny
// next to the volume).  The fp32 mean / sq values replay, in the same order,
// the arithmetic every reference thread performs for its own patch
// (custma/src/stereo_matching_kernel.cu:40-54 mean, :56-69 centred squares),
// so hoisting them per pixel is bit-identical.  The fp64 box sum and
// fp64-accurate second moment feed the fast sliding-window paths.
#include "common.h"

namespace custma {

namespace {
constexpr int TS = 16;  // 16 x 16 pixels per 256-thread workgroup

template <typename T>
__global__ __launch_bounds__(256) void k_stats(const T* __restrict__ img, Geo g, Stats st) {
    extern __shared__ __attribute__((aligned(16))) float tile[];
    const int k = g.k, r = g.r, L = TS + 2 * r;
    const int64_t y0 = (int64_t)blockIdx.y * TS, x0 = (int64_t)blockIdx.x * TS;
    for (int e = threadIdx.x; e < L * L; e += 256) {
        const int ty = e / L, tx = e % L;
        tile[e] = ldpad(img, g.H, g.W, y0 + ty - r, x0 + tx - r);
    }
    __syncthreads();
    const int ly = threadIdx.x / TS, lx = threadIdx.x % TS;
    const int64_t y = y0 + ly, x = x0 + lx;
    if (y >= g.H || x >= g.W) return;
    const float* t = tile + ly * L + lx;
    float m = 0.f;
    double b = 0.0;
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) {
            const float v = t[i * L + j];
            m = m + v;
            b += (double)v;
        }
    m = m / (float)(k * k);
    const double m64 = b / (double)(k * k);
    float s = 0.f;
    double s64 = 0.0;
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) {
            const float v = t[i * L + j];
            const float c = v - m;
            s = __builtin_fmaf(c, c, s);
            const double c64 = (double)v - m64;
            s64 = fma(c64, c64, s64);
        }
    const int64_t p = y * g.W + x;
    st.mean[p] = m;
    st.sq[p] = s;
    st.box[p] = b;
    st.sqt[p] = (float)s64;
}
}  // namespace

hipError_t launch_stats(const void* img, int dtype, const Geo& g, Stats st, hipStream_t s) {
    const dim3 grid((unsigned)cdiv(g.W, TS), (unsigned)cdiv(g.H, TS));
    const int L = TS + 2 * g.r;
    const size_t lds = sizeof(float) * L * L;
    if (dtype == CUSTMA_F16)
        hipLaunchKernelGGL(k_stats<__half>, grid, dim3(256), lds, s, (const __half*)img, g, st);
    else
        hipLaunchKernelGGL(k_stats<float>, grid, dim3(256), lds, s, (const float*)img, g, st);
    return hipGetLastError();
}

}  // namespace custma
