// Exact forward: bit-identical to the reference arithmetic.
//
// Reference (custma/src/stereo_matching_kernel.cu:17-72, nvcc -fmad=true):
//   exy = fma chain over taps t = (i, j) in row-major order of
//         (cam_t - cam_mean) * (proj_t - proj_mean), starting at +0
//   cost = (exy + eps) / sqrtf(fmaf(ex2, ey2, eps))
// Per camera row h this is E_h = Xc_h * Yc_h^T with K = k*k taps: a GEMM.
// gfx950's f32-input MFMA (v_mfma_f32_32x32x2_f32) computes, per output,
// D = fma(a1, b1, fma(a0, b0, C)) -- a k-ordered fp32 fma chain, one rounding
// per product, no wider accumulator -- so feeding taps (2s, 2s+1) at step s
// reproduces the reference chain bit for bit.  ex2/ey2 and the means come
// from the stats pass (same arithmetic as every reference thread).
//
// Tiling: one workgroup = 4 waves = one camera row h, 32 camera columns
// (the MFMA M dim, lane&31) x 256 projector columns (4 waves x 2 N-tiles of
// 32).  The k x (32+2r) camera and k x (256+2r) projector strips are staged
// in LDS once; centred operands are formed on the fly (1 LDS read + 1 sub per
// operand per MFMA step), which is far below the 64-cycle MFMA issue.
#include "common.h"

namespace custma {

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int TWX = 32;   // camera columns per workgroup
constexpr int TDX = 256;  // projector columns per workgroup

template <typename T>
__global__ __launch_bounds__(256) void k_fwd_exact(const T* __restrict__ cam, const T* __restrict__ proj,
                                                   Geo g, Stats sc, Stats sp, float* __restrict__ out,
                                                   int nWT, int nDC) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int k = g.k, r = g.r, K = k * k;
    const int CW = TWX + 2 * r, PW = TDX + 2 * r;
    float* camT = lds;                // [k][CW]
    float* projT = camT + k * CW;     // [k][PW]
    float* csq = projT + k * PW;      // [TWX]
    float* cmn = csq + TWX;           // [TWX]
    float* psq = cmn + TWX;           // [TDX]
    float* pmn = psq + TDX;           // [TDX]

    const int64_t b = blockIdx.x;
    const int dc = (int)(b % nDC);
    const int wt = (int)((b / nDC) % nWT);
    const int64_t h = g.h_lo + b / ((int64_t)nDC * nWT);
    const int64_t w0 = (int64_t)wt * TWX;
    const int64_t dA = (g.layout == CUSTMA_LAYOUT_WINDOW ? w0 : 0) + (int64_t)dc * TDX;

    for (int e = threadIdx.x; e < k * CW; e += 256) {
        const int i = e / CW, x = e % CW;
        camT[e] = ldpad(cam, g.H, g.W, h + i - r, w0 + x - r);
    }
    for (int e = threadIdx.x; e < k * PW; e += 256) {
        const int i = e / PW, x = e % PW;
        projT[e] = ldpad(proj, g.H, g.W, h + i - r, dA + x - r);
    }
    if (threadIdx.x < TWX) {
        const int64_t w = w0 + threadIdx.x;
        const bool ok = w < g.W;
        csq[threadIdx.x] = ok ? sc.sq[h * g.W + w] : 0.f;
        cmn[threadIdx.x] = ok ? sc.mean[h * g.W + w] : 0.f;
    }
    {
        const int64_t d = dA + threadIdx.x;
        const bool ok = d < g.W;
        psq[threadIdx.x] = ok ? sp.sq[h * g.W + d] : 0.f;
        pmn[threadIdx.x] = ok ? sp.mean[h * g.W + d] : 0.f;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wl = lane & 31, kh = lane >> 5;
    const int64_t dt0 = dA + 64 * wave, dt1 = dt0 + 32;
    auto tile_live = [&](int64_t dt) {
        if (dt >= g.W || w0 >= g.WO) return false;
        if (g.layout == CUSTMA_LAYOUT_WINDOW) return dt - (w0 + TWX - 1) <= g.D && dt + 31 - w0 >= 0;
        return true;
    };
    const bool live0 = tile_live(dt0), live1 = tile_live(dt1);
    if (!live0 && !live1) return;

    const float mc = cmn[wl];
    const float mp0 = pmn[64 * wave + wl], mp1 = pmn[64 * wave + 32 + wl];
    const float* pr0 = projT + 64 * wave + wl;
    const float* pr1 = pr0 + 32;
    const float* cr = camT + wl;

    f32x16 acc0, acc1;
    for (int e = 0; e < 16; ++e) { acc0[e] = 0.f; acc1[e] = 0.f; }

    const int steps = (K + 1) / 2;
    int i = 0, j = kh, t = kh;
    if (live0 && live1) {
        for (int s = 0; s < steps; ++s) {
            const bool vt = t < K;
            const int oc = i * CW + j, op = i * PW + j;
            const float a = vt ? cr[oc] - mc : 0.f;
            const float b0 = vt ? pr0[op] - mp0 : 0.f;
            const float b1 = vt ? pr1[op] - mp1 : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);
            t += 2; j += 2;
            if (j >= k) { j -= k; ++i; }
        }
    } else {
        const float* pr = live0 ? pr0 : pr1;
        const float mp = live0 ? mp0 : mp1;
        for (int s = 0; s < steps; ++s) {
            const bool vt = t < K;
            const float a = vt ? cr[i * CW + j] - mc : 0.f;
            const float bb = vt ? pr[i * PW + j] - mp : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc0, 0, 0, 0);
            t += 2; j += 2;
            if (j >= k) { j -= k; ++i; }
        }
        if (!live0) acc1 = acc0;
    }

    // epilogue: cost = (E + eps) / sqrtf(fmaf(X, Y, eps))   (stereo_matching_kernel.cu:71)
    for (int q = 0; q < 2; ++q) {
        if (q == 0 ? !live0 : !live1) continue;
        const int64_t d = (q == 0 ? dt0 : dt1) + wl;
        const float Y = psq[64 * wave + 32 * q + wl];
        const f32x16& acc = q == 0 ? acc0 : acc1;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int wrow = (e & 3) + 8 * (e >> 2) + 4 * kh;
            const int64_t w = w0 + wrow;
            if (!voxel_valid(g, w, d)) continue;
            const float X = csq[wrow];
            const float den = sqrtf(__builtin_fmaf(X, Y, kEps));
            out[voxel_index(g, h, w, d)] = (acc[e] + kEps) / den;
        }
    }
}
}  // namespace

hipError_t launch_fwd_exact(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            float* out, hipStream_t s) {
    const int nWT = (int)cdiv(g.WO, TWX);
    const int nDC = (int)(g.layout == CUSTMA_LAYOUT_WINDOW ? cdiv(TWX + g.D, TDX) : cdiv(g.W, TDX));
    const int64_t blocks = g.HV() * nWT * nDC;
    const size_t lds = sizeof(float) * (g.k * (TWX + 2 * g.r) + g.k * (TDX + 2 * g.r) + 2 * TWX + 2 * TDX);
    hipError_t e = dtype == CUSTMA_F16 ? allow_lds(k_fwd_exact<__half>, lds) : allow_lds(k_fwd_exact<float>, lds);
    if (e != hipSuccess) return e;
    if (dtype == CUSTMA_F16)
        hipLaunchKernelGGL(k_fwd_exact<__half>, dim3((unsigned)blocks), dim3(256), lds, s, (const __half*)cam,
                           (const __half*)proj, g, sc, sp, out, nWT, nDC);
    else
        hipLaunchKernelGGL(k_fwd_exact<float>, dim3((unsigned)blocks), dim3(256), lds, s, (const float*)cam,
                           (const float*)proj, g, sc, sp, out, nWT, nDC);
    return hipGetLastError();
}

}  // namespace custma
