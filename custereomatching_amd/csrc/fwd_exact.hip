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
#include <type_traits>

#include "common.h"
#include "sweep.h"

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

    // the patch rows through batched unconditional loads (common.h tile_to_lds; a bounds-tested load
    // per element was waited for one at a time)
    tile_to_lds<T, 8>(cam, g.H, g.W, h - r, w0 - r, k, CW, camT, CW, (int)threadIdx.x, 256);
    tile_to_lds<T, 8>(proj, g.H, g.W, h - r, dA - r, k, PW, projT, PW, (int)threadIdx.x, 256);
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
// Compile-time kernel size (KT <= kExactMaxKT): the same MFMA chain with the tap loop laid out at
// compile time.  The runtime-k kernel above branches per step on the tap's validity and reads its
// three operands one after another, each behind an lgkmcnt(0) wait (C3 window k = 19: 17.7 ms, 0.25
// of the fp32 MFMA rate).  Here two image rows (2 KT taps = KT MFMA steps, the same tap-pair pattern
// for every row pair) are one unrolled block -- every LDS read is a base VGPR + an immediate offset
// -- looped over the row pairs (a fully unrolled K^2/2-step loop overflows the instruction cache at
// k = 31), then the last row of an odd KT; a lane's tap is t = 2 s + (lane >> 5), so a step's pair
// either stays in one row (the kh = 1 lanes read one column on) or wraps to the next row's column 0
// (they read one row on, KT - 1 columns back): two per-lane bases cover both.
// Each wave keeps NT accumulator tiles (the camera operand feeds NT MFMAs): window layouts use 3
// waves x 3 tiles = 288 projector columns (all 32 + 256 diagonals of a D = 256 window in one
// workgroup, instead of a second 256-column workgroup for the last 32), the full layout 4 x 2.
constexpr int kExactMaxKT = 33;

template <typename T, int KT, int NW, int NT>
__global__ __launch_bounds__(64 * NW) void k_fwd_exact_k(const T* __restrict__ cam, const T* __restrict__ proj,
                                                         Geo g, Stats sc, Stats sp, float* __restrict__ out,
                                                         int nWT, int nDC) {
    constexpr int R0 = KT / 2, NC = 32 * NW * NT, CW = TWX + KT - 1, PW = NC + KT - 1, NTH = 64 * NW;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* camT = lds;              // [KT][CW]
    float* projT = camT + KT * CW;  // [KT][PW]
    float* csq = projT + KT * PW;   // [TWX]
    float* cmn = csq + TWX;         // [TWX]
    float* psq = cmn + TWX;         // [NC]
    float* pmn = psq + NC;          // [NC]

    const int64_t b = blockIdx.x;
    const int dc = (int)(b % nDC);
    const int wt = (int)((b / nDC) % nWT);
    const int64_t h = g.h_lo + b / ((int64_t)nDC * nWT);
    const int64_t w0 = (int64_t)wt * TWX;
    const int64_t dA = (g.layout == CUSTMA_LAYOUT_WINDOW ? w0 : 0) + (int64_t)dc * NC;

    // the patch rows through batched unconditional loads (common.h tile_to_lds): a bounds-tested load per
    // element was waited for one at a time -- ~35 round trips per thread at k = 19, more than the MFMA work
    tile_to_lds<T, 8>(cam, g.H, g.W, h - R0, w0 - R0, KT, CW, camT, CW, (int)threadIdx.x, NTH);
    tile_to_lds<T, 8>(proj, g.H, g.W, h - R0, dA - R0, KT, PW, projT, PW, (int)threadIdx.x, NTH);
    if (threadIdx.x < TWX) {
        const int64_t w = w0 + threadIdx.x;
        const bool ok = w < g.W;
        csq[threadIdx.x] = ok ? sc.sq[h * g.W + w] : 0.f;
        cmn[threadIdx.x] = ok ? sc.mean[h * g.W + w] : 0.f;
    }
    for (int e = threadIdx.x; e < NC; e += NTH) {
        const int64_t d = dA + e;
        const bool ok = d < g.W;
        psq[e] = ok ? sp.sq[h * g.W + d] : 0.f;
        pmn[e] = ok ? sp.mean[h * g.W + d] : 0.f;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wl = lane & 31, kh = lane >> 5;
    const int64_t dW = dA + (int64_t)(32 * NT) * wave;  // the wave's first projector column
    auto tile_live = [&](int64_t dt) {
        if (dt >= g.W || w0 >= g.WO) return false;
        if (g.layout == CUSTMA_LAYOUT_WINDOW) return dt - (w0 + TWX - 1) <= g.D && dt + 31 - w0 >= 0;
        return true;
    };
    bool any = false;
#pragma unroll
    for (int q = 0; q < NT; ++q) any |= tile_live(dW + 32 * q);
    if (!any) return;

    const float mc = cmn[wl];
    float mp[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q) mp[q] = pmn[32 * NT * wave + 32 * q + wl];
    // per-lane bases (floats): [0] the pair stays in one row, [1] it wraps to the next row
    const float* cb0 = camT + wl + kh;
    const float* cb1 = camT + wl + kh * (CW - KT + 1);
    const float* pb0 = projT + 32 * NT * wave + wl + kh;
    const float* pb1 = projT + 32 * NT * wave + wl + kh * (PW - KT + 1);

    f32x16 acc[NT];
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[q][e] = 0.f;

    // one MFMA step: taps (2 s', 2 s' + 1) of the block starting at tap row `row0` of the strips;
    // LAST: the tail row's step whose kh = 1 tap is past the patch (zero operand)
    // one MFMA step = taps (2 s, 2 s + 1) of the block whose first tap row the bases point at:
    // fetch() reads its raw operands, mma() centres them and issues the NT MFMAs; the block issues
    // step s + 1's reads before step s's MFMAs (LDS latency behind the MFMA pipe).  LAST: the tail
    // row's step whose kh = 1 tap lies past the patch (a zero operand).
    struct Ops {
        float a, b[NT];
    };
    auto fetch = [&](auto sc_, const float* c0, const float* c1, const float* p0, const float* p1) {
        constexpr int s = decltype(sc_)::value;
        constexpr int i0 = (2 * s) / KT, j0 = (2 * s) % KT;
        constexpr bool WRAP = (2 * s + 1) / KT != i0;
        constexpr int oc = i0 * CW + j0, op = i0 * PW + j0;
        Ops o;
        o.a = (WRAP ? c1 : c0)[oc];
#pragma unroll
        for (int q = 0; q < NT; ++q) o.b[q] = (WRAP ? p1 : p0)[op + 32 * q];
        return o;
    };
    auto mma = [&](const Ops& o, auto last_) {
        float a = o.a - mc;
        if constexpr (decltype(last_)::value) a = kh ? 0.f : a;
#pragma unroll
        for (int q = 0; q < NT; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, o.b[q] - mp[q], acc[q], 0, 0, 0);
    };
    // NS steps of a block, software-pipelined one step deep
    auto block = [&](auto ns_, auto tail_, const float* c0, const float* c1, const float* p0, const float* p1) {
        constexpr int NS = decltype(ns_)::value;
        constexpr bool TAIL = decltype(tail_)::value;
        Ops cur = fetch(std::integral_constant<int, 0>{}, c0, c1, p0, p1);
        Unroll<0, NS>::run([&](auto sc_) {
            constexpr int s = decltype(sc_)::value;
            Ops nxt = cur;
            if constexpr (s + 1 < NS) nxt = fetch(std::integral_constant<int, s + 1>{}, c0, c1, p0, p1);
            mma(cur, std::integral_constant<bool, TAIL && s + 1 == NS>{});
            cur = nxt;
            // keep the next step's reads ahead of this step's MFMAs: 1 MFMA, then the reads
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, NT + 1, 0);  // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, NT - 1, 0);  // MFMA
        });
    };
    // row pairs (2p, 2p + 1): KT steps each, the same pattern for every pair
    const float *c0 = cb0, *c1 = cb1, *p0 = pb0, *p1 = pb1;
#pragma unroll 1
    for (int p = 0; p < KT / 2; ++p) {
        block(std::integral_constant<int, KT>{}, std::false_type{}, c0, c1, p0, p1);
        c0 += 2 * CW; c1 += 2 * CW; p0 += 2 * PW; p1 += 2 * PW;
    }
    // the last row of an odd KT: (KT + 1) / 2 steps, the final kh = 1 tap empty
    if constexpr (KT % 2 == 1) block(std::integral_constant<int, (KT + 1) / 2>{}, std::true_type{}, c0, c1, p0, p1);

    // epilogue: cost = (E + eps) / sqrtf(fmaf(X, Y, eps))   (stereo_matching_kernel.cu:71)
#pragma unroll
    for (int q = 0; q < NT; ++q) {
        const int64_t dt = dW + 32 * q;
        if (!tile_live(dt)) continue;
        const int64_t d = dt + wl;
        const float Y = psq[32 * NT * wave + 32 * q + wl];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int wrow = (e & 3) + 8 * (e >> 2) + 4 * kh;
            const int64_t w = w0 + wrow;
            if (!voxel_valid(g, w, d)) continue;
            const float X = csq[wrow];
            const float den = sqrtf(__builtin_fmaf(X, Y, kEps));
            out[voxel_index(g, h, w, d)] = (acc[q][e] + kEps) / den;
        }
    }
}

template <typename T, int KT, int NW, int NT>
hipError_t launch_exact_k(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, float* out, hipStream_t s) {
    constexpr int NC = 32 * NW * NT;
    const int nWT = (int)cdiv(g.WO, TWX);
    const int nDC = (int)(g.layout == CUSTMA_LAYOUT_WINDOW ? cdiv(TWX + g.D, NC) : cdiv(g.W, NC));
    const int64_t blocks = g.HV() * nWT * nDC;
    const size_t lds = sizeof(float) * (KT * (TWX + KT - 1) + KT * (NC + KT - 1) + 2 * TWX + 2 * NC);
    hipError_t e = allow_lds(k_fwd_exact_k<T, KT, NW, NT>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_fwd_exact_k<T, KT, NW, NT>), dim3((unsigned)blocks), dim3(64 * NW), lds, s, cam, proj, g,
                       sc, sp, out, nWT, nDC);
    return hipGetLastError();
}

template <typename T, int KT>
hipError_t exact_k(const void* cam, const void* proj, const Geo& g, Stats sc, Stats sp, float* out, hipStream_t s) {
    if (g.layout == CUSTMA_LAYOUT_WINDOW)
        return launch_exact_k<T, KT, 3, 3>((const T*)cam, (const T*)proj, g, sc, sp, out, s);
    return launch_exact_k<T, KT, 4, 2>((const T*)cam, (const T*)proj, g, sc, sp, out, s);
}

template <int KT>
hipError_t exact_dispatch(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, float* out,
                          hipStream_t s) {
    if constexpr (KT > kExactMaxKT) {
        return hipErrorInvalidValue;
    } else {
        if (g.k == KT)
            return dtype == CUSTMA_F16 ? exact_k<__half, KT>(cam, proj, g, sc, sp, out, s)
                                       : exact_k<float, KT>(cam, proj, g, sc, sp, out, s);
        return exact_dispatch<KT + 1>(cam, proj, dtype, g, sc, sp, out, s);
    }
}
}  // namespace

hipError_t launch_fwd_exact(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            float* out, hipStream_t s) {
    if (g.k <= kExactMaxKT) return exact_dispatch<1>(cam, proj, dtype, g, sc, sp, out, s);
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
