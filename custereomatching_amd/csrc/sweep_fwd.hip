// Fast forward: sliding-window ZNCC over disparity diagonals.
//
// For a fixed offset delta = d - w, the reference's exy (custma/src/
// stereo_matching_kernel.cu:56-70) equals
//     E(h, w, delta) = sum_{patch} c * p  -  boxc(h,w) * boxp(h,w+delta) / k^2
// where the products c(y,x) * p(y,x+delta) of fp32 values are exact in fp64
// and the box sums slide: down the rows (one product row enters, one
// leaves) and across the columns (one column sum enters, one leaves).  All
// of that is fp64 (fp32 one-pass box sums cancel catastrophically on smooth
// images), so E is the exact-arithmetic value and differs from
// the reference's fp32 fma chain only by the reference's own rounding.  The
// denominator sqrtf(fmaf(ex2, ey2, eps)) uses the reference's own fp32
// ex2/ey2 (stats pass), so it is bit-identical.
//
// Lanes own disparity diagonals: lane l of a workgroup owns delta0 + l, so
// for a fixed camera column the lanes write consecutive projector columns
// (coalesced along the volume's fastest axis).  A workgroup owns TW = 16
// camera columns and walks a band of TH rows; per lane it keeps the
// TW + 2r column sums Col[] in registers (fp64).  Rows of both images are
// staged in a k-deep LDS ring, so each image element is read from HBM about
// once per band.  Per voxel: ~2(TW+2r)/TW fp64 FMAs for the row update,
// 2 fp64 adds for the column slide, and the fp32 finalisation.
//
// ARGMAX=true is the fused-disparity variant: instead of storing the volume
// it reduces, per camera pixel, (best, second best, first index of best) over
// the workgroup's diagonals and writes one partial per disparity chunk.
#include <float.h>

#include "common.h"
#include "sweep.h"

namespace custma {

namespace {

template <int K, typename T, bool ARGMAX>
__global__ __launch_bounds__(320) void k_sweep_fwd(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                   Stats sc, Stats sp, float* __restrict__ out, SweepGrid sg,
                                                   DispPartial part) {
    constexpr int R = K / 2, NX = TW + 2 * R;
    const int NL = sg.NL, NO = NX + NL - 1, NS = TW + NL - 1;
    extern __shared__ __attribute__((aligned(16))) double ldsd[];
    double* mO = ldsd;                         // [NS]  projector fp64 mean of row h
    double* bU = mO + NS;                      // [TW]  camera fp64 box sum of row h
    float* ringU = (float*)(bU + TW);          // [K][NX]
    float* ringO = ringU + K * NX;             // [K][NO]
    float* qO = ringO + K * NO;                // [NS]  projector ey2 (reference fp32)
    float* qU = qO + NS;                       // [TW]  camera ex2 (reference fp32)
    float* red = qU + TW;                      // [TW][NL] (ARGMAX only)

    int64_t bid = blockIdx.x;
    const int chunk = (int)(bid % sg.nChunk);
    bid /= sg.nChunk;
    const int wt = (int)(bid % sg.nTile);
    const int band = (int)(bid / sg.nTile);
    const int64_t u0 = (int64_t)wt * TW;
    const int64_t h0 = g.h_lo + (int64_t)band * sg.TH, h1 = min(g.h_hi, h0 + sg.TH);
    const int64_t dlo = g.layout == CUSTMA_LAYOUT_WINDOW ? 0 : -(u0 + TW - 1);
    const int64_t dhi = g.layout == CUSTMA_LAYOUT_WINDOW ? g.D : g.W - 1 - u0;
    const int64_t d0 = dlo + (int64_t)chunk * NL;
    const int tid = threadIdx.x;
    const int64_t delta = d0 + tid;
    const double rk2 = 1.0 / (double)(K * K);

    auto stage_row = [&](int64_t y) {
        const int slot = (int)(((y % K) + K) % K);
        for (int x = tid; x < NX; x += NL) ringU[slot * NX + x] = ldpad(cam, g.H, g.W, y, u0 - R + x);
        for (int x = tid; x < NO; x += NL) ringO[slot * NO + x] = ldpad(proj, g.H, g.W, y, u0 - R + d0 + x);
    };
    auto stage_stats = [&](int64_t h) {
        for (int n = tid; n < NS; n += NL) {
            const int64_t o = u0 + d0 + n;
            const bool ok = o >= 0 && o < g.W;
            mO[n] = ok ? sp.box[h * g.W + o] * rk2 : 0.0;
            qO[n] = ok ? sp.sq[h * g.W + o] : 0.f;
        }
        if (tid < TW) {
            const int64_t u = u0 + tid;
            const bool ok = u < g.W;
            bU[tid] = ok ? sc.box[h * g.W + u] : 0.0;
            qU[tid] = ok ? sc.sq[h * g.W + u] : 0.f;
        }
    };

    double col[NX];
#pragma unroll
    for (int x = 0; x < NX; ++x) col[x] = 0.0;

    auto accum_row = [&](int64_t y, double sgn) {
        const int slot = (int)(((y % K) + K) % K);
        const float* ru = ringU + slot * NX;
        const float* ro = ringO + slot * NO + tid;
#pragma unroll
        for (int x = 0; x < NX; ++x) col[x] = fma(sgn * (double)ru[x], (double)ro[x], col[x]);
    };

    // warm-up: rows h0-r .. h0+r-1
    for (int64_t y = h0 - R; y < h0 + R; ++y) stage_row(y);
    __syncthreads();
    for (int64_t y = h0 - R; y < h0 + R; ++y) accum_row(y, 1.0);

    const bool lane_live = delta >= dlo && delta <= dhi;
    for (int64_t h = h0; h < h1; ++h) {
        __syncthreads();  // previous step done with slot (h+R)%K and the stats
        stage_row(h + R);
        stage_stats(h);
        __syncthreads();
        accum_row(h + R, 1.0);

        double s = 0.0;
#pragma unroll
        for (int x = 0; x < 2 * R + 1; ++x) s += col[x];
#pragma unroll
        for (int m = 0; m < TW; ++m) {
            if (m > 0) s = (s + col[m + 2 * R]) - col[m - 1];
            const int64_t u = u0 + m, o = u + delta;
            const bool ok = lane_live && u < g.WO && o >= 0 && o < g.W;
            float c = -FLT_MAX;
            if (ok) {
                const double e = fma(-bU[m], mO[m + tid], s);
                const float num = (float)(e + (double)kEps);
                const float den = sqrtf(__builtin_fmaf(qU[m], qO[m + tid], kEps));
                c = num / den;
                if constexpr (!ARGMAX) {
                    const int64_t sidx = g.layout == CUSTMA_LAYOUT_WINDOW ? delta : o;
                    out[((h - g.h_lo) * g.WO + u) * g.DO + sidx] = c;
                }
            }
            if constexpr (ARGMAX) red[m * NL + tid] = c;
        }
        if constexpr (ARGMAX) {
            __syncthreads();
            // TPR threads per camera column (power of two), PER diagonals each, in order
            int TPR = 1;
            while (TPR * 2 * TW <= NL && TPR < 16) TPR *= 2;
            const int PER = (NL + TPR - 1) / TPR;
            const int m = tid / TPR, part_i = tid % TPR;
            const bool red_live = m < TW;
            float best = -FLT_MAX, second = -FLT_MAX;
            int bi = 0x7fffffff;
            for (int e = 0; red_live && e < PER; ++e) {
                const int l = part_i * PER + e;
                if (l >= NL) break;
                const float v = red[m * NL + l];
                if (v > best) { second = best; best = v; bi = l; }
                else if (v > second) second = v;
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                if (off >= TPR) break;
                const float ob = __shfl_xor(best, off), os = __shfl_xor(second, off);
                const int oi = __shfl_xor(bi, off);
                if (ob > best || (ob == best && oi < bi)) {
                    second = fmaxf(os, best); best = ob; bi = oi;
                } else {
                    second = fmaxf(second, ob);
                }
            }
            const int64_t u = u0 + m;
            if (red_live && part_i == 0 && u < g.WO) {
                const int64_t pidx = ((int64_t)chunk * g.HV() + (h - g.h_lo)) * g.WO + u;
                part.best[pidx] = best;
                part.second[pidx] = second;
                int64_t sidx = -1;
                if (best > -FLT_MAX) {
                    const int64_t dd = d0 + bi;
                    sidx = g.layout == CUSTMA_LAYOUT_WINDOW ? dd : u + dd;
                }
                part.index[pidx] = (int32_t)sidx;
            }
        }
        accum_row(h - R, -1.0);
    }
}

template <int K, typename T>
hipError_t launch_k(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, float* out,
                    DispPartial* part, hipStream_t s) {
    const SweepGrid sg = sweep_grid(g);
    constexpr int R = K / 2, NX = TW + 2 * R;
    const int NL = sg.NL, NO = NX + NL - 1, NS = TW + NL - 1;
    size_t lds = sizeof(double) * (NS + TW) + sizeof(float) * (K * NX + K * NO + NS + TW);
    const int64_t blocks = sweep_blocks(sg);
    if (part) {
        lds += sizeof(float) * TW * NL;
        hipLaunchKernelGGL((k_sweep_fwd<K, T, true>), dim3((unsigned)blocks), dim3(NL), lds, s, cam, proj, g, sc,
                           sp, out, sg, *part);
    } else {
        DispPartial none{};
        hipLaunchKernelGGL((k_sweep_fwd<K, T, false>), dim3((unsigned)blocks), dim3(NL), lds, s, cam, proj, g, sc,
                           sp, out, sg, none);
    }
    return hipGetLastError();
}

template <typename T>
hipError_t dispatch(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, float* out, DispPartial* part,
                    hipStream_t s) {
    switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: return launch_k<KK, T>(cam, proj, g, sc, sp, out, part, s);
        CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_fwd_fast(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                           float* out, hipStream_t s) {
    if (dtype == CUSTMA_F16)
        return dispatch((const __half*)cam, (const __half*)proj, g, sc, sp, out, nullptr, s);
    return dispatch((const float*)cam, (const float*)proj, g, sc, sp, out, nullptr, s);
}

hipError_t launch_disp_partials(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                                DispPartial part, hipStream_t s) {
    if (dtype == CUSTMA_F16)
        return dispatch((const __half*)cam, (const __half*)proj, g, sc, sp, nullptr, &part, s);
    return dispatch((const float*)cam, (const float*)proj, g, sc, sp, nullptr, &part, s);
}

}  // namespace custma
