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
// denominator uses the reference's own fp32 ex2/ey2 (stats pass); the
// finalisation is (E + eps) * rsqrt(fmaf(ex2, ey2, eps)) in fp32 (<= 3 ulp).
//
// Lanes own disparity diagonals: lane l of a workgroup owns delta0 + l, so
// for a fixed camera column the lanes write consecutive projector columns
// (256 contiguous bytes per wave store, along the volume's fastest axis).  A
// workgroup owns TW = 16 camera columns and walks a band of TH rows; per lane
// it keeps the TW + 2r column sums col[] in registers (fp64).  Image rows are
// staged (as fp64) in a (k+1)-deep LDS ring and the per-row statistics in a
// double buffer: the next row's global loads are issued before the current
// row's arithmetic and land in LDS after it, so there is ONE barrier per
// row and the load latency hides under the compute.  Block order is
// XCD-aware: the disparity chunks of one column tile (which write adjacent
// pieces of the same volume rows) run on the same XCD and share its L2.
//
// Per voxel: 2(TW+2r)/TW fp64 FMAs (row update), 2 fp64 adds (column
// slide), 1 fp64 FMA + cvt (E), ~4 fp32 ops incl. one v_rsq (finalise).
//
// ARGMAX=true is the fused-disparity variant: instead of storing the volume
// it reduces, per camera pixel, (best, second best, first index of best) over
// the workgroup's diagonals and writes one partial per disparity chunk.
#include <float.h>

#include <type_traits>

#include "common.h"
#include "sweep.h"

namespace custma {

namespace {

// acc += bcast(a, lane L of each 16-lane row) * b, one instruction (DPP row_newbcast on
// gfx950's fp64 / fp32 FMAC).  Uniform per-step operands (camera pixels, the camera
// column's patch sum and moment) are held row-replicated in one VGPR (lane i has
// element i & 15) instead of being re-read from LDS for every product.
template <int L>
__device__ __forceinline__ void fmac_bc64(double& acc, double a, double b) {
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b), "i"(L));
}
template <int L>
__device__ __forceinline__ void fmac_bc32(float& acc, float a, float b) {
    asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(a), "v"(b), "i"(L));
}
template <int X, int NX>
struct Unroll {
    template <typename F>
    __device__ __forceinline__ static void run(F&& f) {
        f(std::integral_constant<int, X>{});
        Unroll<X + 1, NX>::run(f);
    }
};
template <int NX>
struct Unroll<NX, NX> {
    template <typename F>
    __device__ __forceinline__ static void run(F&&) {}
};

template <int K, int TWT, typename T, bool ARGMAX>
__global__ __launch_bounds__(320, 2) void k_sweep_fwd(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                      Stats sc, Stats sp, float* __restrict__ out, SweepGrid sg,
                                                      DispPartial part) {
    constexpr int R = K / 2, NX = TWT + 2 * R, NSLOT = K + 2;
    static_assert(TWT == 16 && NX <= 32, "row-broadcast layout assumes 16 own columns and <= 32 taps");
    const int NL = sg.NL, NO = NX + NL - 1, NS = TWT + NL - 1;
    extern __shared__ __attribute__((aligned(16))) double ldsd[];
    double* rsM = ldsd;                         // [2][NS]  projector fp64 patch means
    double* usB = rsM + 2 * NS;                 // [2][16]  -(camera fp64 patch sums)
    double* ringU = usB + 2 * 16;               // [NSLOT][2][32]  +c, -c of a camera row
    double* ringO = ringU + NSLOT * 64;         // [NSLOT][NO] projector row
    float* rsQ = (float*)(ringO + NSLOT * NO);  // [2][NS]  projector ey2
    float* usQ = rsQ + 2 * NS;                  // [2][16]  camera ex2
    float* red = usQ + 2 * 16;                  // [TWT][NL] (ARGMAX only)

    const int64_t bid = xcd_remap(blockIdx.x, gridDim.x);
    const int chunk = (int)(bid % sg.nChunk);
    const int64_t rest = bid / sg.nChunk;
    const int wt = (int)(rest % sg.nTile);
    const int band = (int)(rest / sg.nTile);
    const int64_t u0 = (int64_t)wt * TWT;
    const int64_t h0 = g.h_lo + (int64_t)band * sg.TH, h1 = min(g.h_hi, h0 + sg.TH);
    const int64_t dlo = g.layout == CUSTMA_LAYOUT_WINDOW ? 0 : -(u0 + TWT - 1);
    const int64_t dhi = g.layout == CUSTMA_LAYOUT_WINDOW ? g.D : g.W - 1 - u0;
    const int64_t d0 = dlo + (int64_t)chunk * NL;
    const int tid = threadIdx.x;
    const int64_t delta = d0 + tid;
    const double rk2 = 1.0 / (double)(K * K);

    // valid camera-column offsets m in [m_lo, m_hi) for this lane's diagonal
    int m_lo = TWT, m_hi = 0;
    if (delta >= dlo && delta <= dhi) {
        const int64_t lo = max((int64_t)0, -delta - u0);
        const int64_t hi = min((int64_t)TWT, min(g.W - u0 - delta, g.WO - u0));
        m_lo = (int)lo;
        m_hi = (int)max(lo, hi);
    }

    // ---- staging: branch-free raw buffer loads (out-of-range -> 0 = the reference's
    // zero padding, stereo_matching_kernel.cu:6-12); every lane issues every load, so
    // the compiler counts outstanding memory operations exactly and never drains the
    // volume stores (vmcnt(0)) to consume a prefetch ----
    // per-lane byte offsets inside one row (loop-invariant); the row is the descriptor's base,
    // and a row outside the image gets a zero-size descriptor (every load returns 0)
    const int64_t xU0 = u0 - R, xO0 = u0 - R + d0, oS = u0 + d0;
    constexpr uint32_t OOB = 0x80000000u;
    auto colOff = [&](bool have, int64_t x, int esz) -> uint32_t {
        return (have && x >= 0 && x < g.W) ? (uint32_t)(x * esz) : OOB;
    };
    const uint32_t vU = colOff(tid < NX, xU0 + tid, sizeof(T));
    const uint32_t vO0 = colOff(true, xO0 + tid, sizeof(T));
    const uint32_t vO1 = colOff(tid + NL < NO, xO0 + tid + NL, sizeof(T));
    const uint32_t vS0d = colOff(true, oS + tid, 8), vS0f = colOff(true, oS + tid, 4);
    const uint32_t vS1d = colOff(tid + NL < NS, oS + tid + NL, 8), vS1f = colOff(tid + NL < NS, oS + tid + NL, 4);
    const uint32_t vUSd = colOff(tid < TWT, u0 + tid, 8), vUSf = colOff(tid < TWT, u0 + tid, 4);
    auto row_rsrc = [&](const void* base, int64_t row, int esz) {
        const bool ok = row >= 0 && row < g.H;
        return make_rsrc((const char*)base + (ok ? row : 0) * g.W * esz, ok ? (uint32_t)(g.W * esz) : 0u);
    };
    struct Pre {
        float u, o0, o1, q0, q1, uq;
        double m0, m1, ub;
    };
    auto load_row = [&](int64_t y, Pre& p) {
        const auto rC = row_rsrc(cam, y, sizeof(T));
        const auto rP = row_rsrc(proj, y, sizeof(T));
        p.u = ld_buf<T>(rC, vU);
        p.o0 = ld_buf<T>(rP, vO0);
        p.o1 = ld_buf<T>(rP, vO1);
    };
    auto load_stats = [&](int64_t h, Pre& p) {
        const auto rPB = row_rsrc(sp.box, h, 8), rPS = row_rsrc(sp.sq, h, 4);
        const auto rCB = row_rsrc(sc.box, h, 8), rCS = row_rsrc(sc.sq, h, 4);
        p.m0 = ld_buf_f64(rPB, vS0d) * rk2;
        p.q0 = ld_buf<float>(rPS, vS0f);
        p.m1 = ld_buf_f64(rPB, vS1d) * rk2;
        p.q1 = ld_buf<float>(rPS, vS1f);
        p.ub = ld_buf_f64(rCB, vUSd);
        p.uq = ld_buf<float>(rCS, vUSf);
    };
    auto store_row = [&](int slot, const Pre& p) {
        if (tid < 32) {
            ringU[slot * 64 + tid] = (double)p.u;        // p.u is 0 for tid >= NX
            ringU[slot * 64 + 32 + tid] = -(double)p.u;
        }
        ringO[slot * NO + tid] = (double)p.o0;
        if (tid + NL < NO) ringO[slot * NO + tid + NL] = (double)p.o1;
    };
    auto store_stats = [&](int b, const Pre& p) {
        rsM[b * NS + tid] = p.m0;
        rsQ[b * NS + tid] = p.q0;
        if (tid + NL < NS) { rsM[b * NS + tid + NL] = p.m1; rsQ[b * NS + tid + NL] = p.q1; }
        if (tid < 16) { usB[b * 16 + tid] = -p.ub; usQ[b * 16 + tid] = p.uq; }
    };

    double col[NX];
#pragma unroll
    for (int x = 0; x < NX; ++x) col[x] = 0.0;
    const int r16 = tid & 15;
    // col[x] += c(row sAdd, x) p(row sAdd, x + delta) - c(row sSub, x) p(row sSub, x + delta).
    // Operands are loaded in batches of 8 columns ahead of the DPP FMAs (an asm statement
    // is a scheduling boundary, so loads are not hoisted across it by the compiler).
    auto update = [&](int sAdd, int sSub) {
        const double ca0 = ringU[sAdd * 64 + r16], ca1 = ringU[sAdd * 64 + 16 + r16];
        const double cb0 = ringU[sSub * 64 + 32 + r16], cb1 = ringU[sSub * 64 + 48 + r16];  // negated
        const double* oa = ringO + sAdd * NO + tid;
        const double* ob = ringO + sSub * NO + tid;
        constexpr int B = 8;
        Unroll<0, (NX + B - 1) / B>::run([&](auto bc) {
            constexpr int x0 = decltype(bc)::value * B;
            constexpr int nb = NX - x0 < B ? NX - x0 : B;
            double pa[B], pb[B];
            Unroll<0, nb>::run([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                pa[i] = oa[x0 + i];
                pb[i] = ob[x0 + i];
            });
            Unroll<0, nb>::run([&](auto ic) {
                constexpr int i = decltype(ic)::value, x = x0 + i;
                fmac_bc64<(x & 15)>(col[x], x < 16 ? ca0 : ca1, pa[i]);
                fmac_bc64<(x & 15)>(col[x], x < 16 ? cb0 : cb1, pb[i]);
            });
        });
    };
    // first-step "leaving" row: slot NSLOT-1, all zeros
    for (int e = tid; e < 64; e += NL) ringU[(NSLOT - 1) * 64 + e] = 0.0;
    for (int e = tid; e < NO; e += NL) ringO[(NSLOT - 1) * NO + e] = 0.0;

    // ring slot of image row y: (y - (h0 - R)) mod NSLOT, tracked incrementally
    {
        Pre p;
        for (int i = 0; i < K - 1; ++i) {
            load_row(h0 - R + i, p);
            store_row(i, p);
        }
        load_stats(h0, p);
        store_stats(0, p);
    }
    __syncthreads();
#pragma unroll 1
    for (int i = 0; i < K - 1; ++i) update(i, NSLOT - 1);
    int sIn = K - 1, sOut = NSLOT - 1;  // row h+R / row h-R-1 at step h
    {
        Pre p;
        load_row(h0 + R, p);
        store_row(sIn, p);
    }
    __syncthreads();

    // volume stores: per step one descriptor at the first volume element of the tile's
    // rows; per lane byte offset m*stride + column (out-of-range for invalid voxels)
    const int64_t stride = g.layout == CUSTMA_LAYOUT_WINDOW ? g.DO : g.DO + 1;
    const int64_t lane0 = g.layout == CUSTMA_LAYOUT_WINDOW ? delta : u0 + delta;  // column index at m = 0
    const int64_t orow = g.WO * g.DO;
    uint32_t voff[TWT];
#pragma unroll
    for (int m = 0; m < TWT; ++m)
        voff[m] = (m >= m_lo && m < m_hi) ? (uint32_t)((m * stride + lane0) * 4) : 0x80000000u;
    float* obase = out + ((h0 - g.h_lo) * g.WO + u0) * g.DO;

    for (int64_t h = h0; h < h1; ++h) {
        const int buf = (int)((h - h0) & 1);
        Pre p;  // next row (harmless loads past the band's end: results unused)
        load_row(h + R + 1, p);
        load_stats(h + 1, p);
        update(sIn, sOut);

        double s = 0.0;
#pragma unroll
        for (int x = 0; x < 2 * R + 1; ++x) s += col[x];
        const double* mrow = rsM + buf * NS + tid;
        const float* qrow = rsQ + buf * NS + tid;
        const double nb = usB[buf * 16 + r16];  // -(camera patch sum) of column r16
        const float uq = usQ[buf * 16 + r16];   // camera ex2 of column r16
        double mv[TWT];
        float qv[TWT];
#pragma unroll
        for (int m = 0; m < TWT; ++m) { mv[m] = mrow[m]; qv[m] = qrow[m]; }
        const auto rOut = make_rsrc(ARGMAX ? (float*)nullptr : obase, 0x7FFFFFF0u);
        Unroll<0, TWT>::run([&](auto mc) {
            constexpr int m = decltype(mc)::value;
            if (m > 0) s = (s + col[m + 2 * R]) - col[m - 1];
            double e = s;
            fmac_bc64<m>(e, nb, mv[m]);                 // E = S - box_c * mean_p
            float den2 = kEps;
            fmac_bc32<m>(den2, uq, qv[m]);              // ex2 * ey2 + eps
            const float num = (float)e + kEps;
            const float c = num * __builtin_amdgcn_rsqf(den2);
            if constexpr (ARGMAX) {
                red[m * NL + tid] = (m >= m_lo && m < m_hi) ? c : -FLT_MAX;
            } else {
                st_buf(c, rOut, voff[m]);
            }
        });
        if constexpr (!ARGMAX) obase += orow;
        if constexpr (ARGMAX) {
            __syncthreads();
            // TPR threads per camera column (power of two), PER diagonals each, in order
            int TPR = 1;
            while (TPR * 2 * TWT <= NL && TPR < 16) TPR *= 2;
            const int PER = (NL + TPR - 1) / TPR;
            const int m = tid / TPR, part_i = tid % TPR;
            const bool red_live = m < TWT;
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
        // next step: row h+R+1 enters (into the slot after sIn), row h-R leaves
        sOut = sIn + 1 - K >= 0 ? sIn + 1 - K : sIn + 3;  // slot of row h-R = (sIn - 2R) mod (K+2)
        sIn = sIn + 1 == NSLOT ? 0 : sIn + 1;
        store_row(sIn, p);
        store_stats(buf ^ 1, p);
        __syncthreads();
    }
}

template <int K, typename T>
hipError_t launch_k(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, float* out,
                    DispPartial* part, hipStream_t s) {
    const SweepGrid sg = sweep_grid(g);
    constexpr int R = K / 2, NX = TW + 2 * R, NSLOT = K + 2;
    const int NL = sg.NL, NO = NX + NL - 1, NS = TW + NL - 1;
    size_t lds = sizeof(double) * (2 * NS + 2 * 16 + NSLOT * 64 + NSLOT * NO) + sizeof(float) * (2 * NS + 2 * 16);
    const int64_t blocks = sweep_blocks(sg);
    if (part) {
        lds += sizeof(float) * TW * NL;
        hipLaunchKernelGGL((k_sweep_fwd<K, TW, T, true>), dim3((unsigned)blocks), dim3(NL), lds, s, cam, proj, g,
                           sc, sp, out, sg, *part);
    } else {
        DispPartial none{};
        hipLaunchKernelGGL((k_sweep_fwd<K, TW, T, false>), dim3((unsigned)blocks), dim3(NL), lds, s, cam, proj, g,
                           sc, sp, out, sg, none);
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
