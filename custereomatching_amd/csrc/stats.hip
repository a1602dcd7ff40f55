// Per-pixel patch statistics (one pass over each image, tiny next to the volume).
//
// mean, sq: the reference's own fp32 values -- the sequential (i, j) sum / k^2 and the
//   fma chain of centred squares that every reference thread recomputes for its patch
//   (custma/src/stereo_matching_kernel.cu:40-54 mean, :56-69 centred squares) -- so
//   hoisting them per pixel is bit-identical.  This k^2-long dependent chain is the
//   kernel's cost; it runs from an LDS tile, each thread feeding 4 vertically adjacent
//   pixels from one read of every tile value.
// box: fp64 patch sum, exact for fp32 inputs within a 2^29 dynamic range, so its value
//   does not depend on the summation order; formed separably (k-tap row sums in LDS,
//   then k column taps), 2k fp64 adds per pixel instead of k^2.
// sqt: fp64-accurate centred second moment box2 - box^2 / k^2 (separable too), rounded
//   to fp32; only the backward reads it.
#include <type_traits>

#include "common.h"
#include "sweep.h"

namespace custma {

namespace {
#ifndef CUSTMA_STATS_TX
#define CUSTMA_STATS_TX 32  // 16 -> 32 (128-byte rows per store): C5 forward stats 0.77 -> 0.72 ms, backward 0.60 -> 0.51 ms (profiles/r03/stats)
#endif
#ifndef CUSTMA_STATS_PR
#define CUSTMA_STATS_PR 4
#endif
// TX x TY pixels per 256-thread workgroup, PR rows per thread (a tap row read from LDS feeds PR pixels)
constexpr int TX = CUSTMA_STATS_TX, PR = CUSTMA_STATS_PR, TY = 256 / TX * PR;
static_assert(PR % 2 == 0, "pixel pairs");
typedef float f32x2 __attribute__((ext_vector_type(2)));

// KT > 0: the window size as a compile-time constant (the sweep's instantiations), so the
// k^2 tap loops unroll and the per-pixel row masks fold away; KT = 0: runtime k.
// MODE (StatsMode): which outputs are written.
//   STATS_FULL      mean, sq, box, sqt
//   STATS_BOX       box, sqt                  (the generic backward's statistics)
//   STATS_BWD_PREP  box and the fused sweep's prepared fp32 images (bwd_fused.hip k_bwd_sweep's
//                   X = sqt, m' = box / k^2 - shift, raw image; image z at prep + 3 z planes)
//   STATS_FWD       sq, box                   (what the fast forward sweeps read)
//   STATS_MSB       mean, sq, box             (the disparity: its sweep reads sq, box, its exact
//                                              recheck mean, sq; the exact forward reads mean, sq)
template <typename T, int KT, int MODE>
__global__ __launch_bounds__(256) void k_stats(const T* __restrict__ img0, const T* __restrict__ img1, Geo g,
                                               Stats st0, Stats st1, float* __restrict__ prep,
                                               const float* __restrict__ shift, int64_t ybeg, int64_t yend) {
    constexpr bool BOX_ONLY = MODE == STATS_BOX || MODE == STATS_BWD_PREP;
    constexpr bool SQT = MODE != STATS_FWD && MODE != STATS_MSB;  // the fp64 sums of squares only feed sqt
    // blockIdx.z: 0 = camera, 1 = projector (one launch for both images)
    const T* __restrict__ img = blockIdx.z ? img1 : img0;
    const Stats st = blockIdx.z ? st1 : st0;
    extern __shared__ __attribute__((aligned(16))) double lds_d[];
    const int k = KT > 0 ? KT : g.k, r = k / 2, LX = TX + 2 * r, LY = TY + 2 * r;
    double* rs = lds_d;                    // [LY][TX] fp64 k-tap row sums
    double* rs2 = rs + LY * TX;            // [LY][TX] fp64 k-tap row sums of squares
    float* tile = (float*)(rs2 + LY * TX);  // [LY][LX] zero-padded image tile
    // pixel rows [ybeg, yend) (STATS_BAND_ROWS: the volume rows only)
    const int64_t y0 = ybeg + (int64_t)blockIdx.y * TY, x0 = (int64_t)blockIdx.x * TX;
    for (int e = threadIdx.x; e < LY * LX; e += 256) {
        const int ty = e / LX, tx = e % LX;
        tile[e] = ldpad(img, g.H, g.W, y0 + ty - r, x0 + tx - r);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < LY * TX; e += 256) {
        const int ty = e / TX, tx = e % TX;
        const float* t = tile + ty * LX + tx;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int j = 0; j < k; ++j) {
            const double v = (double)t[j];
            a += v;
            if constexpr (SQT) b = fma(v, v, b);
        }
        rs[e] = a;
        if constexpr (SQT) rs2[e] = b;
    }
    __syncthreads();
    const int lx = threadIdx.x % TX, q = threadIdx.x / TX;  // rows PR q .. PR q + PR-1
    if constexpr (BOX_ONLY) {
        const int64_t x = x0 + lx;
        if (x >= g.W) return;
#pragma unroll
        for (int p = 0; p < PR; ++p) {
            const int ly = PR * q + p;
            const int64_t y = y0 + ly;
            if (y >= yend) break;
            double b = 0.0, b2 = 0.0;
#pragma unroll
            for (int i = 0; i < k; ++i) {
                b += rs[(ly + i) * TX + lx];
                b2 += rs2[(ly + i) * TX + lx];
            }
            const int64_t o = y * g.W + x;
            st.box[o] = b;
            const double c2 = b2 - b * b / (double)(k * k);
            const float sqt = (float)(c2 > 0.0 ? c2 : 0.0);
            if constexpr (MODE == STATS_BWD_PREP) {
                const int64_t n = g.H * g.W;
                float* pz = prep + 3 * n * blockIdx.z;
                pz[o] = sqt;
                pz[n + o] = (float)(b / (double)(k * k) - (double)shift[blockIdx.z]);
                pz[2 * n + o] = tile[(ly + r) * LX + lx + r];  // raw: the sweep subtracts the shift after a zero-padded load
            } else {
                st.sqt[o] = sqt;
            }
        }
        return;
    }
    // Each tile value is read once per pass and fed to the PR pixels whose patch holds it;
    // per pixel the taps still arrive in the reference's (i, j) row-major order.
    const float* t = tile + (PR * q) * LX + lx;
    float m[PR], sq[PR];
#pragma unroll
    for (int p = 0; p < PR; ++p) { m[p] = 0.f; sq[p] = 0.f; }
    // Tile rows one at a time (not unrolled: fully unrolled, the compiler keeps all
    // (k+PR-1) k tile values live across both passes -- 182 VGPRs, 2 waves per SIMD); the
    // row's k values feed every pixel whose patch holds that row (a wave-uniform branch).
#pragma unroll 1
    for (int i2 = 0; i2 < k + PR - 1; ++i2) {
        float v[KT > 0 ? KT : 1];
        if constexpr (KT > 0) {
#pragma unroll
            for (int j = 0; j < KT; ++j) v[j] = t[i2 * LX + j];
            if (i2 >= PR - 1 && i2 < k) {  // the row is in all PR patches: pixel pairs in packed fp32 adds
#pragma unroll
                for (int pp = 0; pp < PR / 2; ++pp) {
                    f32x2 a = {m[2 * pp], m[2 * pp + 1]};
#pragma unroll
                    for (int j = 0; j < KT; ++j) a = a + f32x2{v[j], v[j]};
                    m[2 * pp] = a.x;
                    m[2 * pp + 1] = a.y;
                }
            } else {
#pragma unroll
                for (int p = 0; p < PR; ++p)
                    if (i2 - p >= 0 && i2 - p < k) {
#pragma unroll
                        for (int j = 0; j < KT; ++j) m[p] = m[p] + v[j];
                    }
            }
        } else {
            for (int j = 0; j < k; ++j) {
                const float u = t[i2 * LX + j];
#pragma unroll
                for (int p = 0; p < PR; ++p)
                    if (i2 - p >= 0 && i2 - p < k) m[p] = m[p] + u;
            }
        }
    }
#pragma unroll
    for (int p = 0; p < PR; ++p) m[p] = m[p] / (float)(k * k);
#pragma unroll 1
    for (int i2 = 0; i2 < k + PR - 1; ++i2) {
        float v[KT > 0 ? KT : 1];
        if constexpr (KT > 0) {
#pragma unroll
            for (int j = 0; j < KT; ++j) v[j] = t[i2 * LX + j];
            if (i2 >= PR - 1 && i2 < k) {  // packed: v_pk_add_f32 / v_pk_fma_f32, the same IEEE ops per lane half
#pragma unroll
                for (int pp = 0; pp < PR / 2; ++pp) {
                    const f32x2 mm = {m[2 * pp], m[2 * pp + 1]};
                    f32x2 a = {sq[2 * pp], sq[2 * pp + 1]};
#pragma unroll
                    for (int j = 0; j < KT; ++j) {
                        const f32x2 c = f32x2{v[j], v[j]} - mm;
                        a = __builtin_elementwise_fma(c, c, a);
                    }
                    sq[2 * pp] = a.x;
                    sq[2 * pp + 1] = a.y;
                }
            } else {
#pragma unroll
                for (int p = 0; p < PR; ++p)
                    if (i2 - p >= 0 && i2 - p < k) {
#pragma unroll
                        for (int j = 0; j < KT; ++j) {
                            const float c = v[j] - m[p];
                            sq[p] = __builtin_fmaf(c, c, sq[p]);
                        }
                    }
            }
        } else {
            for (int j = 0; j < k; ++j) {
                const float u = t[i2 * LX + j];
#pragma unroll
                for (int p = 0; p < PR; ++p)
                    if (i2 - p >= 0 && i2 - p < k) {
                        const float c = u - m[p];
                        sq[p] = __builtin_fmaf(c, c, sq[p]);
                    }
            }
        }
    }
    const int64_t x = x0 + lx;
    if (x >= g.W) return;
#pragma unroll
    for (int p = 0; p < PR; ++p) {
        const int ly = PR * q + p;
        const int64_t y = y0 + ly;
        if (y >= yend) break;
        double b = 0.0, b2 = 0.0;
#pragma unroll
        for (int i = 0; i < k; ++i) {
            b += rs[(ly + i) * TX + lx];
            if constexpr (SQT) b2 += rs2[(ly + i) * TX + lx];
        }
        const int64_t o = y * g.W + x;
        if constexpr (MODE == STATS_FULL || MODE == STATS_MSB) st.mean[o] = m[p];
        st.sq[o] = sq[p];
        st.box[o] = b;
        if constexpr (MODE == STATS_FULL) {
            const double c2 = b2 - b * b / (double)(k * k);
            st.sqt[o] = (float)(c2 > 0.0 ? c2 : 0.0);
        }
    }
}
}  // namespace

hipError_t launch_stats(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, hipStream_t s,
                        int mode, float* prep, const float* shift, int rows) {
    const int64_t ybeg = rows == STATS_BAND_ROWS ? g.h_lo : 0, yend = rows == STATS_BAND_ROWS ? g.h_hi : g.H;
    if (yend <= ybeg || g.W == 0) return hipSuccess;
    const dim3 grid((unsigned)cdiv(g.W, TX), (unsigned)cdiv(yend - ybeg, TY), 2);
    const int LX = TX + 2 * g.r, LY = TY + 2 * g.r;
    const size_t lds = sizeof(double) * 2 * LY * TX + sizeof(float) * LY * LX;
    hipError_t err = hipSuccess;
    auto go = [&](auto kc) {
        constexpr int KT = decltype(kc)::value;
        auto launch = [&](auto* cast, auto mc) {
            using T = std::remove_const_t<std::remove_pointer_t<decltype(cast)>>;
            constexpr int M = decltype(mc)::value;
            if ((err = allow_lds(k_stats<T, KT, M>, lds)) != hipSuccess) return;
            hipLaunchKernelGGL((k_stats<T, KT, M>), grid, dim3(256), lds, s, (const T*)cam, (const T*)proj, g, sc, sp,
                               prep, shift, ybeg, yend);
        };
        auto by_mode = [&](auto* cast) {
            switch (mode) {
                case STATS_BOX: launch(cast, std::integral_constant<int, STATS_BOX>{}); break;
                case STATS_BWD_PREP: launch(cast, std::integral_constant<int, STATS_BWD_PREP>{}); break;
                case STATS_FWD: launch(cast, std::integral_constant<int, STATS_FWD>{}); break;
                case STATS_MSB: launch(cast, std::integral_constant<int, STATS_MSB>{}); break;
                default: launch(cast, std::integral_constant<int, STATS_FULL>{});
            }
        };
        if (dtype == CUSTMA_F16) by_mode((const __half*)nullptr);
        else by_mode((const float*)nullptr);
    };
    switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: go(std::integral_constant<int, KK>{}); break;
        CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
        default: go(std::integral_constant<int, 0>{});
    }
    return err != hipSuccess ? err : hipGetLastError();
}

}  // namespace custma
