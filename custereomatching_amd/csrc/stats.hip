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
#include "stats_body.h"
#include "sweep.h"

namespace custma {

namespace {
using namespace stats_detail;

template <typename T, int KT, int MODE>
__global__ __launch_bounds__(256) void k_stats(const T* __restrict__ img0, const T* __restrict__ img1, Geo g,
                                               Stats st0, Stats st1, float* __restrict__ prep,
                                               const float* __restrict__ shift, int64_t ybeg, int64_t yend) {
    extern __shared__ __attribute__((aligned(16))) double lds_d[];
    stats_tile<T, KT, MODE>(img0, img1, g, st0, st1, prep, shift, ybeg, yend, (int)blockIdx.x, (int)blockIdx.y,
                            (int)blockIdx.z, lds_d);
}
}  // namespace

hipError_t launch_stats(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, hipStream_t s,
                        int mode, float* prep, const float* shift, int rows) {
    const int64_t ybeg = rows == STATS_BAND_ROWS ? g.h_lo : 0, yend = rows == STATS_BAND_ROWS ? g.h_hi : g.H;
    if (yend <= ybeg || g.W == 0) return hipSuccess;
    const int TY = ty_for(mode);
    const dim3 grid((unsigned)cdiv(g.W, TX), (unsigned)cdiv(yend - ybeg, TY), 2);
    const int LX = lx_for(g.k), LY = TY + g.k - 1;
    const size_t lds =
        sizeof(double) * (mode == STATS_FWD || mode == STATS_MSB ? 1 : 2) * LY * TX + sizeof(float) * LY * LX;
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
