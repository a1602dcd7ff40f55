// Shared geometry of the sliding-window ("sweep") kernels.
#pragma once
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace custma {

// Compile-time loop: f(std::integral_constant<int, X>) for X in [X0, NX).
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

constexpr int TW = 16;  // camera (own-image) columns per workgroup

// acc += bcast(a, lane L of each 16-lane row) * b, one instruction (DPP row_newbcast on
// gfx950's fp64 / fp32 FMAC).  Uniform per-step operands (camera pixels, the camera
// column's patch sum and moment) are held row-replicated in one VGPR (lane i has
// element i & 15) instead of being re-read from LDS for every product.
//
// Hazard: a DPP source VGPR written by a VALU instruction needs 2 wait states before the
// DPP read (gfx9 "VALU write VGPR -> DPP read").  The compiler cannot see the DPP inside
// the asm, so with NOP = true every asm block below starts with `s_nop 1`.  NOP = false
// drops it where the operands are step constants; custereomatching_amd/hazard_check.py
// verifies the emitted listing of such translation units at build time (rule R2).
#define CUSTMA_DPP_ASM(NOP, BODY, ...)                      \
    do {                                                    \
        if constexpr (NOP)                                  \
            asm("s_nop 1\n\t" BODY __VA_ARGS__);            \
        else                                                \
            asm(BODY __VA_ARGS__);                          \
    } while (0)
template <int L, bool NOP = true>
__device__ __forceinline__ void fmac_bc64(double& acc, double a, double b) {
    CUSTMA_DPP_ASM(NOP, "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf",
                   : "+v"(acc) : "v"(a), "v"(b), "i"(L));
}
template <int L, bool NOP = true>
__device__ __forceinline__ void fmac_bc32(float& acc, float a, float b) {
    CUSTMA_DPP_ASM(NOP, "v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf",
                   : "+v"(acc) : "v"(a), "v"(b), "i"(L));
}
// acc[i] += bcast(a, lane L+i) * pa[i] + bcast(b, lane L+i) * pb[i] for i < 4 (in that order)
template <int L, bool NOP = true>
__device__ __forceinline__ void fmac2_bc64_x4(double& c0, double& c1, double& c2, double& c3, double a, double b,
                                              double pa0, double pa1, double pa2, double pa3, double pb0,
                                              double pb1, double pb2, double pb3) {
    CUSTMA_DPP_ASM(NOP,
                   "v_fmac_f64_dpp %0, %4, %6 row_newbcast:%14 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %1, %4, %7 row_newbcast:%15 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %2, %4, %8 row_newbcast:%16 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %3, %4, %9 row_newbcast:%17 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %0, %5, %10 row_newbcast:%14 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %1, %5, %11 row_newbcast:%15 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %2, %5, %12 row_newbcast:%16 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %3, %5, %13 row_newbcast:%17 row_mask:0xf bank_mask:0xf",
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
                   : "v"(a), "v"(b), "v"(pa0), "v"(pa1), "v"(pa2), "v"(pa3), "v"(pb0), "v"(pb1), "v"(pb2),
                     "v"(pb3), "i"(L), "i"(L + 1), "i"(L + 2), "i"(L + 3));
}
template <int L, bool NOP = true>
__device__ __forceinline__ void fmac2_bc64_x2(double& c0, double& c1, double a, double b, double pa0, double pa1,
                                              double pb0, double pb1) {
    CUSTMA_DPP_ASM(NOP,
                   "v_fmac_f64_dpp %0, %2, %4 row_newbcast:%8 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %1, %2, %5 row_newbcast:%9 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %0, %3, %6 row_newbcast:%8 row_mask:0xf bank_mask:0xf\n\t"
                   "v_fmac_f64_dpp %1, %3, %7 row_newbcast:%9 row_mask:0xf bank_mask:0xf",
                   : "+v"(c0), "+v"(c1)
                   : "v"(a), "v"(b), "v"(pa0), "v"(pa1), "v"(pb0), "v"(pb1), "i"(L), "i"(L + 1));
}
// e = s + bcast(nb, lane L) * mv;  den2 = eps + bcast(uq, lane L) * qv  (the finalisation's
// two DPP FMAs).  The two initialising moves go first inside the asm: they are the 2 wait
// states a DPP source written by the previous VALU op needs, so no `s_nop` is spent.
template <int L>
__device__ __forceinline__ void fin_bc(double& e, float& den2, double s, double nb, double mv, float uq, float qv) {
    static_assert(kEps == 1e-8f, "the asm's literal is kEps");
    asm("v_mov_b64 %0, %6\n\t"
        "v_mov_b32 %1, 0x322bcc77\n\t"
        "v_fmac_f64_dpp %0, %2, %3 row_newbcast:%7 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %4, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf"
        : "=&v"(e), "=&v"(den2)
        : "v"(nb), "v"(mv), "v"(uq), "v"(qv), "v"(s), "i"(L));
}

// Kernel sizes with a compile-time sweep instantiation (register-resident
// column sums need a static trip count): every k <= 31 (round 5: even k 18 .. 30 too; the
// backward's K-deep ring of 16 rows fills the CU's LDS at 31, the forward's 16 + k - 1 camera
// columns its three broadcast registers at 33).  Other sizes up to CUSTMA_MAX_KERNEL run on the
// exact forward and the generic fp64 backward.
#define CUSTMA_SWEEP_KS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31)

struct SweepGrid {
    int nChunk;  // diagonal chunks per column tile
    int nTile;   // column tiles of TW
    int nBand;   // row bands
    int TH;      // rows per band
    int NL;      // diagonal lanes per workgroup (compute waves x 64)
    int S;       // chunk stride in volume columns (== NL unless chunks own aligned columns)
};

struct DispPartial {
    float* best;     // [nChunk][HV][WO]
    float* second;   // [nChunk][HV][WO]
    int32_t* index;  // [nChunk][HV][WO] layout index s of best, -1 if none
    // soft-argmax (examples/verify.py:31-39): with kb = beta * log2(e) > 0, the chunk's
    // sum of exp(beta (cost - best)) and of s * exp(beta (cost - best)) (s = layout index)
    float* s0;       // [nChunk][HV][WO] or null
    float* s1;       // [nChunk][HV][WO] or null
    float kb;
};

// Online soft-argmax accumulation next to the running (best, second, first index): the
// weights are taken relative to the running best (rescaled when it grows), so they never
// overflow; invalid entries (-FLT_MAX) carry no weight.
__device__ __forceinline__ void soft_add(float v, float idx, float best_before, float kb, float& s0, float& s1) {
    // branch-free, one exp2: a new best rescales the sums by exp2(kb (best_before - v)) and adds
    // weight 1, otherwise the element adds exp2(kb (v - best_before))
    const bool gt = v > best_before;
    const float e = __builtin_amdgcn_exp2f(kb * (gt ? best_before - v : v - best_before));
    s0 = gt ? s0 * e + 1.f : s0 + e;
    s1 = gt ? s1 * e + idx : s1 + e * idx;
}
// merge another accumulator (bo, o0, o1) into (b, s0, s1); both relative to their own best
__device__ __forceinline__ void soft_merge(float b, float bo, float o0, float o1, float kb, float& s0, float& s1) {
    const float m = b > bo ? b : bo;
    // the side holding the max has factor 1 exactly (no inf - inf when both are empty)
    const float fa = b == m ? 1.f : __builtin_amdgcn_exp2f(kb * (b - m));
    const float fb = bo == m ? 1.f : __builtin_amdgcn_exp2f(kb * (bo - m));
    s0 = s0 * fa + o0 * fb;
    s1 = s1 * fa + o1 * fb;
}

// Lane / chunk geometry.
//
// owned = false: the diagonal range of a column tile is split into disjoint
// chunks of NL (disparity partials, backward).
// owned = true (volume stores): chunk c owns the columns [b_c, b_c+1) of every
// volume row, b_c = the first column >= c*S that starts a 64-byte sector, so
// every sector of the volume has one writer (two workgroups writing parts of
// one sector halve the store bandwidth, scripts/micro/store_sim.hip).  A row
// range of up to S+15 columns shifted by the 16 camera columns of the tile
// (full layout) needs S + 15 (+15 when volume rows are not sector aligned)
// diagonal lanes, so neighbouring chunks compute a few diagonals twice.
inline int owned_margin(const Geo& g) {
    if (g.layout == CUSTMA_LAYOUT_WINDOW) return 16;
    return g.DO % 16 == 0 ? 16 : 32;
}

inline SweepGrid sweep_grid(const Geo& g, bool owned = false) {
    SweepGrid sg;
    const int64_t ncol = g.DO;  // volume columns per row (full: W, window: D+1)
    const int64_t nd = g.layout == CUSTMA_LAYOUT_WINDOW ? (int64_t)g.D + 1 : g.W + TW - 1;
    const int margin = owned ? owned_margin(g) : 0;
    // cost = diagonal lanes launched, penalised for single-wave workgroups
    double best = 1e300;
    sg.NL = 256;
    for (int nw = 1; nw <= 5; ++nw) {
        if (owned && 64 * nw <= margin) continue;
        if (!owned && g.layout != CUSTMA_LAYOUT_WINDOW && nw > 4) continue;
        const int64_t per = owned ? 64 * nw - margin : 64 * nw;
        const int64_t n = owned ? cdiv(ncol, per) : cdiv(nd, per);
        // the disparity partials (!owned): 3-wave chunks run best where lane counts tie (C2 full:
        // 1.98 ms against 2.39 for 2 waves and 3.06 for 4, profiles/r03/disp2), so ties go to more
        // waves and 4 waves pay 10 %
        const double cost = (double)(n * 64 * nw) * (nw == 1 ? 1.1 : 1.0) * (nw == 5 ? 1.05 : 1.0) *
                            (!owned && nw == 4 ? 1.1 : 1.0);
        if (cost < best || (!owned && cost == best)) { best = cost; sg.NL = 64 * nw; }
    }
    sg.S = owned ? sg.NL - margin : sg.NL;
    sg.nChunk = (int)(owned ? cdiv(ncol, (int64_t)sg.S) : cdiv(nd, (int64_t)sg.NL));
    sg.nTile = (int)cdiv(g.WO, TW);
    // band height: the volume (owned) sweeps 128 rows -- half the K - 1 warm-up steps per output row of 64:
    // C3 full 9.27-9.36 -> 9.11-9.12 ms, C2 full 1.13-1.16 -> 1.12-1.14 ms; the disparity partials keep 64
    // (C2 full 1.77 -> 1.81 ms at 128), profiles/r06/j
#ifdef CUSTMA_SWEEP_TH
    sg.TH = CUSTMA_SWEEP_TH;  // (A/B builds)
#else
    sg.TH = owned ? 128 : 64;
#endif
    // keep >= ~4 workgroups per CU on small problems
    while (sg.TH > 8 && (int64_t)sg.nTile * sg.nChunk * cdiv(g.HV(), sg.TH) < 2048) sg.TH /= 2;
    sg.nBand = (int)cdiv(g.HV(), sg.TH);
    return sg;
}

// Wave-independent forward (sweep_wave.hip): one wave per (row band, column tile, chunk of
// 64 diagonals).
struct WaveGrid {
    int nChunk, nTile, nBand, TH;
    bool rem;  // window, (D+1) % 64 == 1: the last chunk's waves add diagonal D
};
WaveGrid wave_grid(const Geo& g, bool disparity = false);
hipError_t launch_fwd_lds(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                          float* out, hipStream_t s);

inline int64_t sweep_blocks(const SweepGrid& sg) { return (int64_t)sg.nBand * sg.nTile * sg.nChunk; }

// per-kernel-size entry points of sweep_wave.hip (one translation unit per size)
template <int K>
hipError_t sw_fwd(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, float* out,
                  hipStream_t s);
template <int K>
hipError_t sw_amx(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, DispPartial part,
                  hipStream_t s);

hipError_t launch_disp_partials(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                                DispPartial part, hipStream_t s);
// window layout, D + 1 <= 257: the tile kernel writes ONE partial per pixel (all diagonals)
bool disp_tile_ok(const Geo& g);
hipError_t launch_disp_tile(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            DispPartial part, hipStream_t s);

}  // namespace custma
