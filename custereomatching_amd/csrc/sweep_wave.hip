// Fast forward, wave-independent form: the default volume-writing sweep.
//
// Same arithmetic as k_sweep_fwd (sweep_fwd.hip; reference: custma/src/
// stereo_matching_kernel.cu:39-71): per disparity diagonal delta = d - w the
// patch sums of c * p slide down the rows and across the columns in fp64
// (fp32 x fp32 products are exact there), the mean correction uses the fp64
// patch sums, and the denominator the reference's own fp32 moments:
//     cost = (float)(S + eps - boxc * boxp / k^2) * rsq(fma(ex2, ey2, eps)).
//
// Work unit = ONE wave: 64 consecutive diagonals (lane l: delta = d0 + l) x 16
// camera columns (u0 .. u0+15) x a band of TH rows.  Unlike k_sweep_fwd there
// is no loader wave, no workgroup barrier and no output staging: every wave
// loads its own image rows and statistics (14 buffer loads per row step, two
// steps in flight, issued as inline asm with hand-counted `s_waitcnt vmcnt`
// -- the compiler's own tracking drains the pipeline at the loop header), puts
// the two projector row segments and the projector statistics in a 3.5 KB
// wave-private LDS slice (the sliding-window reads need them there), keeps the
// camera values row-replicated in registers (DPP row_newbcast operands), and
// stores the 16 volume rows of a step straight from registers: lane l writes
// volume column d0 + l (window layout) / u0 + m + d0 + l (full layout), so
// each store instruction is 256 contiguous bytes of one volume row.
//
// Per voxel: 2(16+2r)/16 fp64 FMAs + as many ds_read_b64 (row update), 2 fp64
// adds (column slide), 1 fp64 FMA + cvt (mean correction), fp32 fma + rsq + mul.
#include <float.h>
#include <limits.h>
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "sweep.h"

// Build: compiled once per kernel size with -DCUSTMA_SW_K=<k> (the kernels and launchers of
// that size: sw_fwd<k>, sw_amx<k>) and once with -DCUSTMA_SW_DISPATCH (grid planning and the
// run-time dispatch over k), so the instantiations compile in parallel.
namespace custma {

constexpr int kTileMaxChunks = 4;  // k_fwd_tile: diagonal chunks (waves) per workgroup

#ifndef CUSTMA_SW_DISPATCH
namespace {

typedef __attribute__((address_space(3))) volatile double lds_vd;
typedef __attribute__((address_space(3))) volatile float lds_vf;

constexpr int kRowP = 128;  // LDS row stride (>= 16 + 2r + 63)
// The row update's DPP FMAs keep their `s_nop 1` only where a camera operand may have just
// been converted (the first group of each 16-column half); hazard_check.py checks the
// listing at build time.
constexpr int kFwdPF = 2;  // outputs whose projector statistics are read ahead from LDS

// REM: this wave (window layout, last chunk, (D+1) % 64 == 1) also computes the single
// remainder diagonal d0 + 64 = D: lane x < 16 + 2r keeps its column sum, the horizontal box
// is summed from LDS, and lanes m < 16 store volume column D of tile row m.
//
// STAGED (window layout, k_fwd_tile): the workgroup holds every diagonal chunk of one
// column tile; each wave puts its 16 x 64 outputs of a step into an LDS image of the 16
// contiguous volume rows (two step buffers), and after one barrier the workgroup stores
// the whole 16 * DO-float block with dword stores, SS per thread (OOB-masked, so every
// thread issues exactly SS and the hand-counted vmcnt holds): every volume sector is
// written once, by one workgroup, in one burst.
//
// AMX > 0 (STAGED, fused disparity): no volume; after the barrier each 16-lane group scans
// one of the 16 LDS rows (all D+1 diagonals of one camera pixel) for (best, second, first
// index of best), AMX passes of 4 rows per wave, and writes them as one disparity partial.
// AMX < 0: fused disparity with the soft-argmax sums (DispPartial::s0 / s1), -AMX passes.
//
// Taps (the reference's `kernel_size / 2` origin, stereo_matching_kernel.cu:44,60): rows h - R0 .. h + R1
// and columns w - R0 .. w + R1 with R0 = K/2, R1 = K-1-K/2 (R0 = R1 = r for odd K; even K is asymmetric).
//
// CPL (STAGED): the workgroup's camera rows h0 - R0 .. h1 + R1 - 1, columns u0 - R0 .. u0 - R0 + NX - 1
// (every wave needs the same ones) are loaded once into LDS (camL, zero-padded) before the sweep,
// instead of four 16-address loads per wave and step: those loads were most of the sweep's load
// cost (C5: 9.80 -> 8.25 ms with every camera load out of range, profiles/r03/fwdabl).
// the fused disparity's stage row pitch: all D + 1 <= 64 kTileMaxChunks + 1 diagonals, rounded up to the
// scan's 16 lanes (the columns past DO padded with -FLT_MAX)
constexpr int kAmxPitch = 16 * ((64 * kTileMaxChunks + 1 + 15) / 16);
template <int K, typename T, bool FULL_EDGE, bool REM, bool STAGED = false, int SS = TW, int P = 2, int AMX_ = 0,
          bool CPL = false>
__device__ __forceinline__ void wave_body(const T* __restrict__ cam, const T* __restrict__ proj, const Geo& g,
                                          const Stats& sc, const Stats& sp, float* __restrict__ out,
                                          int64_t u0, int64_t h0, int64_t h1, int64_t d0,
                                          double* rowE, double* rowL, double* sM, float* sQ, double* sR,
                                          float* stage = nullptr, DispPartial part = DispPartial{},
                                          T* camL = nullptr) {
    static_assert(!CPL || STAGED, "the camera preload is shared by the workgroup's waves");
    typedef std::conditional_t<sizeof(T) == 2, unsigned short, uint32_t> RawT;  // raw image bits
    constexpr int AMX = AMX_ < 0 ? -AMX_ : AMX_;
    constexpr bool SOFT = AMX_ < 0;
    constexpr int R0 = K / 2, R1 = K - 1 - K / 2, NX = TW + K - 1;
    static_assert(NX + 63 <= kRowP && NX <= 48, "row segment fits the LDS slice and three broadcast registers");
    constexpr bool C3R = NX > 32;  // a third camera register (columns 32 .. 47 of the tile, k >= 19)
    constexpr uint32_t OOB = 0x80000000u;
    // SS (STAGED): dword stores per thread per step, the same for every wave of the workgroup;
    // SS < 0: -SS 16-byte stores + one dword store (the block's < 4-float tail) per thread
    const int l = threadIdx.x & 63, r16 = l & 15;
    const int64_t hs = h0 - (K - 1);  // K - 1 warm-up steps fill the column sums
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    const double rk2 = 1.0 / (double)(K * K);

    // ---- per-lane column byte offsets (out of the image -> OOB -> 0: the reference's zero
    // padding, stereo_matching_kernel.cu:6-12); rows are selected by the descriptors ----
    auto colOff = [&](bool have, int64_t x, int esz) -> uint32_t {
        return (have && x >= 0 && x < g.W) ? (uint32_t)(x * esz) : OOB;
    };
    const int64_t xO0 = u0 - R0 + d0, oS = u0 + d0;
    const uint32_t vP0 = colOff(true, xO0 + l, sizeof(T)), vP1 = colOff(64 + l < NX + 64, xO0 + 64 + l, sizeof(T));
    const uint32_t vC0 = colOff(true, u0 - R0 + r16, sizeof(T)), vC1 = colOff(16 + r16 < NX, u0 - R0 + 16 + r16, sizeof(T));
    const uint32_t vC2 = colOff(32 + r16 < NX, u0 - R0 + 32 + r16, sizeof(T));
    const uint32_t vM0 = colOff(true, oS + l, 8), vM1 = colOff(64 + l < TW + 64, oS + 64 + l, 8);
    const uint32_t vQ0 = colOff(true, oS + l, 4), vQ1 = colOff(64 + l < TW + 64, oS + 64 + l, 4);
    const uint32_t vUB = colOff(true, u0 + r16, 8), vUQ = colOff(true, u0 + r16, 4);
    // Rows by SGPR soffset from one descriptor per array, based at the band's first row rb
    // (so every offset stays small whatever the image size); a row outside the image gets
    // soffset OOBS, past num_records (<= OOBS), so its loads read 0 -- also when the lane's
    // column offset is OOB itself (0x80000000 + OOBS does not wrap).
    constexpr uint32_t OOBS = 0x7FFFFFF0u;
    const int Hi = (int)g.H, h0i = (int)h0, h1i = (int)h1;
    const int rb = max(0, h0i - 3 * R0 - 1);  // <= the first consumed row h0 - R0
    const uint32_t rbT = (uint32_t)(g.W * sizeof(T)), rb8 = (uint32_t)(g.W * 8), rb4 = (uint32_t)(g.W * 4);
    auto band_rsrc = [&](const void* base, uint32_t rowbytes) {
        const uint64_t n = (uint64_t)(g.H - rb) * rowbytes;
        return make_rsrc_sgpr((const char*)base + (int64_t)rb * rowbytes, n < OOBS ? (uint32_t)n : OOBS);
    };
    const i32x4 dCam = band_rsrc(cam, rbT), dProj = band_rsrc(proj, rbT);
    const i32x4 dPB = band_rsrc(sp.box, rb8), dPS = band_rsrc(sp.sq, rb4);
    const i32x4 dCB = band_rsrc(sc.box, rb8), dCS = band_rsrc(sc.sq, rb4);
    // (wave-uniform; readfirstlane pins it to an SGPR for the asm loads, whose `s_nop 4`
    // covers the VALU-writes-SGPR hazard)
    auto so_row = [&](int row, uint32_t rowbytes, bool ok) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)((ok && (unsigned)row < (unsigned)Hi) ? (uint32_t)(row - rb) * rowbytes : OOBS));
    };

    struct Stage {
        uint32_t pe0, pe1, pl0, pl1, ce0, ce1, cl0, cl1, ce2, cl2, q0, q1, uq;
        double m0, m1, ub;
    };
    constexpr int kLoads = CPL ? 10 : C3R ? 16 : 14;
    if constexpr (CPL) {
        // camera rows h0 - R0 + i (i < h1 - h0 + K - 1), columns u0 - R0 + j (j < NX), raw, 0 outside the image
        typedef __attribute__((address_space(3))) RawT lds_t;
        const RawT* cr = (const RawT*)cam;
        const int nr = (int)(h1 - h0) + K - 1;
        for (int e = (int)threadIdx.x; e < nr * NX; e += (int)blockDim.x) {
            const int64_t row = h0 - R0 + e / NX, c = u0 - R0 + e % NX;
            ((lds_t*)camL)[e] = (row >= 0 && row < g.H && c >= 0 && c < g.W) ? cr[row * g.W + c] : (RawT)0;
        }
        __syncthreads();
    }
    // step t adds image row t+R1 and removes row t-R0-1 (rows from h0-R0 on were added, so the
    // first removal is at t = h0+1); statistics of row t (only for t in [h0, h1))
    auto load_step = [&](int64_t t, Stage& p) {
        const int ti = (int)t;
        const uint32_t sE = so_row(ti + R1, rbT, true), sL = so_row(ti - R0 - 1, rbT, ti > h0i);
        if constexpr (CPL)
            asm_ld_img4<T>(p.pe0, p.pe1, p.pl0, p.pl1, vP0, vP1, dProj, sE, sL);
        else
        {
            asm_ld_img8<T>(p.pe0, p.pe1, p.pl0, p.pl1, p.ce0, p.ce1, p.cl0, p.cl1, vP0, vP1, vC0, vC1, dProj, dCam,
                           sE, sL);
            if constexpr (C3R) asm_ld_img2<T>(p.ce2, p.cl2, vC2, dCam, sE, sL);
        }
        const bool st = ti >= h0i && ti < h1i;
        asm_ld_stat6(p.m0, p.m1, p.q0, p.q1, p.ub, p.uq, vM0, vM1, vQ0, vQ1, vUB, vUQ, dPB, dPS, dCB, dCS,
                     so_row(ti, rb8, st), so_row(ti, rb4, st));
    };
    auto tie = [&](Stage& p) {
        asm_tie(p.pe0); asm_tie(p.pe1); asm_tie(p.pl0); asm_tie(p.pl1);
        asm_tie(p.ce0); asm_tie(p.ce1); asm_tie(p.cl0); asm_tie(p.cl1);
        if constexpr (C3R && !CPL) { asm_tie(p.ce2); asm_tie(p.cl2); }
        asm_tie(p.q0); asm_tie(p.q1); asm_tie(p.uq); asm_tie(p.m0); asm_tie(p.m1); asm_tie(p.ub);
    };

    // ---- output addressing: one descriptor per step (volume rows (h, u0 .. u0+15), clipped
    // to the valid camera columns), the tile row m in soffset, the column in voffset ----
    const int64_t DO = g.DO;
    const int64_t a0 = window ? d0 + l : u0 + d0 + l;  // volume column of tile row 0
    uint32_t vOut = OOB;                              // constant per lane unless FULL_EDGE
    if (window) vOut = (d0 + l <= g.D) ? (uint32_t)(a0 * 4) : OOB;
    else if (!FULL_EDGE) vOut = (uint32_t)(a0 * 4);  // interior chunk: every voxel valid
    const int64_t nrow = min((int64_t)TW, g.WO - u0);
    const uint32_t tile_bytes = (uint32_t)(nrow * DO * 4);
    // volume block of output row t: orow = out + ((t - h_lo) WO + u0) DO, advanced one row per
    // output step (no 64-bit multiply per step)
    float* orow = out + ((h0 - g.h_lo) * g.WO + u0) * DO;
    const int64_t ostep = g.WO * DO;
    const int sstep = (int)((DO + (window ? 0 : 1)) * 4);  // soffset per tile row

    double col[NX];
#pragma unroll
    for (int x = 0; x < NX; ++x) col[x] = 0.0;
    double colR = 0.0;  // REM: column sum of diagonal d0 + 64 for column x = lane (lanes < NX)

    // The loads of step t are issued at the end of step t-P (P = 2, or 3 in the staged
    // kernel).  The first P issues happen in P warm-up iterations of the loop itself
    // (t = hs-P .. hs-1: loads only), not in a
    // prologue: the compiler believes an asm load's destination is written when the asm
    // issues, so a peeled prologue with another register assignment would be joined to the
    // loop by register copies -- reads of registers whose loads are still in flight.
    Stage st[P];
    // stores per step (every thread issues exactly ST: the hand-counted waits rely on it).  Each store
    // site below restates its own count in a static_assert (ST_*), so a site whose store count changes
    // without ST fails to compile; every store there is unconditional (masked by an out-of-range
    // offset, never by a branch), so the count is the same for every thread and step.
    constexpr int ST_AMX = (SOFT ? 5 : 3) * AMX, ST_X4 = -SS + 1, ST_DW = SS, ST_DIRECT = TW + (REM ? 1 : 0);
    constexpr int ST = AMX > 0 ? ST_AMX : STAGED ? (SS < 0 ? ST_X4 : ST_DW) : ST_DIRECT;
    static_assert((P - 1) * (kLoads + ST) <= 63, "vmcnt holds the pipeline");
    // out_c: std::true_type for an output step (t >= h0: stores), std::false_type for a warm-up step
    // (P == 2: both fixed at compile time, so the waits are too); a runtime bool with P == 3
    auto compute = [&](Stage& p, int64_t t, auto out_c) {
        const bool out = out_c;
        // loads(t) were issued at the end of step t-P; after them, for each step s in
        // t-P+1 .. t-1: its stores (from step h0 on) and loads(s+P)
        if constexpr (P == 3) {
            if (t - 2 >= h0) asm_vmcnt<2 * (kLoads + ST)>();
            else if (t - 1 >= h0) asm_vmcnt<2 * kLoads + ST>();
            else asm_vmcnt<2 * kLoads>();
        } else if constexpr (std::is_same<decltype(out_c), std::true_type>::value) {
            // the previous step stored (or, for t = h0, the null stores between the phases stand in)
            asm_vmcnt<kLoads + ST>();
        } else {
            asm_vmcnt<kLoads>();
        }
        tie(p);
        rowE[l] = raw_to_f64<T>(p.pe0);
        rowE[64 + l] = raw_to_f64<T>(p.pe1);
        rowL[l] = raw_to_f64<T>(p.pl0);
        rowL[64 + l] = raw_to_f64<T>(p.pl1);
        sM[l] = p.m0 * rk2;
        sM[64 + l] = p.m1 * rk2;
        sQ[l] = __builtin_bit_cast(float, p.q0);
        sQ[64 + l] = __builtin_bit_cast(float, p.q1);
        uint32_t ce0 = p.ce0, ce1 = p.ce1, cl0 = p.cl0, cl1 = p.cl1, ce2 = 0u, cl2 = 0u;
        if constexpr (C3R && !CPL) {
            ce2 = p.ce2;
            cl2 = p.cl2;
        }
        if constexpr (CPL) {
            // the rows enter t + R1 and leave t - R0 - 1 (from t = h0 + 1 on) of the preloaded block
            typedef __attribute__((address_space(3))) const RawT lds_ct;
            const lds_ct* cr = (const lds_ct*)camL;
            const int er = (int)(t - h0) + K - 1, lr = (int)(t - h0) - 1;
            const bool hi = 16 + r16 < NX, lv = t > h0;
            ce0 = (uint32_t)cr[er * NX + r16];
            ce1 = hi ? (uint32_t)cr[er * NX + 16 + r16] : 0u;
            cl0 = lv ? (uint32_t)cr[lr * NX + r16] : 0u;
            cl1 = lv && hi ? (uint32_t)cr[lr * NX + 16 + r16] : 0u;
            if constexpr (C3R) {
                const bool h2 = 32 + r16 < NX;
                ce2 = h2 ? (uint32_t)cr[er * NX + 32 + r16] : 0u;
                cl2 = lv && h2 ? (uint32_t)cr[lr * NX + 32 + r16] : 0u;
            }
        }
        const double ca0 = raw_to_f64<T>(ce0), ca1 = raw_to_f64<T>(ce1);
        const double cb0 = -raw_to_f64<T>(cl0), cb1 = -raw_to_f64<T>(cl1);
        const double ca2 = C3R ? raw_to_f64<T>(ce2) : 0.0, cb2 = C3R ? -raw_to_f64<T>(cl2) : 0.0;
        const double nb = -p.ub;                           // -(camera patch sum) of column r16
        const float uq = __builtin_bit_cast(float, p.uq);  // camera ex2 of column r16

        // ---- col[x] += c(enter, x) p(enter, x + delta) - c(leave, x) p(leave, x + delta) ----
        {
            const lds_vd* oa = (const lds_vd*)(rowE + l);
            const lds_vd* ob = (const lds_vd*)(rowL + l);
            constexpr int B = 4, NB = (NX + B - 1) / B;
            double pa[2][B], pb[2][B];
            auto fetch = [&](auto bc) {
                constexpr int bb = decltype(bc)::value, x0 = bb * B;
                constexpr int nb_ = NX - x0 < B ? NX - x0 : B;
                Unroll<0, nb_>::run([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    pa[bb & 1][i] = oa[x0 + i];
                    pb[bb & 1][i] = ob[x0 + i];
                });
            };
            fetch(std::integral_constant<int, 0>{});
            Unroll<0, NB>::run([&](auto bc) {
                constexpr int bb = decltype(bc)::value, x0 = bb * B;
                constexpr int nb_ = NX - x0 < B ? NX - x0 : B;
                if constexpr (bb + 1 < NB) fetch(std::integral_constant<int, bb + 1>{});
                const double a = x0 < 16 ? ca0 : x0 < 32 ? ca1 : ca2, b = x0 < 16 ? cb0 : x0 < 32 ? cb1 : cb2;  // x0 % 4 == 0
                const double* qa = pa[bb & 1];
                const double* qb = pb[bb & 1];
                if constexpr (nb_ == 4) {
                    fmac2_bc64_x4<(x0 & 15), (x0 & 15) == 0>(col[x0], col[x0 + 1], col[x0 + 2], col[x0 + 3], a, b, qa[0], qa[1],
                                             qa[2], qa[3], qb[0], qb[1], qb[2], qb[3]);
                } else if constexpr (nb_ == 2) {
                    fmac2_bc64_x2<(x0 & 15), (x0 & 15) == 0>(col[x0], col[x0 + 1], a, b, qa[0], qa[1], qb[0], qb[1]);
                } else {
                    Unroll<0, nb_>::run([&](auto ic) {
                        constexpr int i = decltype(ic)::value, x = x0 + i;
                        fmac_bc64<(x & 15), (x0 & 15) == 0>(col[x], a, qa[i]);
                        fmac_bc64<(x & 15), (x0 & 15) == 0>(col[x], b, qb[i]);
                    });
                }
            });
        }

        if constexpr (REM) {
            const double cRe = l < 16 ? ca0 : l < 32 ? ca1 : ca2, cRl = l < 16 ? cb0 : l < 32 ? cb1 : cb2;  // column u0 - R0 + l
            colR = __builtin_fma(cRe, *(const lds_vd*)(rowE + 64 + l), colR);
            colR = __builtin_fma(cRl, *(const lds_vd*)(rowL + 64 + l), colR);
        }
        if (out) {
            const auto rOut = make_rsrc(orow, tile_bytes);
            orow += ostep;
            double s = col[0] + (double)kEps;  // E + eps: eps rides along the sliding sum
#pragma unroll
            for (int x = 1; x < K; ++x) s += col[x];
            // the projector mean / moment of output m, read PF outputs ahead (plain reads, issued
            // in program order before the stage writes of the outputs in between)
            typedef __attribute__((address_space(3))) const double lds_d;
            typedef __attribute__((address_space(3))) const float lds_f;
            const lds_d* mrow = (const lds_d*)(sM + l);
            const lds_f* qrow = (const lds_f*)(sQ + l);
            constexpr int PF = kFwdPF;
            double mq[PF];
            float qq[PF];
            Unroll<0, PF>::run([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                mq[i] = mrow[i];
                qq[i] = qrow[i];
            });
            // STAGED: this step's buffer; rows at pitch DO (the block the stores copy out), or at
            // kAmxPitch with the fused disparity (the columns past DO hold -FLT_MAX, k_fwd_tile)
            const int SPc = AMX > 0 ? kAmxPitch : (int)DO;
            lds_vf* sb = (lds_vf*)(stage + (t & 1) * TW * SPc);
            const bool dv = d0 + l <= g.D;
            // every lane of the chunk valid (all but a partial last chunk): unmasked stage writes,
            // no per-output exec branch
            const bool allv = d0 + 63 <= g.D;
            // FULL_EDGE: the column base opaque per step, so that the per-row store offsets below are
            // not hoisted out of the output loop (16 VGPRs held across it: 141 -> 169 VGPRs)
            int64_t a0S = a0;
            if constexpr (FULL_EDGE) asm volatile("" : "+v"(a0S));
            auto outputs = [&](auto masked_c) {
            constexpr bool MASKED = decltype(masked_c)::value;
            Unroll<0, TW>::run([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                if (m > 0) s = (s + col[m + K - 1]) - col[m - 1];
                double e;
                float den2;
                const double mv = mq[m % PF];
                const float qv = qq[m % PF];
                if constexpr (m + PF < TW) {
                    mq[m % PF] = mrow[m + PF];
                    qq[m % PF] = qrow[m + PF];
                }
                // E + eps = S + eps - box_c * mean_p;  ex2 * ey2 + eps
                fin_bc<m>(e, den2, s, nb, mv, uq, qv);
                const float c = (float)e * __builtin_amdgcn_rsqf(den2);
                uint32_t vo = vOut, so = (uint32_t)(m * sstep);
                if constexpr (FULL_EDGE) {  // per-row mask; the whole offset in voffset
                    vo = ((uint64_t)(a0S + m) < (uint64_t)g.W) ? (uint32_t)((a0S + m + m * DO) * 4) : OOB;
                    so = 0;
                }
                if constexpr (STAGED) {
                    if (!MASKED || dv) sb[m * SPc + d0 + l] = c;
                } else {
                    static_assert(STAGED || ST == TW + (REM ? 1 : 0), "ST_DIRECT: one store per tile row (+ REM's)");
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, c), rOut, vo, so,
                                                      kStoreAux);
                }
            });
            };
            if (!STAGED || allv) outputs(std::false_type{});
            else outputs(std::true_type{});
            if constexpr (REM) {
                // diagonal D for tile row m = lane: box over the column sums of lanes m .. m + K - 1
                sR[l] = colR;
                double sr = (double)kEps;
                const lds_vd* rr = (const lds_vd*)(sR + (l & 15));
#pragma unroll
                for (int x = 0; x < K; ++x) sr += rr[x];
                const double e = __builtin_fma(nb, *(const lds_vd*)(sM + 64 + (l & 15)), sr);
                const float den2 = __builtin_fmaf(uq, *(const lds_vf*)(sQ + 64 + (l & 15)), kEps);
                const float c = (float)e * __builtin_amdgcn_rsqf(den2);
                if constexpr (STAGED) {
                    if (l < 16) sb[l * SPc + g.D] = c;
                } else {
                    const uint32_t vo = l < 16 ? (uint32_t)((l * DO + g.D) * 4) : OOB;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, c), rOut, vo, 0u,
                                                          kStoreAux);
                }
            }
            if constexpr (STAGED) {
                // every wave's part of the 16 rows is in LDS: store the block (256 contiguous
                // bytes per wave instruction, the whole workgroup's instruction contiguous)
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                const int NT = (int)blockDim.x;
                // opaque per step: the block's store offsets are recomputed at each step instead of
                // hoisted out of the output loop, where they would hold SS VGPRs across it (141 -> 166-171
                // VGPRs, two waves per SIMD instead of three)
                int tid = (int)threadIdx.x;
                asm volatile("" : "+v"(tid));
                const int total = (int)(nrow * DO);
                if constexpr (AMX > 0) {
                    const int wv = tid >> 6, nw = NT >> 6, sub = l & 15;
                    const int64_t prow = (t - g.h_lo) * g.WO + u0;
                    const uint32_t pb = (uint32_t)(nrow * 4);
                    const auto rB = make_rsrc(part.best + prow, pb), rS = make_rsrc(part.second + prow, pb);
                    const auto rI = make_rsrc(part.index + prow, pb);
                    // soft-argmax sums (null arrays: out-of-range stores, so the store count holds)
                    constexpr bool soft = SOFT;
                    const auto rQ0 = make_rsrc(soft ? part.s0 + prow : part.best, soft ? pb : 0u);
                    const auto rQ1 = make_rsrc(soft ? part.s1 + prow : part.best, soft ? pb : 0u);
                    const float kb = part.kb;
                    // AMX passes x (best, second, index [, s0, s1]) stores
                    static_assert(ST == AMX * (3 + (SOFT ? 2 : 0)), "ST_AMX");
#pragma unroll
                    for (int ps = 0; ps < AMX; ++ps) {
                        const int m = (ps * nw + wv) * 4 + (l >> 4);  // tile row of this 16-lane group
                        const int mr = m < TW ? m : 0;
                        // No bound test in the scans: the row's columns DO .. 16 nsc - 1 hold -FLT_MAX, which
                        // changes none of the results, so the reads batch up (an exec-masked read per element
                        // waited for each one: the scan was 28 % of the kernel, profiles/r05/k).  Partly
                        // unrolled: fully unrolled, the compiler hoists all 17 LDS reads (and the soft sums'
                        // exp2 operands) and the kernel needs 168-206 VGPRs.
                        const int nsc = ((int)DO + 15) >> 4;
                        const lds_vf* row = sb + mr * kAmxPitch + sub;
                        auto rot = [&](float x, auto ctl) {
                            return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                0, __builtin_bit_cast(int, x), decltype(ctl)::value, 0xf, 0xf, false));
                        };
                        float b = -FLT_MAX, sec = -FLT_MAX, q0 = 0.f, q1 = 0.f;
                        int bi = INT_MAX;
                        if constexpr (SOFT) {
                            // Two passes (round 6).  Pass 1: the top two VALUES (exact floats; duplicates count,
                            // so a tie leaves sec == b) by v_max / v_med3, 2 VALU per element, the 16 lanes of the
                            // row combined by DPP row rotations (8, 4, 2, 1: every lane meets each other lane's
                            // part once).  Pass 2, the row's best known: the first index holding it (v == b: the
                            // first index wins among equal values, torch.argmax semantics) and the soft sums
                            // weighted relative to it, so no running rescale.  C3 soft 1.75 -> 1.40 ms, C5
                            // 14.4 -> 11.4 ms; the plain argmax measured slower this way (C3 1.24 -> 1.26 ms:
                            // pass 2 re-reads the row) and keeps the one-pass scan below (profiles/r06/c).
#pragma unroll 6
                            for (int i = 0; i < nsc; ++i) {
                                const float v = row[16 * i];
                                sec = __builtin_amdgcn_fmed3f(b, sec, v);  // b >= sec: the new second
                                b = __builtin_fmaxf(b, v);
                            }
                            Unroll<0, 4>::run([&](auto lc) {
                                const std::integral_constant<int, 0x120 + (8 >> decltype(lc)::value)> ctl;  // row_ror
                                const float ob = rot(b, ctl), os = rot(sec, ctl);
                                sec = __builtin_amdgcn_fmed3f(b, ob, __builtin_fmaxf(sec, os));  // top two of four
                                b = __builtin_fmaxf(b, ob);
                            });
                            int fi = INT_MAX;  // the first i with row[16 i] == b (this lane)
                            float qi = 0.f;    // sum of i w (w = exp2(kb (v - b)); q0 = sum of w)
                            const float nkb = b > -FLT_MAX ? -kb * b : 0.f;  // (a row without values: every w = 0)
#pragma unroll 3
                            for (int i = nsc - 1; i >= 0; --i) {
                                const float v = row[16 * i];
                                fi = v == b ? i : fi;
                                const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(kb, v, nkb));
                                q0 += w;
                                qi = __builtin_fmaf(w, (float)i, qi);
                            }
                            bi = fi == INT_MAX || !(b > -FLT_MAX) ? INT_MAX : sub + 16 * fi;
                            q1 = __builtin_fmaf((float)sub, q0, 16.f * qi);  // sum of s w, s = sub + 16 i
                            Unroll<0, 4>::run([&](auto lc) {
                                const std::integral_constant<int, 0x120 + (8 >> decltype(lc)::value)> ctl;
                                bi = min(bi, __builtin_amdgcn_update_dpp(0, bi, decltype(ctl)::value, 0xf, 0xf, false));
                                q0 += rot(q0, ctl);
                                q1 += rot(q1, ctl);
                            });
                        } else {
                            // one scan chain per lane (increasing s: the strict compare keeps the first index among
                            // equal values; the top two by v_med3 / v_max, C3 1.234 -> 1.208 ms against round 5's
                            // three selects, profiles/r06/f), then the 16 lanes of the row combined by DPP row
                            // rotations (8, 4, 2, 1).
#pragma unroll 6
                            for (int i = 0; i < nsc; ++i) {
                                const int s2 = sub + 16 * i;
                                const float v = row[16 * i];
                                const bool gt = v > b;
                                bi = gt ? s2 : bi;
                                sec = __builtin_amdgcn_fmed3f(b, sec, v);  // b >= sec: the new second
                                b = __builtin_fmaxf(b, v);
                            }
                            Unroll<0, 4>::run([&](auto lc) {
                                const std::integral_constant<int, 0x120 + (8 >> decltype(lc)::value)> ctl;
                                const float ob = rot(b, ctl), os = rot(sec, ctl);
                                const int oi = __builtin_amdgcn_update_dpp(0, bi, decltype(ctl)::value, 0xf, 0xf, false);
                                if (ob > b || (ob == b && oi < bi)) { sec = fmaxf(os, b); b = ob; bi = oi; }
                                else sec = fmaxf(sec, ob);
                            });
                        }
                        const uint32_t vo = (sub == 0 && m < TW) ? (uint32_t)(m * 4) : OOB;
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, b), rB, vo, 0u, 0);
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, sec), rS, vo, 0u, 0);
                        __builtin_amdgcn_raw_buffer_store_b32((unsigned int)(bi == INT_MAX ? -1 : bi), rI, vo, 0u, 0);
                        if constexpr (soft) {
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, q0), rQ0, vo, 0u, 0);
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, q1), rQ1, vo, 0u, 0);
                        }
                    }
                } else if constexpr (SS < 0) {  // block base 16-byte aligned (checked at launch)
                    static_assert(ST == -SS + 1, "ST_X4: -SS 16-byte stores + the tail's dword store");
                    const int n4 = total >> 2;
                    typedef __attribute__((address_space(3))) volatile i32x4 lds_v4;
#pragma unroll
                    for (int i = 0; i < -SS; ++i) {
                        const int j = i * NT + tid;
                        const i32x4 v = ((lds_v4*)sb)[j < n4 ? j : 0];
                        __builtin_amdgcn_raw_buffer_store_b128(v, rOut, j < n4 ? (uint32_t)(j * 16) : OOB, 0u,
                                                               kStoreAux);
                    }
                    const int j = 4 * n4 + tid;
                    const float v = sb[j < total ? j : 0];
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), rOut,
                                                          (tid < 4 && j < total) ? (uint32_t)(j * 4) : OOB, 0u,
                                                          kStoreAux);
                } else {
                    static_assert(ST == SS, "ST_DW: SS dword stores");
#pragma unroll
                    for (int i = 0; i < SS; ++i) {
                        const int idx = i * NT + tid;
                        const float v = sb[idx < total ? idx : 0];
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), rOut,
                                                              idx < total ? (uint32_t)(idx * 4) : OOB, 0u,
                                                              kStoreAux);
                    }
                }
            }
        }
    };
    // comp: compute the step (false: the first P steps, which only issue loads); P == 2 passes
    // compile-time constants throughout, so no step has a runtime test around its compute
    auto step = [&](auto kc, int64_t t, auto out_c, auto comp) {
        Stage& p = st[decltype(kc)::value];
        if (comp) compute(p, t, out_c);
        // past the band's end: harmless (rows out of range read zeros)
        load_step(t + P, p);
    };
    const std::true_type yes{};
    const std::false_type no{};
    if constexpr (P == 2) {
        // Three phases, every wait fixed at compile time, so that vmcnt_check.py can prove them on the
        // emitted code (a runtime choice between two waits, a runtime test around a step's compute, or a
        // `break` after each step gives paths the hardware never takes, on which the proof fails):
        //   t = hs - 2, hs - 1:  loads only;
        //   t = hs .. h0 - 1:    the K - 1 warm-up steps, no stores;
        //   t = h0 .. h1 - 1:    ST stores per step -- pairs with the loop's only exit at its test, then
        //                        an odd last step; ST null stores before it stand in for the stores of
        //                        the step before t = h0.
        // The stage buffers alternate throughout: the output phase starts on st[(K - 1) % 2].
        constexpr int A = (K - 1) % 2;
        int64_t t = hs - 2;
        asm volatile("" : "+s"(t));  // (opaque: the load-only steps stay one issue each)
        step(std::integral_constant<int, 0>{}, t, no, no);
        step(std::integral_constant<int, 1>{}, t + 1, no, no);
        t += 2;
#pragma unroll 1
        for (int i = 0; i < (K - 1) / 2; ++i, t += 2) {
            step(std::integral_constant<int, 0>{}, t, no, yes);
            step(std::integral_constant<int, 1>{}, t + 1, no, yes);
        }
        if constexpr (A == 1) {
            step(std::integral_constant<int, 0>{}, t, no, yes);
            ++t;
        }
        asm_null_stores<ST>(dCam);
        for (; t + 1 < h1; t += 2) {
            step(std::integral_constant<int, A>{}, t, yes, yes);
            step(std::integral_constant<int, 1 - A>{}, t + 1, yes, yes);
        }
        if (t < h1) step(std::integral_constant<int, A>{}, t, yes, yes);
    } else {
        int64_t t_first = hs - P;  // opaque: the warm-up iterations must not be peeled
        asm volatile("" : "+s"(t_first));
        for (int64_t t = t_first;; t += P) {
            step(std::integral_constant<int, 0>{}, t, t >= h0, t >= hs);
            if (t + 1 >= h1) break;
            step(std::integral_constant<int, 1>{}, t + 1, t + 1 >= h0, t + 1 >= hs);
            if (t + 2 >= h1) break;
            step(std::integral_constant<int, 2 % P>{}, t + 2, t + 2 >= h0, t + 2 >= hs);
            if (t + 3 >= h1) break;
        }
    }
    asm_vmcnt<0>();  // every wave drains its own loads before it ends
    // The last steps' loads (rows past the band) are dead, but their registers must not be reused
    // before they land -- a late load would overwrite the new value: keep them live until here.
#pragma unroll
    for (int i = 0; i < P; ++i) tie(st[i]);
}

template <int K, typename T>
__global__ __launch_bounds__(64) void k_fwd_wave(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                 Stats sc, Stats sp, float* __restrict__ out, WaveGrid wg) {
    __shared__ __attribute__((aligned(16))) double rowE[kRowP], rowL[kRowP], sM[kRowP];
    __shared__ __attribute__((aligned(16))) float sQ[kRowP];
    __shared__ __attribute__((aligned(16))) double sR[64];
    const int64_t bid = xcd_remap(blockIdx.x, gridDim.x);
    const int chunk = (int)(bid % wg.nChunk);
    const int64_t rest = bid / wg.nChunk;
    const int wt = (int)(rest % wg.nTile);
    const int band = (int)(rest / wg.nTile);
    const int64_t u0 = (int64_t)wt * TW;
    const int64_t h0 = g.h_lo + (int64_t)band * wg.TH, h1 = min(g.h_hi, h0 + wg.TH);
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    const int64_t dlo = window ? 0 : -(u0 + TW - 1);
    const int64_t d0 = dlo + (int64_t)chunk * 64;
    // full layout: a chunk with a voxel outside [0, W) for some tile row needs per-row masks
    const bool edge = !window && (u0 + d0 < 0 || u0 + TW - 1 + d0 + 63 >= g.W);
    if (edge)
        wave_body<K, T, true, false>(cam, proj, g, sc, sp, out, u0, h0, h1, d0, rowE, rowL, sM, sQ, sR);
    else if (window && wg.rem && chunk == wg.nChunk - 1)
        wave_body<K, T, false, true>(cam, proj, g, sc, sp, out, u0, h0, h1, d0, rowE, rowL, sM, sQ, sR);
    else
        wave_body<K, T, false, false>(cam, proj, g, sc, sp, out, u0, h0, h1, d0, rowE, rowL, sM, sQ, sR);
}

// Window layout, D + 1 <= 64 * kTileMaxChunks (+1): one workgroup per (column tile, row
// band) holding all diagonal chunks, wave w = chunk w (the last one also takes the
// remainder diagonal when wg.rem); outputs leave through the LDS block image (STAGED).
constexpr int kTileP = 2;  // load pipeline depth (steps; 3 measured no faster)
constexpr int kWaveLds = (3 * kRowP + 64) * 8 + kRowP * 4;  // rowE, rowL, sM, sR (f64) + sQ (f32)

template <int K, typename T, bool X4, int AMX = 0, bool CPL = false>
__global__ __launch_bounds__(64 * kTileMaxChunks) void k_fwd_tile(const T* __restrict__ cam,
                                                                 const T* __restrict__ proj, Geo g, Stats sc,
                                                                 Stats sp, float* __restrict__ out, WaveGrid wg,
                                                                 DispPartial part) {
    extern __shared__ __attribute__((aligned(16))) double lds_t[];
    const int w = (int)(threadIdx.x >> 6);
    const int64_t bid = xcd_remap(blockIdx.x, gridDim.x);
    const int wt = (int)(bid % wg.nTile), band = (int)(bid / wg.nTile);
    char* mine = (char*)lds_t + w * kWaveLds;
    double* rowE = (double*)mine;
    double* rowL = rowE + kRowP;
    double* sM = rowL + kRowP;
    double* sR = sM + kRowP;
    float* sQ = (float*)(sR + 64);
    float* stage = (float*)((char*)lds_t + wg.nChunk * kWaveLds);
    T* camL = (T*)(stage + 2 * TW * g.DO);  // CPL: the camera block after the two stage buffers
    const int64_t u0 = (int64_t)wt * TW;
    const int64_t h0 = g.h_lo + (int64_t)band * wg.TH, h1 = min(g.h_hi, h0 + wg.TH);
    const int64_t d0 = (int64_t)w * 64;
    if constexpr (AMX != 0) {  // the stage rows' padding columns (both buffers), once per workgroup
        for (int e = (int)threadIdx.x; e < 2 * TW * kAmxPitch; e += (int)blockDim.x)
            if (e % kAmxPitch >= (int)g.DO) stage[e] = -FLT_MAX;
    }
    // SS stores per thread cover the 16 DO-float block: DO <= 64 nChunk, or 64 nChunk + 1 (rem);
    // X4: 4 (5 with rem) 16-byte stores per thread
    constexpr int S0 = X4 ? -4 : TW, S1 = X4 ? -5 : TW + 1;
    constexpr int kTP = X4 ? kTileP : 2;  // deeper pipelines only with the 16-byte stores (vmcnt range)
    if (!wg.rem)
        wave_body<K, T, false, false, true, S0, kTP, AMX, CPL>(cam, proj, g, sc, sp, out, u0, h0, h1, d0, rowE,
                                                                         rowL, sM, sQ, sR, stage, part, camL);
    else if (w == wg.nChunk - 1)
        wave_body<K, T, false, true, true, S1, kTP, AMX, CPL>(cam, proj, g, sc, sp, out, u0, h0, h1, d0, rowE,
                                                                        rowL, sM, sQ, sR, stage, part, camL);
    else
        wave_body<K, T, false, false, true, S1, kTP, AMX, CPL>(cam, proj, g, sc, sp, out, u0, h0, h1, d0, rowE,
                                                                         rowL, sM, sQ, sR, stage, part, camL);
}

// CPL: fp16 images, when the camera block keeps the tile kernel at three workgroups per CU (LDS
// <= 160 KiB / 3).  Volume form: C5 9.81 -> 9.15 ms, C3 unchanged (profiles/r03/cpl); the fused
// disparity keeps its per-step camera loads (3 % slower with the preload).
template <int K, typename T>
size_t cpl_bytes(const WaveGrid& wg) {
    constexpr int NX = TW + K - 1;
    return ((size_t)(wg.TH + K - 1) * NX * sizeof(T) + 15) & ~(size_t)15;
}
template <int K, typename T>
bool cpl_ok(const Geo& g, const WaveGrid& wg, size_t lds) {
    (void)g;
    return sizeof(T) == 2 && lds + cpl_bytes<K, T>(wg) <= 163840 / 3;
}

template <int K, typename T>
hipError_t launch_k(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, float* out, hipStream_t s) {
    const WaveGrid wg = wave_grid(g);
    const bool tile = g.layout == CUSTMA_LAYOUT_WINDOW && wg.nChunk <= kTileMaxChunks;
    prof_begin(PROF_FWD, s);
    if (tile) {
        const int64_t blocks = (int64_t)wg.nBand * wg.nTile;
        size_t lds = (size_t)wg.nChunk * kWaveLds + 2 * TW * (size_t)g.DO * 4;
        const bool cpl = cpl_ok<K, T>(g, wg, lds);
        if (cpl) lds += cpl_bytes<K, T>(wg);
        // 16-byte stores when every block base is 16-byte aligned: out aligned and
        // ((t - h_lo) WO + u0) DO = 0 mod 4 for all t (u0 = 0 mod 16)
        const bool x4 = ((uintptr_t)out % 16 == 0) && (g.WO % 4 == 0 || g.DO % 4 == 0);
        const dim3 blk(64 * wg.nChunk);
        if (x4 && cpl) {
            if constexpr (sizeof(T) == 2)
                hipLaunchKernelGGL((k_fwd_tile<K, T, true, 0, true>), dim3((unsigned)blocks), blk, lds, s, cam, proj, g,
                                   sc, sp, out, wg, DispPartial{});
        } else if (x4)
            hipLaunchKernelGGL((k_fwd_tile<K, T, true>), dim3((unsigned)blocks), blk, lds, s, cam, proj, g, sc, sp,
                               out, wg, DispPartial{});
        else
            hipLaunchKernelGGL((k_fwd_tile<K, T, false>), dim3((unsigned)blocks), blk, lds, s, cam, proj, g, sc, sp,
                               out, wg, DispPartial{});
    } else {
        const int64_t blocks = (int64_t)wg.nBand * wg.nTile * wg.nChunk;
        hipLaunchKernelGGL((k_fwd_wave<K, T>), dim3((unsigned)blocks), dim3(64), 0, s, cam, proj, g, sc, sp, out,
                           wg);
    }
    prof_end(PROF_FWD, s);
    return hipGetLastError();
}

// Fused disparity through the tile kernel (window layout, D + 1 <= 257): one partial per pixel.
template <int K, typename T>
hipError_t launch_amx(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, DispPartial part, hipStream_t s) {
    const WaveGrid wg = wave_grid(g, /*disparity=*/true);
    const int64_t blocks = (int64_t)wg.nBand * wg.nTile;
    // (no camera preload here: it measured slower, C5 9.69 -> 9.99 ms, C3 1.15 -> 1.18 ms)
    const size_t lds = (size_t)wg.nChunk * kWaveLds + 2 * TW * (size_t)kAmxPitch * 4;
    prof_begin(PROF_FWD, s);
    const int passes = wg.nChunk == 4 ? 1 : wg.nChunk >= 2 ? 2 : 4;  // 16 rows over the waves, 4 per pass
    auto go = [&](auto amx) {
        hipLaunchKernelGGL((k_fwd_tile<K, T, false, decltype(amx)::value>), dim3((unsigned)blocks),
                           dim3(64 * wg.nChunk), lds, s, cam, proj, g, sc, sp, nullptr, wg, part);
    };
    const bool soft = part.s0 != nullptr;  // soft-argmax sums requested
    if (passes == 1) soft ? go(std::integral_constant<int, -1>{}) : go(std::integral_constant<int, 1>{});
    else if (passes == 2) soft ? go(std::integral_constant<int, -2>{}) : go(std::integral_constant<int, 2>{});
    else soft ? go(std::integral_constant<int, -4>{}) : go(std::integral_constant<int, 4>{});
    prof_end(PROF_FWD, s);
    return hipGetLastError();
}

}  // namespace

template <int K>
hipError_t sw_fwd(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, float* out,
                  hipStream_t s) {
    if (dtype == CUSTMA_F16) return launch_k<K, __half>((const __half*)cam, (const __half*)proj, g, sc, sp, out, s);
    return launch_k<K, float>((const float*)cam, (const float*)proj, g, sc, sp, out, s);
}
template <int K>
hipError_t sw_amx(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, DispPartial part,
                  hipStream_t s) {
    if (dtype == CUSTMA_F16) return launch_amx<K, __half>((const __half*)cam, (const __half*)proj, g, sc, sp, part, s);
    return launch_amx<K, float>((const float*)cam, (const float*)proj, g, sc, sp, part, s);
}
#ifdef CUSTMA_SW_K
template hipError_t sw_fwd<CUSTMA_SW_K>(const void*, const void*, int, const Geo&, Stats, Stats, float*, hipStream_t);
template hipError_t sw_amx<CUSTMA_SW_K>(const void*, const void*, int, const Geo&, Stats, Stats, DispPartial,
                                        hipStream_t);
#endif

#else  // CUSTMA_SW_DISPATCH


WaveGrid wave_grid(const Geo& g, bool disparity) {
    WaveGrid wg;
    const int64_t nd = g.layout == CUSTMA_LAYOUT_WINDOW ? (int64_t)g.D + 1 : g.W + TW - 1;
    wg.nChunk = (int)cdiv(nd, 64);
    // window with (D+1) % 64 == 1 (D = 64 n): the last full chunk's waves also compute the
    // single remainder diagonal D (no fifth, nearly idle chunk of waves)
    wg.rem = g.layout == CUSTMA_LAYOUT_WINDOW && nd > 64 && nd % 64 == 1;
    if (wg.rem) --wg.nChunk;
    wg.nTile = (int)cdiv(g.WO, TW);
#ifndef CUSTMA_WAVE_TH
#define CUSTMA_WAVE_TH 64
#endif
    wg.TH = CUSTMA_WAVE_TH;  // band height (32 / 128 measured within 2 %; A/B builds set CUSTMA_WAVE_TH)
    // keep >= ~8 waves per SIMD on small problems
    while (wg.TH > 8 && (int64_t)wg.nTile * wg.nChunk * cdiv(g.HV(), wg.TH) < 8192) wg.TH /= 2;
    // (a tail-balanced band height -- the one with the fewest rounds x (TH + k - 1) steps on 3 workgroups per
    // CU, TH = 61 at C3 -- measured no faster for the volume and 1.7 % slower for the disparity, round 6:
    // profiles/r06/g)
    // The fused disparity on large grids (>= 16 rounds of 128-row bands on 3 workgroups per CU of a 256-CU
    // part: configs[4]'s whole image) takes 128-row bands, half the K - 1 warm-up steps per output row: C5
    // disparity 9.69 -> 9.50 ms; C3 unchanged, a C5 rank band 1.45 -> 1.61 ms and every volume forward slower
    // at 128 (profiles/r06/ab), so those keep 64.
    if (disparity && wg.TH == 64 && (int64_t)wg.nTile * cdiv(g.HV(), 128) >= 16 * 3 * 256) wg.TH = 128;
    wg.nBand = (int)cdiv(g.HV(), wg.TH);
    return wg;
}

bool disp_tile_ok(const Geo& g) {
    return g.layout == CUSTMA_LAYOUT_WINDOW && wave_grid(g).nChunk <= kTileMaxChunks;
}

hipError_t launch_disp_tile(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            DispPartial part, hipStream_t s) {
    switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: return sw_amx<KK>(cam, proj, dtype, g, sc, sp, part, s);
        CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fwd_fast(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                           float* out, hipStream_t s) {
    // Full layout: the workgroup form (loader wave + LDS-staged, sector-owned stores) is
    // faster -- this kernel's direct stores split 64-byte sectors between chunks there (C2:
    // 1.35 vs 1.47 ms, WRITE_SIZE +10 %).  CUSTMA_FWD_LDS=0/1 overrides (benchmarking only).
    const char* e = getenv("CUSTMA_FWD_LDS");
    const bool lds = e ? atoi(e) != 0 : g.layout != CUSTMA_LAYOUT_WINDOW;
    if (lds) return launch_fwd_lds(cam, proj, dtype, g, sc, sp, out, s);
    switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: return sw_fwd<KK>(cam, proj, dtype, g, sc, sp, out, s);
        CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
        default: return hipErrorInvalidValue;
    }
}
#endif  // CUSTMA_SW_DISPATCH

}  // namespace custma
