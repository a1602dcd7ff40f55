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

typedef __attribute__((address_space(3))) volatile double lds_vd;
constexpr int kFwdNST = 2;  // loader register stages (x loads per step <= 63 + one step)
#ifndef CUSTMA_SWEEP_AUX
#define CUSTMA_SWEEP_AUX kStoreAux
#endif
constexpr int kSweepAux = CUSTMA_SWEEP_AUX;  // volume store policy (A/B builds set CUSTMA_SWEEP_AUX)


// X4 (volume form, D_out a multiple of 16, a 16-byte aligned volume): every chunk's owned columns of a row are
// whole 64-byte sectors (sweep.h owned chunks, beta = 0), so the step's 16 x S owned floats leave as 16-byte
// stores, a lane taking up to 4 groups of 4 consecutive columns instead of 16 dword stores.  The staging rows
// are padded (pitch NL + 4) and row m shifted by (m + 1) & 3 floats (full layout), which puts every group on
// a 16-byte LDS boundary: one conflict-free ds_read_b128 per group.  (Round 6's first form read each group as
// four ds_read_b32 at a 16-byte lane stride -- bank conflicts -- and measured slower than the dword stores,
// profiles/r06/b; the bare store patterns: 0.954 ms dword vs 0.850 ms x4 at C2 full, profiles/r06/d.)
template <int K, int TWT, typename T, bool ARGMAX, bool X4 = false>
__global__ __launch_bounds__(384) void k_sweep_fwd(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                   Stats sc, Stats sp, float* __restrict__ out, SweepGrid sg,
                                                   DispPartial part) {
    // taps rows h - R0 .. h + R1, columns w - R0 .. w + R1 (R0 = K/2, R1 = K-1-K/2: the reference's
    // kernel_size / 2 origin, stereo_matching_kernel.cu:44,60)
    constexpr int R0 = K / 2, R1 = K - 1 - K / 2, NX = TWT + K - 1;
    static_assert(TWT == 16 && NX <= 48, "row-broadcast layout assumes 16 own columns and <= 48 camera columns");
    constexpr int NL_MAX = 320, LO = (NX + NL_MAX - 1 + 63) / 64, LS = (TWT + NL_MAX - 1 + 63) / 64;
    const int NL = sg.NL, NO = NX + NL - 1, NS = TWT + NL - 1;
    const int NLS = X4 ? NL + 4 : NL;  // staging row pitch of the volume form
    // LDS rows are padded to whole loader-lane chunks (OP = 64 LO, SP = 64 LS), so the loader
    // writes every lane of every chunk unconditionally (the padding takes zeros / ignored
    // values): its step is straight-line code, which keeps three steps of loads in flight
    constexpr int OP = 64 * LO, SP = 64 * LS;
    extern __shared__ __attribute__((aligned(16))) double ldsd[];
    double* ringO = ldsd;                  // [2 buf][2 enter/leave][OP] projector rows
    double* ringU = ringO + 4 * OP;        // [2 buf][2][64]: +c of the entering row, -c of the leaving row
    double* rsM = ringU + 4 * 64;          // [2][SP]  projector fp64 patch means
    double* usB = rsM + 2 * SP;            // [2][64]  -(camera fp64 patch sums) (lanes 0-15)
    float* rsQ = (float*)(usB + 2 * 64);   // [2][SP]  projector ey2
    float* usQ = rsQ + 2 * SP;             // [2][64]  camera ex2 (lanes 0-15)
    float* stg = usQ + 2 * 64;             // [2][16][NLS] cost tile staging (ARGMAX: [16][NL] reduction)

    const int64_t bid = xcd_remap(blockIdx.x, gridDim.x);
    const int chunk = (int)(bid % sg.nChunk);
    const int64_t rest = bid / sg.nChunk;
    const int wt = (int)(rest % sg.nTile);
    const int band = (int)(rest / sg.nTile);
    const int64_t u0 = (int64_t)wt * TWT;
    const int64_t h0 = g.h_lo + (int64_t)band * sg.TH, h1 = min(g.h_hi, h0 + sg.TH);
    const int64_t hs = h0 - (K - 1);  // first step: K - 1 warm-up steps fill the column sums
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    const int64_t dlo = window ? 0 : -(u0 + TWT - 1);
    const int64_t dhi = window ? g.D : g.W - 1 - u0;
    const int64_t d0 = dlo + (int64_t)chunk * sg.S;
    const int tid = threadIdx.x;
    // The last wave of the workgroup is the loader: it stages image rows and statistics
    // into LDS a step ahead and never stores to HBM.  The other waves compute and store
    // and never load from HBM.  (vmcnt counts loads and stores in issue order, so a wave
    // doing both waits for its earlier volume stores whenever it consumes a load.)
    const bool loader = __builtin_amdgcn_readfirstlane(tid) >= NL;
    if constexpr (ARGMAX) {
        // the reduction rows' padding columns NL .. NLP - 1 (NLP below), ordered before the scans by barrier #0
        int TPR = 1;
        while (TPR * 2 * TWT <= NL && TPR < 16) TPR *= 2;
        const int NLP = NL + TPR;
        for (int e = tid; e < TWT * NLP; e += (int)blockDim.x)
            if (e % NLP >= NL) stg[e] = -FLT_MAX;
    }
    const double rk2 = 1.0 / (double)(K * K);
    constexpr uint32_t OOB = 0x80000000u;

    if (loader) {
        // ---- branch-free raw buffer loads (out-of-range -> 0 = the reference's zero
        // padding, stereo_matching_kernel.cu:6-12): loop-invariant per-lane byte offsets,
        // the row chosen by the descriptor (zero-size for rows outside the image) ----
        const int li = tid - NL;
        const int64_t xU0 = u0 - R0, xO0 = u0 - R0 + d0, oS = u0 + d0;
        auto colOff = [&](bool have, int64_t x, int esz) -> uint32_t {
            return (have && x >= 0 && x < g.W) ? (uint32_t)(x * esz) : OOB;
        };
        auto row_rsrc = [&](const void* base, int64_t row, int esz, bool ok) {
            ok = ok && row >= 0 && row < g.H;
            return make_rsrc_sgpr((const char*)base + (ok ? row : 0) * g.W * esz, ok ? (uint32_t)(g.W * esz) : 0u);
        };
        uint32_t vO[LO], vSd[LS], vSf[LS];
        const uint32_t vUe = colOff(li < NX, xU0 + li, sizeof(T));  // the leaving row: the same columns
        const uint32_t vUSd = colOff(li < TWT, u0 + li, 8), vUSf = colOff(li < TWT, u0 + li, 4);
#pragma unroll
        for (int j = 0; j < LO; ++j) vO[j] = colOff(li + 64 * j < NO, xO0 + li + 64 * j, sizeof(T));
#pragma unroll
        for (int j = 0; j < LS; ++j) {
            vSd[j] = colOff(li + 64 * j < NS, oS + li + 64 * j, 8);
            vSf[j] = colOff(li + 64 * j < NS, oS + li + 64 * j, 4);
        }
        // Raw bits only: nothing consumes a load in the step that issues it, and every load is
        // unconditional (unused lanes / chunks carry the out-of-range offset), so the loads of
        // three steps stay in flight (the compiler's vmcnt waits only for the oldest stage).
        constexpr int NST = kFwdNST;
        struct Stage {
            uint32_t ue, ul, oe[LO], ol[LO], q[LS], uq;
            double m[LS], ub;
        };
        // step t adds image row t+R1 and removes row t-R0-1 (once it was added: rows from
        // h0-R0 on are added, so the first removal is at t = h0+1)
        auto load_step = [&](int64_t t, Stage& p) {
            const bool rem = t > h0;
            const auto rCe = row_rsrc(cam, t + R1, sizeof(T), true), rCl = row_rsrc(cam, t - R0 - 1, sizeof(T), rem);
            const auto rPe = row_rsrc(proj, t + R1, sizeof(T), true), rPl = row_rsrc(proj, t - R0 - 1, sizeof(T), rem);
            asm_ld_raw<T>(p.ue, vUe, rCe);
            asm_ld_raw<T>(p.ul, vUe, rCl);
#pragma unroll
            for (int j = 0; j < LO; ++j) {
                asm_ld_raw<T>(p.oe[j], vO[j], rPe);
                asm_ld_raw<T>(p.ol[j], vO[j], rPl);
            }
            const bool st = t >= h0 && t < h1;
            const auto rPB = row_rsrc(sp.box, t, 8, st), rPS = row_rsrc(sp.sq, t, 4, st);
            const auto rCB = row_rsrc(sc.box, t, 8, st), rCS = row_rsrc(sc.sq, t, 4, st);
#pragma unroll
            for (int j = 0; j < LS; ++j) {
                asm_ld_f64(p.m[j], vSd[j], rPB);
                asm_ld_raw<float>(p.q[j], vSf[j], rPS);
            }
            asm_ld_f64(p.ub, vUSd, rCB);
            asm_ld_raw<float>(p.uq, vUSf, rCS);
        };
        constexpr int kLoadsPerStep = 4 + 2 * LO + 2 * LS;
        // the oldest stage has landed once at most (NST - 1) steps of loads are outstanding
        auto wait_oldest = [&](Stage& p) {
            asm_vmcnt<kLoadsPerStep * (NST - 1)>();
            asm_tie(p.ue);
            asm_tie(p.ul);
            asm_tie(p.uq);
            asm_tie(p.ub);
#pragma unroll
            for (int j = 0; j < LO; ++j) { asm_tie(p.oe[j]); asm_tie(p.ol[j]); }
#pragma unroll
            for (int j = 0; j < LS; ++j) { asm_tie(p.m[j]); asm_tie(p.q[j]); }
        };
        auto store_step = [&](int b, const Stage& p) {
            ringU[(2 * b) * 64 + li] = raw_to_f64<T>(p.ue);  // 0 past NX
            ringU[(2 * b + 1) * 64 + li] = -raw_to_f64<T>(p.ul);
#pragma unroll
            for (int j = 0; j < LO; ++j) {
                ringO[(2 * b) * OP + li + 64 * j] = raw_to_f64<T>(p.oe[j]);
                ringO[(2 * b + 1) * OP + li + 64 * j] = raw_to_f64<T>(p.ol[j]);
            }
#pragma unroll
            for (int j = 0; j < LS; ++j) {
                rsM[b * SP + li + 64 * j] = p.m[j] * rk2;
                rsQ[b * SP + li + 64 * j] = __builtin_bit_cast(float, p.q[j]);
            }
            usB[b * 64 + li] = -p.ub;
            usQ[b * 64 + li] = __builtin_bit_cast(float, p.uq);
        };
        // NST register stages: the loads of step hs+s are issued in iteration s-NST and
        // stored to LDS in iteration s (vmcnt counts at most 63 loads in flight: NST x the
        // loads of one step must stay below that, or the compiler waits for all of them).  The
        // warm-up iterations (s < 0) run the same loop body with the LDS store and the
        // barrier skipped: no loads are issued outside the loop, so the loop-header state
        // the compiler's vmcnt tracking sees is the loop's own (a peeled prologue with a
        // different register assignment made it wait for the newest loads every iteration).
        // Iteration s >= 0 ends with barrier #s: compute step hs+s-1 ends with it (#0: the
        // first stage), and the loader issues as many barriers as the compute waves.
        Stage st[NST];
        const int n = (int)(h1 - hs);
        auto step = [&](auto kc, int s) {
            constexpr int k = decltype(kc)::value;  // == (s + NST) % NST
            // the wait outside the test (at s < 0 it finds nothing older in flight): no path of the
            // emitted code skips it, so vmcnt_check.py can prove it
            wait_oldest(st[k]);
            if (s >= 0) store_step(s & 1, st[k]);
            load_step(hs + s + NST, st[k]);  // past the band's end: harmless, unused
            if (s >= 0) {
                if constexpr (ARGMAX) {
                    if (s >= 1 && hs + s - 1 >= h0) __syncthreads();
                }
                __syncthreads();
            }
        };
        // opaque start: the compiler must not peel the warm-up iterations into a prologue
        int s_first = -NST;
        asm volatile("" : "+s"(s_first));
        for (int s = s_first;; s += NST) {
            bool done = false;
            Unroll<0, NST>::run([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                if (done) return;
                step(kc, s + k);
                done = s + k >= n;
            });
            if (done) break;
        }
        if constexpr (!ARGMAX) __syncthreads();  // the compute waves' final store phase
        return;
    }

    // ---- compute waves: lane tid owns diagonal delta = d0 + tid ----
    const int64_t delta = d0 + tid;
    int m_lo = TWT, m_hi = 0;  // valid camera-column offsets m in [m_lo, m_hi) (ARGMAX)
    if (delta >= dlo && delta <= dhi) {
        const int64_t lo = max((int64_t)0, -delta - u0);
        const int64_t hi = min((int64_t)TWT, min(g.W - u0 - delta, g.WO - u0));
        m_lo = (int)lo;
        m_hi = (int)max(lo, hi);
    }
    double col[NX];
#pragma unroll
    for (int x = 0; x < NX; ++x) col[x] = 0.0;
    const int r16 = tid & 15;
    // col[x] += c(enter, x) p(enter, x + delta) - c(leave, x) p(leave, x + delta)
    auto update = [&](int b) {
        const double* ue = ringU + (2 * b) * 64;
        const double* ul = ringU + (2 * b + 1) * 64;  // negated
        const double ca0 = ue[r16], ca1 = ue[16 + r16], ca2 = NX > 32 ? ue[32 + r16] : 0.0;
        const double cb0 = ul[r16], cb1 = ul[16 + r16], cb2 = NX > 32 ? ul[32 + r16] : 0.0;
        // volatile: keeps these as single ds_read_b64 (2 LDS cycles per wave-instruction)
        // instead of pairs merged into ds_read2_b64 (8 cycles, half the bandwidth)
        const lds_vd* oa = (const lds_vd*)(ringO + (2 * b) * OP + tid);
        const lds_vd* ob = (const lds_vd*)(ringO + (2 * b + 1) * OP + tid);
        // batches of B columns, double-buffered: batch b+1's reads are in flight while
        // batch b's FMAs issue (an asm statement is a scheduling boundary)
        constexpr int B = 4, NB = (NX + B - 1) / B;
        double pa[2][B], pb[2][B];
        auto fetch = [&](auto bc) {
            constexpr int bb = decltype(bc)::value, x0 = bb * B;
            constexpr int nb = NX - x0 < B ? NX - x0 : B;
            Unroll<0, nb>::run([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                pa[bb & 1][i] = oa[x0 + i];
                pb[bb & 1][i] = ob[x0 + i];
            });
        };
        fetch(std::integral_constant<int, 0>{});
        Unroll<0, NB>::run([&](auto bc) {
            constexpr int bb = decltype(bc)::value, x0 = bb * B;
            constexpr int nb = NX - x0 < B ? NX - x0 : B;
            if constexpr (bb + 1 < NB) fetch(std::integral_constant<int, bb + 1>{});
            Unroll<0, nb>::run([&](auto ic) {
                constexpr int i = decltype(ic)::value, x = x0 + i;
                fmac_bc64<(x & 15)>(col[x], x < 16 ? ca0 : x < 32 ? ca1 : ca2, pa[bb & 1][i]);
                fmac_bc64<(x & 15)>(col[x], x < 16 ? cb0 : x < 32 ? cb1 : cb2, pb[bb & 1][i]);
            });
        });
    };

    // ---- store phase: the previous step's staged tile, written so that every 64-byte
    // sector of the volume is covered by one store instruction of one workgroup.  Row m
    // of the tile, chunk c: owned columns [cb, cb + len) (sweep.h), lane tid stores column
    // cb + tid; a per-row descriptor of len columns drops the lanes past the range ----
    const int DO = (int)g.DO;
    auto bound = [&](int c, int beta) -> int {  // first owned column of chunk c in a row
        if (c <= 0) return 0;
        if (c >= sg.nChunk) return DO;
        const int x = c * sg.S;
        return min(DO, x + ((16 - ((beta + x) & 15)) & 15));
    };
    // Sector phase of each volume row of the tile: the same for every row band step when
    // WO*DO is a multiple of 16 (then computed once); otherwise the chunks split at c*S
    // (S is a multiple of 16) -- still a partition, only not sector aligned.
    // Per lane and tile row m: byte offset of its volume element inside the row tile
    // (out of range for lanes past the owned columns); the staging slot of that element
    // is the same offset plus a per-row constant.
    uint32_t voff[X4 ? 1 : TWT];
    if constexpr (!X4) {
        const bool phase_fixed = ((g.WO * g.DO) & 15) == 0;
        const int r0 = (int)((((h0 - g.h_lo) * g.WO + u0)) & 15), dm = phase_fixed ? DO & 15 : 0;
#pragma unroll
        for (int m = 0; m < TWT; ++m) {
            const int beta = ((r0 + m) * dm) & 15;
            const int cb = bound(chunk, beta), ce = bound(chunk + 1, beta);
            const bool ok = u0 + m < g.WO && cb + tid < ce;
            voff[m] = ok ? (uint32_t)((m * DO + cb + tid) * 4) : OOB;
        }
    }
    // staging index of column c in row m: m*NL + c - d0 - (u0 + m) (full) / m*NL + c - d0
    // (window); with c = voff/4 - m*DO that is voff/4 + m*stgA + stgB
    const int stgA = NL - DO - (window ? 0 : 1), stgB = -(int)d0 - (window ? 0 : (int)u0);
    // X4: staging row m starts (m + 1) & 3 floats in (full layout; window: 0), so that the 4-column groups,
    // which start on owned sector boundaries, sit on 16-byte LDS boundaries
    auto stg_shift = [&](int m) { return window ? 0 : ((m + 1) & 3); };
    constexpr int NG = X4 ? TWT / 4 : 1;  // groups per lane: ceil(TWT S / (4 NL)) <= TWT / 4 (S <= NL)
    uint32_t gvo[NG], gso[NG];
    if constexpr (X4) {
        const int gpr = sg.S / 4, cb = bound(chunk, 0), ce = bound(chunk + 1, 0);
#pragma unroll
        for (int i = 0; i < NG; ++i) {
            const int q = tid + NL * i, m = q / gpr, c = cb + 4 * (q - m * gpr);
            const bool ok = m < TWT && u0 + m < g.WO && c < ce;
            gvo[i] = ok ? (uint32_t)((m * DO + c) * 4) : OOB;
            gso[i] = ok ? (uint32_t)((m * NLS + stg_shift(m) + c - (int)d0 - (window ? 0 : (int)u0 + m)) * 4) : 0u;
        }
    }
    auto store_tile = [&](int64_t h, int b) {
        const auto rOut = make_rsrc(out + ((h - g.h_lo) * g.WO + u0) * g.DO, 0x7FFFFFF0u);
        const char* tile = (const char*)(stg + b * 16 * NLS);
        if constexpr (X4) {
            i32x4 v[NG];
#pragma unroll
            for (int i = 0; i < NG; ++i) v[i] = *(const i32x4*)(tile + gso[i]);
#pragma unroll
            for (int i = 0; i < NG; ++i) __builtin_amdgcn_raw_buffer_store_b128(v[i], rOut, gvo[i], 0u, kSweepAux);
        } else {
            float v[TWT];
#pragma unroll
            for (int m = 0; m < TWT; ++m) v[m] = *(const float*)(tile + voff[m] + 4 * (m * stgA + stgB));
#pragma unroll
            for (int m = 0; m < TWT; ++m)
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v[m]), rOut, voff[m], 0,
                                                      kSweepAux);
        }
    };

    __syncthreads();  // the loader's first stage
    for (int64_t h = hs; h < h1; ++h) {
        const int buf = (int)((h - hs) & 1);
        if constexpr (!ARGMAX) {
            if (h > h0) store_tile(h - 1, buf ^ 1);
        }
        update(buf);
        if (h >= h0) {
            double s = col[0] + (double)kEps;  // E + eps: eps rides along the sliding sum
#pragma unroll
            for (int x = 1; x < K; ++x) s += col[x];
            const lds_vd* mrow = (const lds_vd*)(rsM + buf * SP + tid);
            const float* qrow = rsQ + buf * SP + tid;
            const double nb = usB[buf * 64 + r16];  // -(camera patch sum) of column r16
            const float uq = usQ[buf * 64 + r16];   // camera ex2 of column r16
            double mv[TWT];
            float qv[TWT];
#pragma unroll
            for (int m = 0; m < TWT; ++m) { mv[m] = mrow[m]; qv[m] = qrow[m]; }
            // ARGMAX: tile rows at pitch NL + TPR (the reduction's TPR-lane groups read column m's row
            // at banks m TPR + lane: conflict-free)
            int TPR = 1;
            while (TPR * 2 * TWT <= NL && TPR < 16) TPR *= 2;
            const int NLP = ARGMAX ? NL + TPR : NL;
            float* srow = stg + (ARGMAX ? 0 : buf * 16 * NLS) + tid;
            Unroll<0, TWT>::run([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                if (m > 0) s = (s + col[m + K - 1]) - col[m - 1];
                double e = s;
                fmac_bc64<m>(e, nb, mv[m]);                 // E + eps = S + eps - box_c * mean_p
                float den2 = kEps;
                fmac_bc32<m>(den2, uq, qv[m]);              // ex2 * ey2 + eps
                const float c = (float)e * __builtin_amdgcn_rsqf(den2);
                if constexpr (ARGMAX) {
                    srow[m * NLP] = (m >= m_lo && m < m_hi) ? c : -FLT_MAX;
                } else if constexpr (X4) {
                    srow[m * NLS + stg_shift(m)] = c;
                } else {
                    srow[m * NL] = c;
                }
            });
            if constexpr (ARGMAX) {
                __syncthreads();
                // TPR lanes per camera column (a power of two, TPR x 16 <= NL)
                const int m = tid / TPR, part_i = tid % TPR;
                const bool red_live = m < TWT;
                const bool soft = part.s0 != nullptr;
                // layout index s of diagonal lane l for camera column u0 + m
                const float sbase = (float)(window ? d0 : u0 + m + d0);
                const float* rowp = stg + (red_live ? m : 0) * NLP;
                // nsc diagonals per lane, no bound test: the row's columns NL .. NLP - 1 hold -FLT_MAX
                // (written once, below the loader split), which changes none of the results, so the LDS
                // reads batch up instead of one exec-masked, waited read per element.
                const int nsc = (NL + TPR - 1) / TPR;
                auto mvf = [&](float x, auto ctl) {
                    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x),
                                                                                 decltype(ctl)::value, 0xf, 0xf, false));
                };
                typedef std::integral_constant<int, 0xB1> X1;   // quad_perm [1,0,3,2]
                typedef std::integral_constant<int, 0x4E> X2;   // quad_perm [2,3,0,1]
                typedef std::integral_constant<int, 0x141> HM;  // row_half_mirror
                typedef std::integral_constant<int, 0x140> RM;  // row_mirror
                // the TPR lanes of a column combined by DPP (quad xor 1, xor 2, half-row mirror, row mirror:
                // each lane meets every other lane's part once)
                auto over_tpr = [&](auto f) {
                    if (TPR >= 2) f(X1{});
                    if (TPR >= 4) f(X2{});
                    if (TPR >= 8) f(HM{});
                    if (TPR >= 16) f(RM{});
                };
                float best = -FLT_MAX, second = -FLT_MAX, q0 = 0.f, q1 = 0.f;
                int bi = 0x7fffffff;
                if (soft) {
                    // Two passes (round 6, as the tile kernel's soft scan, sweep_wave.hip): the top two values
                    // by v_max / v_med3, then the first diagonal holding the best and the soft sums weighted
                    // relative to it (no running rescale).  C2 full soft 2.58 -> 2.27 ms; the plain argmax
                    // keeps the one-pass scan (two passes: 1.84 -> 2.07 ms, profiles/r06/c).
#pragma unroll 4
                    for (int e = 0; e < nsc; ++e) {
                        const float v = red_live ? rowp[part_i + TPR * e] : -FLT_MAX;
                        second = __builtin_amdgcn_fmed3f(best, second, v);  // best >= second: the new second
                        best = __builtin_fmaxf(best, v);
                    }
                    over_tpr([&](auto ctl) {
                        const float ob = mvf(best, ctl), os = mvf(second, ctl);
                        second = __builtin_amdgcn_fmed3f(best, ob, __builtin_fmaxf(second, os));  // top two of four
                        best = __builtin_fmaxf(best, ob);
                    });
                    int fe = 0x7fffffff;  // the first e with row[part_i + TPR e] == best (this lane)
                    float qe = 0.f;       // sum of e w (w = exp2(kb (v - best)); q0 = sum of w)
                    const float nkb = best > -FLT_MAX ? -part.kb * best : 0.f;  // (no value: every w = 0)
#pragma unroll 4
                    for (int e = nsc - 1; e >= 0; --e) {
                        const float v = red_live ? rowp[part_i + TPR * e] : -FLT_MAX;
                        fe = v == best ? e : fe;
                        const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(part.kb, v, nkb));
                        q0 += w;
                        qe = __builtin_fmaf(w, (float)e, qe);
                    }
                    bi = fe == 0x7fffffff || !(best > -FLT_MAX) ? 0x7fffffff : part_i + TPR * fe;
                    // sum over the lane's diagonals of s w, s = sbase + part_i + TPR e
                    q1 = __builtin_fmaf(sbase + (float)part_i, q0, (float)TPR * qe);
                    over_tpr([&](auto ctl) {
                        bi = min(bi, __builtin_amdgcn_update_dpp(0, bi, decltype(ctl)::value, 0xf, 0xf, false));
                        q0 += mvf(q0, ctl);
                        q1 += mvf(q1, ctl);
                    });
                } else {
                    // one pass: each lane scans its diagonals in increasing order (branch-free: the strict
                    // compare keeps the first index among equal values; the top two by v_med3 / v_max:
                    // C2 full 1.79 -> 1.76 ms, profiles/r06/f)
#pragma unroll 4
                    for (int e = 0; e < nsc; ++e) {
                        const int l = part_i + TPR * e;
                        const float v = red_live ? rowp[l] : -FLT_MAX;
                        const bool gt = v > best;
                        bi = gt ? l : bi;
                        second = __builtin_amdgcn_fmed3f(best, second, v);  // best >= second: the new second
                        best = __builtin_fmaxf(best, v);
                    }
                    over_tpr([&](auto ctl) {
                        const float ob = mvf(best, ctl), os = mvf(second, ctl);
                        const int oi = __builtin_amdgcn_update_dpp(0, bi, decltype(ctl)::value, 0xf, 0xf, false);
                        if (ob > best || (ob == best && oi < bi)) {
                            second = fmaxf(os, best);
                            best = ob;
                            bi = oi;
                        } else {
                            second = fmaxf(second, ob);
                        }
                    });
                }
                const int64_t u = u0 + m;
                if (red_live && part_i == 0 && u < g.WO) {
                    const int64_t pidx = ((int64_t)chunk * g.HV() + (h - g.h_lo)) * g.WO + u;
                    part.best[pidx] = best;
                    part.second[pidx] = second;
                    int64_t sidx = -1;
                    if (best > -FLT_MAX) {
                        const int64_t dd = d0 + bi;
                        sidx = window ? dd : u + dd;
                    }
                    part.index[pidx] = (int32_t)sidx;
                    if (soft) {
                        part.s0[pidx] = q0;
                        part.s1[pidx] = q1;
                    }
                }
            }
        }
        __syncthreads();
    }
    if constexpr (!ARGMAX) {
        if (h1 > h0) store_tile(h1 - 1, (int)((h1 - 1 - hs) & 1));
        __syncthreads();
    }
}

template <int K, typename T>
hipError_t launch_k(const T* cam, const T* proj, const Geo& g, Stats sc, Stats sp, float* out,
                    DispPartial* part, hipStream_t s) {
    // (per-lane 256-byte stores straight from registers, one chunk of all D+1 diagonals of a window,
    // measured slower: 2.56 vs 2.34 ms at 2048^2, D = 256, k = 11)
    const SweepGrid sg = sweep_grid(g, /*owned=*/part == nullptr);
    constexpr int NX = TW + K - 1;
    constexpr int NL_MAX = 320, OP = 64 * ((NX + NL_MAX - 1 + 63) / 64), SP = 64 * ((TW + NL_MAX - 1 + 63) / 64);
    const int NL = sg.NL;
    const size_t lds = sizeof(double) * (4 * OP + 4 * 64 + 2 * SP + 2 * 64) +
                       sizeof(float) * (2 * SP + 2 * 64 + (part ? TW * (NL + 16) : 2 * TW * (NL + 4)));
    const int64_t blocks = sweep_blocks(sg);
    if (part) {
        hipLaunchKernelGGL((k_sweep_fwd<K, TW, T, true>), dim3((unsigned)blocks), dim3(NL + 64), lds, s, cam,
                           proj, g, sc, sp, out, sg, *part);
    } else {
        DispPartial none{};
        // 16-byte stores: every owned segment starts on a 64-byte sector (D_out % 16 == 0, so beta = 0 in every
        // row) of a 16-byte aligned volume
#ifdef CUSTMA_SWEEP_NO_X4
        const bool x4 = false;  // A/B build (scripts/build_ablations.py sweep_dword)
#else
        const bool x4 = g.DO % 16 == 0 && (uintptr_t)out % 16 == 0 && sg.S % 16 == 0;
#endif
        prof_begin(PROF_FWD, s);
        if (x4)
            hipLaunchKernelGGL((k_sweep_fwd<K, TW, T, false, true>), dim3((unsigned)blocks), dim3(NL + 64), lds, s, cam,
                               proj, g, sc, sp, out, sg, none);
        else
            hipLaunchKernelGGL((k_sweep_fwd<K, TW, T, false>), dim3((unsigned)blocks), dim3(NL + 64), lds, s, cam,
                               proj, g, sc, sp, out, sg, none);
        prof_end(PROF_FWD, s);
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

hipError_t launch_fwd_lds(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
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
