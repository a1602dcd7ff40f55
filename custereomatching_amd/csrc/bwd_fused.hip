// Backward: gradients of sum(grad * volume) w.r.t. both images in ONE pass
// over the incoming gradient volume (deterministic, no atomics).
//
// The reference (custma/src/stereo_matching_kernel.cu:75-179) forms, per
// voxel and tap t, g * (y_t / S - Y x_t (E+eps) / S^3) and scatters it with
// float atomics (k^2 recomputed taps + k^2 atomics per voxel).  Summed over
// voxels, with A = g / S and V = g (E+eps) / S^3 = A * cost / S (`cost` = the
// forward's output), the gradients split into per-diagonal box sums:
//
//   dC(y,x) = T1c(y,x) - Box[Am](y,x) - c'(y,x) Box[B](y,x)  + Box[mc' B](y,x)
//   dP(y,o) = T1p(y,o) - Box[Ac](y,o) - p'(y,o) Box[Bp](y,o) + Box[mp' Bp](y,o)
//
//   BoxA(y,x,dl) = sum of A(h,w,dl) over |h-y|,|w-x| <= r     (fixed diagonal dl = d - w)
//   T1c(y,x) = sum_dl p'(y,x+dl) BoxA(y,x,dl)      T1p(y,o) = sum_dl c'(y,o-dl) BoxA(y,o-dl,dl)
//   Am(h,w)  = sum_dl A mp'(h,w+dl)   B(h,w)  = sum_dl V Y(h,w+dl)
//   Ac(h,o)  = sum_w  A mc'(h,w)      Bp(h,o) = sum_w  V X(h,w)
//
// X, Y are the centred second moments of the camera / projector patches, m
// their means, and c' = c - cbar, p' = p - pbar (zero padding included, so an
// out-of-image tap is -cbar): the gradient is exactly invariant under a
// global shift of either image, and shifting by the image mean removes the
// cancellation between T1 and Box[Am] (and between c Box[B] and Box[mc B])
// that otherwise makes fp32 accumulation lose ~1e-5 of the result on smooth
// images.  With the shift every sum here is fp32 (validated against the fp64
// oracle on textured, smooth, quantised and all-ones inputs).
//
// Sweep layout ("column sweep"): one wave = 64 consecutive diagonals (lane
// l owns dl = d0 + l) x 16 image rows (registers), walking the camera
// columns w.  Per step it loads the gradient row segment g[h][w][w+dl] of
// NY = 16 + 2r rows (256 contiguous bytes per row), forms A, keeps the
// horizontal sliding sums HA[y] of A (NY registers, the leaving column's A
// recomputed from its gradient -- an L2/MALL re-read), and the vertical box
// over the registers gives BoxA for its 16 own rows.  Camera-side values of
// one step belong to one camera pixel per row and are summed across the
// lanes (permlane32/16 swaps + DPP butterflies, 106 VALU for 48 sums);
// projector-side values of lane l belong to projector column w + dl + const,
// which moves down one lane per step, so they accumulate in registers with a
// DPP wave_shl:1 fused into the add, and lane 0's completed column is
// emitted every step.  Both go through a 16-step LDS buffer to coalesced
// stores of fp32 partial sums per diagonal chunk; k_bwd_gather sums the
// chunks and k_bwd_combine applies the box filters.
#include <algorithm>
#include <cmath>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "common.h"
#include "sweep.h"
#include "xlane.h"

namespace custma {

namespace {

// own rows per unit (workgroup); 32-row units re-read fewer halo rows but one 8-wave workgroup per
// CU ran slower (C5 44.3 vs 39.1 ms, round 2)
constexpr int TRB = 16;
constexpr int NLB = 64;   // diagonals per wave
constexpr int NTYPE = 6;  // partial types: T1c, Am, B (camera) | T1p, Ac, Bp (projector)
// 128 -> 512 columns: C5 window backward 28.9 -> 27.6-28.0 ms, C2 full 3.57 -> 3.38 ms (profiles/r03/seg_ab.txt)
// most pixel columns per unit; a unit sweeps its segment + 2 r columns, so the 2 r halo steps are
// 2 r / segment of redundant work.  A chunk's columns are cut into equal segments of at most kSeg
// (chunk_geo; an unequal last segment left the last round of units half idle: C3 has 4 segments
// of 451 columns, not 3 of 512 + 1 of 266).  Every segment holds >= 64 + 2 r columns whenever a
// chunk has two or more, so segments s and s + 2 never overlap (slot parity).
constexpr int kSeg = 512;
constexpr uint32_t kOOB = 0x80000000u;
// The slot-parity argument (plan_bwd's S = 2 x the max chunk overlap) needs every segment of a
// multi-segment chunk (>= kSeg / 2 columns) to hold >= k + NLB - 1 columns for the largest sliding k
// (CUSTMA_SWEEP_KS: 31); a violation would only show at run time as NaN gradients (k_bwd_cover).
static_assert(kSeg / 2 >= 31 + 64 - 1, "segments too narrow for the slot parity at the largest sliding k");

// Chunk geometry (host and device): diagonals [d0, d0+64); camera columns that carry
// a valid voxel for some lane: [wlo, whi); pixel columns whose box touches one:
// [wlo - r, whi + r), cut into equal segments of seg <= kSeg columns (one unit each).
struct ChunkGeo {
    int64_t d0, wlo, whi, seg;
};
__host__ __device__ inline ChunkGeo chunk_geo(const Geo& g, int64_t dlo, int j) {
    ChunkGeo c;
    c.d0 = dlo + (int64_t)NLB * j;
    if (g.layout == CUSTMA_LAYOUT_WINDOW) {
        c.wlo = 0;
        c.whi = g.WO;
    } else {
        const int64_t a = -(c.d0 + NLB - 1);
        c.wlo = a > 0 ? a : 0;
        const int64_t b = g.W - c.d0;
        c.whi = b < g.W ? b : g.W;
    }
    const int64_t span = c.whi - c.wlo + (g.k - 1);
    int64_t n = span > kSeg ? (span + kSeg - 1) / kSeg : 1;
    // run_bwd's tail balancing asks for more (narrower) segments, never narrower than the slot-parity
    // minimum of k + NLB - 1 columns
    if (g.seg_min > n) {
        const int64_t nmax = span / (g.k + NLB - 1);
        n = nmax > n ? (g.seg_min < nmax ? g.seg_min : nmax) : n;
    }
    c.seg = span > 0 ? (span + n - 1) / n : 1;
    return c;
}
// Taps: the forward's patch of voxel (h, w) covers rows h - r0 .. h + r1 (r0 = k/2, r1 = k-1-k/2, the
// reference's kernel_size / 2 origin, stereo_matching_kernel.cu:44,60), so an output pixel (y, x) gathers
// the voxels h in [y - r1, y + r0], w in [x - r1, x + r0] (r0 = r1 = r for odd k).
struct Taps {
    int r0, r1;
};
__host__ __device__ inline Taps taps_of(const Geo& g) { return Taps{g.k / 2, g.k - 1 - g.k / 2}; }
__host__ __device__ inline int chunk_nseg(const ChunkGeo& c, Taps t) {
    return (int)((c.whi - c.wlo + t.r0 + t.r1 + c.seg - 1) / c.seg);
}
// Segment s of chunk c: output pixel columns [xs, xe); the sweep runs w in [xs - r1, xe + r0).
__host__ __device__ inline void seg_cols(const ChunkGeo& c, Taps tp, int s, int64_t* xs, int64_t* xe) {
    const int64_t tlo = c.wlo - tp.r0, thi = c.whi + tp.r1;
    *xs = tlo + (int64_t)s * c.seg;
    const int64_t e = *xs + c.seg;
    *xe = e < thi ? e : thi;
}
// Written column range [lo, hi) of partial type t for segment s of chunk c (before clipping
// to [0, W)).  Camera types: the segment's own columns.  Projector types: every column
// whose accumulator passed lane 0 during the sweep or sat in the wave at its end.
__host__ __device__ inline void seg_range(const ChunkGeo& c, Taps tp, int s, int t, int64_t* lo, int64_t* hi) {
    int64_t xs, xe;
    seg_cols(c, tp, s, &xs, &xe);
    const int64_t w0 = xs - tp.r1, w1 = xe + tp.r0;  // sweep steps [w0, w1)
    switch (t) {
        case 0: case 1: case 2: *lo = xs; *hi = xe; break;                                // T1c, Am, B
        case 3: *lo = w0 - 1 - tp.r0 + c.d0; *hi = w1 - 1 - tp.r0 + c.d0 + NLB; break;      // T1p
        default: *lo = w0 - 1 + c.d0; *hi = w1 - 1 + c.d0 + NLB; break;                     // Ac, Bp
    }
}
// Union over the chunk's segments (contiguous).
__host__ __device__ inline void type_range(const ChunkGeo& c, Taps tp, int t, int64_t* lo, int64_t* hi) {
    int64_t l0, h0, l1, h1;
    seg_range(c, tp, 0, t, &l0, &h0);
    seg_range(c, tp, chunk_nseg(c, tp) - 1, t, &l1, &h1);
    *lo = l0;
    *hi = h1;
}

struct BwdArgs {
    const void* cam;
    const void* proj;
    Stats sc, sp;
    // prepared fp32 images [H][W] (k_bwd_prep): camera X, mc', c and projector Y, mp', p
    const float *Xc, *mcc, *cc, *Yp, *mpp, *pp;
    const float* grad;
    const float* vol;
    const float* shift;  // [2]: cbar, pbar
    float* part;         // [NTYPE][S][H][W]
    // window layouts with D = 64 n (BwdPlan::rem): the remainder diagonal D's terms, written by the
    // row-walking remainder kernel (k_bwd_rem_rows), added by k_bwd_gather:
    //   remT [4][HV][WO]       A mp'(h, w+D), V Y(h, w+D), A mc'(h, w), V X(h, w)
    //   remT1[2][yhi-ylo][W]   T1c at (y, x): p'(y, x+D) BoxA_D(y, x);  T1p at (y, x+D): c'(y, x) BoxA_D(y, x)
    float* remT;
    float* remT1;
    const int* cover;    // k_bwd_cover: slot counts and lists per (range class, column)
    int S, Sj, nChunk, nRG, jc, nsegMax;
    int order;  // block order of k_bwd_coop (see there)
    int64_t dlo, ylo, yhi;
};

__device__ __forceinline__ int chunk_of_rank(int r, int n, int jc) {
    // longest chunks (diagonals near 0 in the full layout) first: jc, jc+1, jc-1, ...
    const int below = jc, above = n - 1 - jc, m = below < above ? below : above;
    if (r <= 2 * m) {
        if (r == 0) return jc;
        const int s = (r + 1) / 2;
        return (r & 1) ? jc + s : jc - s;
    }
    const int rest = r - 2 * m;
    return above > below ? jc + m + rest : jc - m - rest;
}

// ---------------------------------------------------------------------------------------
// Cooperative column sweep.  One WORKGROUP of NWC waves owns a (chunk, segment, row group)
// unit of TRB rows: wave v owns rows y0 + 4v .. y0 + 4v + 3.  Per step every gradient
// element of the unit's TRB + 2r rows is loaded and turned into A = g / S exactly once
// (own rows by their owner, the 2r halo rows spread over the waves) and published in a
// double-buffered LDS row array; after one barrier each wave forms the vertical k-row sums
// V of its own rows and slides them horizontally with a k-deep LDS ring of its own V
// (HV += V(w) - V(w-k)).  So the leaving column is never re-read, no halo row is loaded
// twice within a unit, and the leaving column's Y is not needed at all.  Taller units
// (32 rows: 8 waves) would re-read fewer halo rows of the gradient: (TRB + 2r) / TRB gradient
// reads per voxel.
constexpr int TRW = 4;           // own rows per wave
constexpr int NWC = TRB / TRW;   // waves per cooperative workgroup
#ifndef CUSTMA_BWD_DEPTH
#define CUSTMA_BWD_DEPTH 1
#endif
constexpr int BDP = CUSTMA_BWD_DEPTH;  // steps of loads in flight (1 or 2)
// The per-voxel projector values Y, mp', p' of a lane at column w + dl are the next lane's
// values of the previous step, so they slide down one lane per step (DPP wave_shl:1) and only
// lane 63 takes a new column, read from a register loaded once per 64 steps -- instead of a
// 64-lane load of each per step (those image rows do not stay in L2 beside the gradient
// stream: ~half of the kernel's L2 misses).
// Steps per flush, a multiple of BDP + 1 (every flush block starts on load buffer 0).  16 (all 64
// lanes store: 4 rows x 16 steps) where the LDS allows it: C5 window backward op 27.7 -> 26.7 ms,
// C3 3.26 -> 3.19 ms (profiles/r03/win_fbc_ab.txt); k <= 9 keeps 8, so its 3 workgroups per CU fit.
template <int K>
constexpr int fbc_for() { return BDP == 2 ? (K >= 11 ? 12 : 6) : K >= 11 ? 16 : 8; }

// Finish 3 registers (each already summed over the 4 lanes {l, l+16, l+32, l+48}, one
// value per 16-lane row): afterwards every lane holds the full 64-lane sum of one of the 12.
__device__ __forceinline__ float reduce_tail3(float w0, float w1, float w2, int lane) {
    const float x0 = pair_level<kMirror16, 8>(w0, w1, lane);
    const float x1 = w2 + dpp<kMirror16>(w2);
    const float y0 = pair_level<kMirror8, 4>(x0, x1, lane);
    const float z = y0 + dpp<kQuad3210>(y0);
    return z + dpp<kQuad1032>(z);
}

// Window-layout form (WIN): a step's gradient / volume / camera addresses are a per-lane loop
// constant plus a wave-uniform part, so the step adds the wave-uniform part as the SGPR soffset
// (SALU) instead of recomputing every lane's offset and bounds (VALU).  Out-of-range markers are
// kWinNR (>= the window descriptors' num_records, so any one of them is out of range, and any sum
// of three stays below 2^32); in-range offsets stay below kWinNR (win_path_ok).
constexpr uint32_t kWinNR = 0x55555550u;

template <int N, typename F>
__device__ __forceinline__ F tree_sum(const F* c) {
    if constexpr (N == 1) return c[0];
    else return tree_sum<N / 2>(c) + tree_sum<N - N / 2>(c + N / 2);
}

// Camera values of a step (X of the own and halo rows at column w, mc' of the own rows, c at w - R)
// from a wave-private LDS block instead of four per-step loads: one lane-per-column load of each of
// the 12 + HP rows every 64 steps (a block ahead, like the sliding projector columns), written to
// LDS at the block's first step, read back row-replicated (lane l: row l & 3) by four ds_reads per
// step.  The per-step loads touched four lines each for 16 useful bytes (a third of the step's
// line requests).  k <= 11 (profiles/r03/caml: k = 5 -8 %, k = 9 -4..-5 % although the 3.9 KB per wave
// costs k = 7, 9 their third workgroup per CU, k = 11 -4 %); k = 13 would drop to one workgroup per CU
// (+54 %), k = 15, 17 are there already.
template <int K>
constexpr bool cam_lds_for() {
    return K <= 11;
}
constexpr int kCamP = 65;  // LDS row pitch of the camera block (65: the four rows of a read in different banks)

template <int K, bool WIN>
__device__ __forceinline__ void bwd_coop_body(const Geo& g, const BwdArgs& a, int j, int sg, int rg, float* Abuf,
                                              float* ring, float (*cbuf)[12], float (*pbuf)[12], float* camb) {
    constexpr bool CAML = cam_lds_for<K>();
    // A rows of the unit: image rows y0 - R1 .. y0 + TRB - 1 + R0 (R1 halo rows above, R0 below)
    constexpr int R0 = K / 2, R1 = K - 1 - K / 2, NY = TRB + K - 1, NH = K - 1;  // NH halo rows
    constexpr int FBC = fbc_for<K>();
    static_assert(FBC % (BDP + 1) == 0 && FBC <= 16, "flush blocks start on load buffer 0; 4 FBC lanes");
    constexpr int HPW = (NH + NWC - 1) / NWC;                // halo rows per wave (at most)
    static_assert(HPW <= 8, "a wave's halo rows fit one octet of a 16-lane row");
    constexpr int HSL = HPW > 4 ? 8 : 4;  // halo camera slots per 16-lane row (lane l: halo row l % HSL)

    const ChunkGeo cg = chunk_geo(g, a.dlo, j);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int Wi = (int)g.W, Hi = (int)g.H;
    const int d0 = (int)cg.d0, dl = d0 + lane;
    const int64_t y0 = a.ylo + (int64_t)TRB * rg;
    const int y0i = (int)y0;
    int64_t xs64, xe64;
    seg_cols(cg, Taps{R0, R1}, sg, &xs64, &xe64);
    const int xs = (int)xs64, xe = (int)xe64;
    const int w0 = xs - R1, wend = xe + R0;  // step w completes the horizontal box of output column w - R0
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    int lwlo, lwhi;
    if (window) {
        lwlo = 0;
        lwhi = (dl >= 0 && dl <= g.D) ? (int)g.WO : 0;
    } else {
        lwlo = dl < 0 ? -dl : 0;
        lwhi = min((int)g.WO, Wi - dl);
    }
    const int gsU = (int)g.DO + (window ? 0 : 1);
    const int slot = 2 * (j % a.Sj) + (sg & 1);
    const size_t plane = (size_t)g.H * g.W;
    const float cb = a.shift[0], pb = a.shift[1];

    const uint32_t ib = (uint32_t)(plane * 4);
    const size_t slab = (size_t)g.WO * g.DO;
    const int64_t vrow0 = max(g.h_lo, y0 - R1);
    const auto rG = make_rsrc(a.grad + (size_t)(vrow0 - g.h_lo) * slab, 0x7FFFFFF0u);
    const auto rV = make_rsrc(a.vol + (size_t)(vrow0 - g.h_lo) * slab, 0x7FFFFFF0u);
    const int64_t ir0 = y0 - R1;
    const uint32_t vstride = (uint32_t)(slab * 4);
    const uint32_t vNR = WIN ? kWinNR : 0x7FFFFFF0u;  // the volume descriptors' num_records
    const int hlo = (int)g.h_lo, hhi = (int)g.h_hi, vrow0i = (int)vrow0;
    // The six prepared images are one array (k_bwd_prep: X, mc', c, Y, mp', p) read through ONE
    // descriptor, the image selected by a per-lane offset: two descriptors instead of eight keep
    // the kernel's SGPRs (spilled to VGPR lanes before) in registers.
    enum { kX = 0, kMc = 1, kC = 2, kY = 3, kMp = 4, kP = 5 };
    const uint32_t pb4 = ib;  // bytes per prepared image
    auto img_off_a = [&](int row, int col, int arr) -> uint32_t {
        return (row >= 0 && row < Hi && col >= 0 && col < Wi) ? (uint32_t)((row * Wi + col) * 4) + arr * pb4 : kOOB;
    };
    auto col_off_a = [&](int col, int arr) -> uint32_t {
        return (col >= 0 && col < Wi) ? (uint32_t)(col * 4) + arr * pb4 : kOOB;
    };
    auto img_off = [&](int row, int col) -> uint32_t {
        return (row >= 0 && row < Hi && col >= 0 && col < Wi) ? (uint32_t)((row * Wi + col) * 4) : kOOB;
    };
    auto col_off = [&](int col) -> uint32_t { return (col >= 0 && col < Wi) ? (uint32_t)(col * 4) : kOOB; };

    float HV[TRW];  // horizontal running sums of the vertical box sums V (own rows)
    float P[3][TRW];
#pragma unroll
    for (int m = 0; m < TRW; ++m) {
        HV[m] = 0.f;
        P[0][m] = P[1][m] = P[2][m] = 0.f;
    }
    // ring[s][m][lane]: V of own row m at the step s (mod K) before
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
        for (int m = 0; m < TRW; ++m) ring[(s * TRW + m) * 64 + lane] = 0.f;

    const int yw = TRW * wv;  // first own row of this wave (unit row index)
    const uint32_t prow_bytes = (uint32_t)(max((int64_t)0, min((int64_t)TRW, a.yhi - y0 - yw)) * g.W * 4);
    auto part_rsrc = [&](int t) {
        return make_rsrc(a.part + ((size_t)t * a.S + slot) * plane + (size_t)(y0 + yw) * g.W, prow_bytes);
    };
    // loads per issue() (asm_ld2s / asm_ld1s / asm_ld4), per thread
#ifdef CUSTMA_KO_NOVOL
    // knock-out (timing only, wrong results): no volume loads, every cost 0.5
    constexpr int NLD = TRW + (HPW > 0 ? HPW : 1) + (CAML ? 0 : 4);
#else
    constexpr int NLD = TRW * 2 + (HPW > 0 ? HPW : 1) + (CAML ? 0 : 4);
#endif
    auto flush = [&](int wfirst, int nsteps) {
        if constexpr (BDP == 2) asm_vmcnt<NLD>();  // all but the newest issue
        int ln = lane;
        asm volatile("" : "+v"(ln));
        // lanes 0..4 FBC-1: step jcol, own row m (the rest idle)
        const int jcol = ln % FBC, m = (ln / FBC) & 3;
        const bool live = jcol < nsteps && ln < 4 * FBC;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int p = 4 * t + m;
            const int col = wfirst + jcol - (t == 0 ? R0 : 0);
            const bool cok = live && col >= xs && col < xe && col >= 0 && col < Wi;
            st_buf(cbuf[jcol][p], part_rsrc(t), cok ? (uint32_t)((m * Wi + col) * 4) : kOOB);
            const int pcol = wfirst + jcol - 1 + (t == 0 ? -R0 : 0) + d0;
            const uint32_t poff = (live && pcol >= 0 && pcol < Wi) ? (uint32_t)((m * Wi + pcol) * 4) : kOOB;
            st_buf(pbuf[jcol][p], part_rsrc(3 + t), poff);
        }
    };
    // which of the 12 camera sums (type * 4 + own row) each lane ends up with
    int qlane;
    {
        const bool l0 = lane == 0;
        auto mk = [&](int q) { return l0 ? (float)q : 0.f; };
        const float w0r = red16(red32(mk(4), mk(8)), red32(mk(5), mk(9)));
        const float w1r = red16(red32(mk(6), mk(10)), red32(mk(7), mk(11)));
        const float w2r = red16(red32(mk(0), mk(1)), red32(mk(2), mk(3)));
        qlane = (int)reduce_tail3(w0r, w1r, w2r, lane);
    }

    // rows of the unit this wave turns into A: its own rows, then its share of the halo
    auto halo_row = [&](int q) { return q < R1 ? q : q + TRB; };  // q in [0, K - 1)
    constexpr int HP = HPW > 0 ? HPW : 1;

    // ---- loads: issued one step ahead as inline asm (hand-counted waits; the compiler's
    // own tracking would drain them at the loop header).  Rows by wave-uniform soffset
    // (image rows clamped into the image: a clamped row only meets a zero gradient or feeds
    // outputs that are not stored; volume rows outside the volume get an soffset past the
    // descriptor, and the gfx950 range check includes soffset), columns by voffset. ----
    auto iso = [&](int y) -> uint32_t {
        int rr = (int)ir0 + y;
        rr = rr < 0 ? 0 : rr >= Hi ? Hi - 1 : rr;
        return (uint32_t)rr * (uint32_t)(Wi * 4);
    };
    auto vso = [&](int y) -> uint32_t {
        const int row = (int)ir0 + y;
        return (row >= hlo && row < hhi) ? (uint32_t)(row - vrow0i) * vstride : vNR;
    };
    uint32_t sIo[TRW], sVo[TRW], sIh[HP], sVh[HP];
#pragma unroll
    for (int m = 0; m < TRW; ++m) {
        sIo[m] = __builtin_amdgcn_readfirstlane(iso(R1 + yw + m));
        sVo[m] = __builtin_amdgcn_readfirstlane(vso(R1 + yw + m));
    }
#pragma unroll
    for (int i = 0; i < HP; ++i) {
        const int q = wv + NWC * i;
        const int y = halo_row(q < NH ? q : 0);
        sIh[i] = __builtin_amdgcn_readfirstlane(iso(y));
        // WIN: a wave without this halo row reads it out of range (its soffset is the marker)
        sVh[i] = __builtin_amdgcn_readfirstlane(WIN && q >= NH ? vNR : vso(y));
    }
    const i32x4 dG = make_rsrc_sgpr(a.grad + (size_t)(vrow0 - g.h_lo) * slab, vNR);
    const i32x4 dV = make_rsrc_sgpr(a.vol + (size_t)(vrow0 - g.h_lo) * slab, vNR);
    const i32x4 dPr = make_rsrc_sgpr(a.Xc, 6u * ib);  // a.Xc = the prepared array's base
    // WIN: the camera-value loads through a descriptor whose range is the marker bound (offsets
    // stay inside the prepared array: rows checked per lane, columns per step)
    const i32x4 dPc = make_rsrc_sgpr(a.Xc, kWinNR);
    const int orow_l = y0i + yw + (lane & 3);  // own image row of this lane's quad slot
    int hrow_l = -1;                           // halo image row of this lane's halo slot (or none)
    const int hq = lane & (HSL - 1);
    if (hq < HPW && wv + NWC * hq < NH) hrow_l = (int)ir0 + halo_row(wv + NWC * hq);
    struct Ld {
        // xo / mc / cx: lane l holds own row l & 3 (row-replicated per 16 lanes, read back with
        // DPP row_newbcast); xh: lane l holds the wave's halo row l % HSL
        uint32_t ge[TRW], cv[TRW], hg[HP], xo, xh, mc, cx;
    };
    // NOP: open each load group with `s_nop 4` (VALU SGPR write -> VMEM read); the in-loop
    // issues go without -- their descriptors / soffsets are loop constants, written (by
    // readfirstlane) only in the prologue, which custereomatching_amd/hazard_check.py checks at build time
    // WIN per-lane loop constants: the lane's diagonal (or the marker past D) and its camera-value
    // offsets (own row / halo row of its quad slot, each prepared array; the marker outside the image)
    const uint32_t vLane = dl <= g.D ? (uint32_t)dl * 4u : kWinNR;
    // WIN: the rows' parts of the gradient / volume offsets folded into per-lane loop constants, so a
    // step's loads all take the step's column as their one SGPR soffset (no per-load SALU add)
    uint32_t vLO[TRW], vLH[HP];
#pragma unroll
    for (int m = 0; m < TRW; ++m) vLO[m] = vLane + sVo[m];
#pragma unroll
    for (int i = 0; i < HP; ++i) vLH[i] = vLane + sVh[i];
    auto img_row_a = [&](int row, int arr) -> uint32_t {
        return (row >= 0 && row < Hi) ? (uint32_t)(row * Wi * 4) + arr * pb4 : kWinNR;
    };
    const uint32_t vXo = img_row_a(orow_l, kX), vXh = hrow_l >= 0 ? img_row_a(hrow_l, kX) : kWinNR;
    const uint32_t vMo = img_row_a(orow_l, kMc), vCo = img_row_a(orow_l, kC);
    const uint32_t gsU4 = (uint32_t)gsU * 4u;
    auto issue = [&](int w, Ld& b, auto nop_) {
        constexpr bool NOP = decltype(nop_)::value;
        const int xb = w - R0;
        if constexpr (WIN) {
            // wave-uniform parts: the step's volume column (marker outside [0, WO)) and the two
            // camera columns w and w - R (marker outside [0, W))
            // (w is wave-uniform; pinned to an SGPR so that sW, the loads' only soffset, is SALU-computed)
            const int ws = __builtin_amdgcn_readfirstlane(w);
            const uint32_t sW = (ws >= 0 && ws < (int)g.WO) ? (uint32_t)ws * gsU4 : kWinNR;
            const uint32_t sC = (w >= 0 && w < Wi) ? (uint32_t)w * 4u : kWinNR;
            const uint32_t sX = (xb >= 0 && xb < Wi) ? (uint32_t)xb * 4u : kWinNR;
#pragma unroll
            for (int m = 0; m < TRW; ++m) {
#ifdef CUSTMA_KO_NOVOL
                asm_ld1s<NOP>(b.ge[m], vLO[m], dG, sW);
                b.cv[m] = 0x3f000000u;
#else
                asm_ld2s<NOP>(b.ge[m], b.cv[m], vLO[m], vLO[m], dG, dV, sW, sW);
#endif
            }
#pragma unroll
            for (int i = 0; i < HP; ++i) asm_ld1s<NOP>(b.hg[i], vLH[i], dG, sW);
            if constexpr (!CAML) asm_ld4s<NOP>(b.xo, b.xh, b.mc, b.cx, vXo, vXh, vMo, vCo, dPc, sC, sX);
            return;
        }
        const bool ve = w >= lwlo && w < lwhi;
        const uint32_t oGe = ve ? (uint32_t)((w * gsU + dl) * 4) : kOOB;
#pragma unroll
        for (int m = 0; m < TRW; ++m) {
#ifdef CUSTMA_KO_NOVOL
            asm_ld1s<NOP>(b.ge[m], oGe, dG, sVo[m]);
            b.cv[m] = 0x3f000000u;
#else
            asm_ld2s<NOP>(b.ge[m], b.cv[m], oGe, oGe, dG, dV, sVo[m], sVo[m]);
#endif
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) asm_ld1s<NOP>(b.hg[i], wv + NWC * i < NH ? oGe : kOOB, dG, sVh[i]);
        if constexpr (!CAML)
        asm_ld4<NOP>(b.xo, b.xh, b.mc, b.cx, img_off_a(orow_l, w, kX), hrow_l >= 0 ? img_off_a(hrow_l, w, kX) : kOOB,
                img_off_a(orow_l, w, kMc), img_off_a(orow_l, xb, kC), dPr, dPr, dPr);
    };
    // the current step's projector-side columns (lane l: column w + dl, p': w - R + dl)
    // and the once-per-64-steps column block whose lane i feeds lane 63 at step w0 + 1 + 64k + i
    // sc[3m + {0, 1, 2}] = Y, mp', p' of own row m; bc the same for the block
    uint32_t sc[3 * TRW], shY[HP], bc[3 * TRW], bhY[HP];
    auto load_cols = [&](uint32_t* c, uint32_t* hY, int cb) {
        const uint32_t oY = col_off_a(cb + dl, kY), oM = col_off_a(cb + dl, kMp), oP = col_off_a(cb - R0 + dl, kP);
#pragma unroll
        for (int m = 0; m < TRW; ++m) {
            asm_ld2s(c[3 * m], c[3 * m + 1], oY, oM, dPr, dPr, sIo[m], sIo[m]);
            asm_ld1s(c[3 * m + 2], oP, dPr, sIo[m]);
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) asm_ld1s(hY[i], wv + NWC * i < NH ? oY : kOOB, dPr, sIh[i]);
    };
    // CAML: the camera block registers (lane i: column wb + i of own row m's X / mc' (3m, 3m + 1),
    // column wb - R + i of its c (3m + 2); halo row i's X at 12 + i), loaded a block ahead
    constexpr int NCB = CAML ? 12 + HP : 1;
    uint32_t cbk[NCB];
    auto load_cam = [&](int wb) {
        if constexpr (CAML) {
            const uint32_t oX = col_off_a(wb + lane, kX), oM = col_off_a(wb + lane, kMc), oC = col_off_a(wb - R0 + lane, kC);
#pragma unroll
            for (int m = 0; m < TRW; ++m) {
                asm_ld2s(cbk[3 * m], cbk[3 * m + 1], oX, oM, dPr, dPr, sIo[m], sIo[m]);
                asm_ld1s(cbk[3 * m + 2], oC, dPr, sIo[m]);
            }
#pragma unroll
            for (int i = 0; i < HP; ++i) asm_ld1s(cbk[12 + i], wv + NWC * i < NH ? oX : kOOB, dPr, sIh[i]);
        }
    };
    auto tie_cols = [&]() {
        if constexpr (CAML) {
#pragma unroll
            for (int r = 0; r < NCB; ++r) asm_tie(cbk[r]);
        }
#pragma unroll
        for (int m = 0; m < TRW; ++m) {
            asm_tie(sc[3 * m]); asm_tie(sc[3 * m + 1]); asm_tie(sc[3 * m + 2]);
            asm_tie(bc[3 * m]); asm_tie(bc[3 * m + 1]); asm_tie(bc[3 * m + 2]);
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) { asm_tie(shY[i]); asm_tie(bhY[i]); }
    };
    const uint64_t lane63 = 1ull << 63;
    auto tie = [&](Ld& b) {
#pragma unroll
        for (int m = 0; m < TRW; ++m) {
            asm_tie(b.ge[m]); asm_tie(b.cv[m]);
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) asm_tie(b.hg[i]);
        asm_tie(b.xo); asm_tie(b.xh); asm_tie(b.mc); asm_tie(b.cx);
        tie_cols();
    };
    auto F = [](uint32_t u) { return __builtin_bit_cast(float, u); };

    int sidx = 0;  // ring slot of the current step (step count mod K)
    // loads per issue() and stores per flush(), per thread
    constexpr int NL = NLD, SF = 6;
    static_assert(NL + SF <= 63, "vmcnt holds the pipeline");
    // cur was issued BDP steps ago; issued since: the later steps' loads, and a flush's SF
    // stores after step s = FBC-1 of the previous block (flush() itself waits until only
    // the newest issue is in flight: at s = 0 of a block after a flush cur has landed)
    // A step's 12 camera sums are reduced across the lanes during the NEXT step's A phase
    // (before its barrier), where the reduction's dependency chain overlaps independent
    // work; the block's last step is reduced before the flush (drain()).
    float rA[TRW], rB[TRW], rT[TRW];
    auto reduce_to = [&](int slot) {
        // red16(red32(amv0, bv0), red32(amv1, bv1)), ... with the swaps of a level in one asm
        swap32x6(rA[0], rB[0], rA[1], rB[1], rA[2], rB[2], rA[3], rB[3], rT[0], rT[1], rT[2], rT[3]);
        float u0 = rA[0] + rB[0], u1 = rA[1] + rB[1], u2 = rA[2] + rB[2], u3 = rA[3] + rB[3];
        float u4 = rT[0] + rT[1], u5 = rT[2] + rT[3];
        swap16x3(u0, u1, u2, u3, u4, u5);
        const float w0r = u0 + u1, w1r = u2 + u3, w2r = u4 + u5;
        cbuf[slot][qlane] = reduce_tail3(w0r, w1r, w2r, lane);
    };
    // fl_c: BDP == 1 -- std::true_type at a block's first step (after the previous block's flush, or
    // after the prologue's wait), std::false_type elsewhere, so every wait is fixed at compile time
    // and vmcnt_check.py can prove it on the emitted code; BDP == 2 -- a runtime bool (flushed)
    auto step = [&](Ld& cur, Ld& nxt, int w, int s, auto fl_c) {
        if constexpr (BDP == 2) {
            const bool flushed = fl_c;
            // a column block issued at s = 0 (after the flush's stores) feeds step 1
            if (!flushed || s >= 1) asm_vmcnt<NL>();
            else if (s == 1) asm_vmcnt<NL + SF>();
        } else if constexpr (std::is_same<decltype(fl_c), std::true_type>::value) {
            // the step's loads, not the flush's SF stores issued after them: a store's completion
            // is not needed here, and on gfx950 `s_waitcnt vmcnt(N)` counts loads, stores, atomics
            // and LDS-DMA together in issue order, so vmcnt(SF) waits for every load issued before
            // those SF stores (MI355X_MICROARCH.md, the vmcnt paragraph after the cycle constants;
            // LLVM's own waitcnt pass does not assume this ordering, hence the hand-counted wait)
            asm_vmcnt<SF>();
        } else {
            asm_vmcnt<0>();
        }
        tie(cur);
        if (w > w0) {  // move the columns down one lane; lane 63 takes column w + 63 (+ offset)
            slide_rows<HP>(sc, bc, shY, bhY, lane63);
        }
        // the block for steps w + 1 .. w + 64 (lane i -> step w + 1 + i): columns w + 64 + i (+ offset);
        // issued after this step's reads of the previous block
        if (((w - w0) & 63) == 0) load_cols(bc, bhY, w + 64);
        uint32_t cxo_r = cur.xo, cxh_r = cur.xh, cmc_r = cur.mc, ccx_r = cur.cx;
        if constexpr (CAML) {
            typedef __attribute__((address_space(3))) float lds_f;
            lds_f* cl = (lds_f*)camb;
            const int cc = (w - w0) & 63;
            if (cc == 0) {  // the block of steps w .. w + 63 into LDS, then the next block's loads
#pragma unroll
                for (int r = 0; r < NCB; ++r) cl[r * kCamP + lane] = F(cbk[r]);
                load_cam(w + 64);
            }
            const int q = lane & 3;
            cxo_r = __builtin_bit_cast(uint32_t, cl[(3 * q) * kCamP + cc]);
            cmc_r = __builtin_bit_cast(uint32_t, cl[(3 * q + 1) * kCamP + cc]);
            ccx_r = __builtin_bit_cast(uint32_t, cl[(3 * q + 2) * kCamP + cc]);
            cxh_r = __builtin_bit_cast(uint32_t, cl[(12 + (q < HP ? q : HP - 1)) * kCamP + cc]);
        }
        issue(w + BDP, nxt, std::false_type{});  // past the segment's end: harmless, drained before the wave ends
        float* Acur = Abuf + ((w - w0) & 1) * ((NY + 1) * 64);  // double-buffered: one barrier per step
        // this wave's ring slot of the step (V of its rows K steps ago): wave-private, so read
        // ahead of the barrier
        float rsv[TRW];
#pragma unroll
        for (int m = 0; m < TRW; ++m) rsv[m] = ring[(sidx * TRW + m) * 64 + lane];
        if (lane == 0) {
#pragma unroll
            for (int t = 0; t < 3; ++t)
                *(float4*)&pbuf[s][4 * t] = make_float4(P[t][0], P[t][1], P[t][2], P[t][3]);
        }
        const int xb = w - R0;
        const float tf = xb >= xs ? 1.f : 0.f, af = (w >= xs && w < xe) ? 1.f : 0.f;
        const float mco = F(cmc_r) * af;
        const float cxo = (F(ccx_r) - cb) * tf;
        // ---- own rows: A, and the per-voxel terms (unit rows R + yw .. R + yw + 3); the
        // row's camera values come from quad slot m of the row-replicated registers ----
        float amv[TRW], bv[TRW];
        Unroll<0, TRW>::run([&](auto mi) {
            constexpr int m = decltype(mi)::value;
            const int y = R1 + yw + m;
            const float Xf = rbc<m>(F(cxo_r)), Ye = F(sc[3 * m]);
            const float rSe = __builtin_amdgcn_rsqf(__builtin_fmaf(Xf, Ye, kEps));
            const float Ae = F(cur.ge[m]) * rSe;
            Acur[y * 64 + lane] = Ae;
            const float V = Ae * F(cur.cv[m]) * rSe;
            amv[m] = Ae * F(sc[3 * m + 1]);
            bv[m] = V * Ye;
            P[1][m] = shl1_add(P[1][m], Ae * rbc<m>(mco));
            P[2][m] = shl1_add(P[2][m], (V * af) * Xf);
        });
        // halo rows: no per-step branch -- a wave without a last halo row computes it from its
        // out-of-range (zero) loads anyway and stores it to the spare row NY of the A buffer
        Unroll<0, HPW>::run([&](auto ii) {
            constexpr int i = decltype(ii)::value;
            constexpr bool ALL = NWC * i + NWC - 1 < NH;  // every wave has halo row i
            const int q = wv + NWC * i;
            const int y = ALL || q < NH ? halo_row(q) : NY;
            Acur[y * 64 + lane] = F(cur.hg[i]) * __builtin_amdgcn_rsqf(
                                                     __builtin_fmaf(rbc<i>(F(cxh_r)), F(shY[i]), kEps));
        });
        if (s > 0) reduce_to(s - 1);
        __syncthreads();  // the unit's A rows of this step are published
        // ---- vertical k-row sums of own rows, horizontal slide through the ring ----
        float col[TRW + K - 1];
#pragma unroll
        for (int y = 0; y < TRW + K - 1; ++y) col[y] = Acur[(yw + y) * 64 + lane];
        float v = tree_sum<K>(col);  // a pairwise tree: depth log2(k) instead of a k-long chain
        float t1v[TRW];
        Unroll<0, TRW>::run([&](auto mi) {
            constexpr int m = decltype(mi)::value;
            if (m > 0) v = (v + col[m + K - 1]) - col[m - 1];
            HV[m] += v - rsv[m];
            ring[(sidx * TRW + m) * 64 + lane] = v;
            t1v[m] = (F(sc[3 * m + 2]) - pb) * HV[m];  // p'(row, xb + dl) BoxA
            P[0][m] = shl1_add(P[0][m], rbc<m>(cxo) * HV[m]);
        });
        sidx = sidx + 1 == K ? 0 : sidx + 1;
#pragma unroll
        for (int m = 0; m < TRW; ++m) {
            rA[m] = amv[m];
            rB[m] = bv[m];
            rT[m] = t1v[m];
        }
    };

    Ld L[BDP + 1];
    load_cols(sc, shY, w0);  // the first step's columns, all lanes
    load_cam(w0);  // CAML: the first block (written to LDS at step w0)
    issue(w0, L[0], std::true_type{});
    if constexpr (BDP == 2) issue(w0 + 1, L[1], std::true_type{});
    // The prologue's loads land before the loop: the compiler joins the prologue to the loop with
    // register copies where it assigns the loop's registers differently (it takes an asm load's
    // destination as written at issue), and a copy of a register whose load is still in flight reads
    // what the previous wave on the SIMD left there.  (k = 2..4 did: the window k = 4 backward was
    // wrong on cold caches -- the first call of a process, or after another large kernel.)
    asm_vmcnt<0>();
#pragma unroll
    for (int i = 0; i <= BDP; ++i) tie(L[i]);
    tie_cols();
    if constexpr (BDP == 2) {
        for (int wfirst = w0; wfirst < wend; wfirst += FBC) {
            const int nsteps = min(FBC, wend - wfirst);  // FBC = a multiple of BDP + 1: blocks start on L[0]
            const bool fl = wfirst > w0;
            for (int s = 0; s < nsteps; s += 3) {
                step(L[0], L[2], wfirst + s, s, fl);
                if (s + 1 >= nsteps) break;
                step(L[1], L[0], wfirst + s + 1, s + 1, fl);
                if (s + 2 >= nsteps) break;
                step(L[2], L[1], wfirst + s + 2, s + 2, fl);
            }
            reduce_to(nsteps - 1);
            flush(wfirst, nsteps);
        }
    } else {
        // Full blocks (FBC steps, FBC even: a block starts and ends on L[0]), then the last, shorter
        // one.  No exit of the full-block loop depends on a step count, so the compiler's control-flow
        // graph has no path from a block that ended on an odd step into the next block (on such a path
        // it may take the pending L[1] loads as dead and reuse their registers, vmcnt_check.py).
        static_assert(FBC % 2 == 0, "a full block ends on L[0]");
        int wfirst = w0;
        for (; wfirst + FBC <= wend; wfirst += FBC) {
            step(L[0], L[1], wfirst, 0, std::true_type{});
            for (int s = 1; s < FBC - 1; s += 2) {
                step(L[1], L[0], wfirst + s, s, std::false_type{});
                step(L[0], L[1], wfirst + s + 1, s + 1, std::false_type{});
            }
            step(L[1], L[0], wfirst + FBC - 1, FBC - 1, std::false_type{});
            reduce_to(FBC - 1);
            flush(wfirst, FBC);
        }
        // (the last step's loads have landed where the two paths below join: the compiler joins them
        // with register copies too -- of loads past the segment's end, dead, but kept provable)
        asm_vmcnt<0>();
        tie(L[0]);
        tie_cols();
        if (wfirst < wend) {
            const int nsteps = wend - wfirst;
            step(L[0], L[1], wfirst, 0, std::true_type{});
            for (int s = 1; s < nsteps; s += 2) {
                step(L[1], L[0], wfirst + s, s, std::false_type{});
                if (s + 1 >= nsteps) break;
                step(L[0], L[1], wfirst + s + 1, s + 1, std::false_type{});
            }
            reduce_to(nsteps - 1);
            flush(wfirst, nsteps);
        }
    }
    // The last steps' prefetches are still in flight: keep their registers live (the compiler
    // would otherwise reuse them in the last flush) until they have landed.
    asm_vmcnt<0>();
#pragma unroll
    for (int i = 0; i <= BDP; ++i) tie(L[i]);
    tie_cols();
    // ---- final projector state: lane l holds column (wend - 1) + off + d0 + l
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int col = wend - 1 + (t == 0 ? -R0 : 0) + d0 + lane;
        const uint32_t c4 = (col >= 0 && col < g.W) ? (uint32_t)(col * 4) : kOOB;
        const auto rp = part_rsrc(3 + t);
#pragma unroll
        for (int m = 0; m < TRW; ++m) st_buf(P[t][m], rp, c4 == kOOB ? kOOB : c4 + (uint32_t)(m * Wi * 4));
    }
}

// The remainder diagonal D of a window with D = 64 n (BwdPlan::rem): its voxels (h, w, D) are the
// float right after the last chunk's 64 in every volume row, so every one of them is a separate
// 128-byte line.  They are not swept with the chunks: a fifth chunk of sweeps with one live lane
// in 64, or light units whose lanes are unit rows (eight loads per step, each lane a different
// line of the gradient, the volume and the six prepared images: 445 M line requests per C5 launch
// beside the sweep's ~1 G), both cost k_bwd_coop ~4 ms at C5 (20.8 ms without the diagonal,
// profiles/r03/rem); so does copying the two values out in the last chunk's sweep (two more
// lane-masked loads per step: +1.8 ms, the sweep is bound by its line requests).
// k_bwd_rem_rows instead walks ROWS with lanes = 64 consecutive camera columns w: per step (volume
// row h) ONE strided load (the gradient at diagonal D: one line per lane, unavoidable), the
// prepared-image values coalesced, A_D and V_D, the vertical box of A_D as a K-deep sliding sum (ring in
// LDS), the horizontal box through a wave-private LDS row (no
// barrier), and the six terms stored per row (a.remT / a.remT1, added by k_bwd_gather).
// The cost of diagonal D is recomputed from the images instead of read from the volume (a second
// line per voxel; the reference's backward recomputes every voxel's cost, stereo_matching_kernel.cu:
// 97-151): E + eps = sum c p - box_c box_p / k^2 + eps in fp64 (the products of row h + R enter a
// K-deep ring of their horizontal box sums, so the patch sum is exact for fp16 inputs and within
// the forward's own fp64 arithmetic for fp32), cost = (float)(E + eps) rsq(X Y + eps) with the
// same fp32 moments as A_D.  A wave owns the 64 - 2R middle columns of its 64 (the outer R on each
// side only feed the horizontal boxes); one wave per (column tile, row band).
constexpr int kRemRB = 64;  // output rows per row band (at most; run_bwd halves it on small grids)
#ifndef CUSTMA_REM_WAVES
#define CUSTMA_REM_WAVES 4096
#endif
constexpr int kRemWaves = CUSTMA_REM_WAVES;  // waves k_bwd_rem_rows aims for (A/B builds set CUSTMA_REM_WAVES)

template <int K>
__global__ __launch_bounds__(256) void k_bwd_rem_rows(Geo g, BwdArgs a, int ntile, int rb) {
    constexpr int R = K / 2, OWN = 64 - 2 * R;
    __shared__ float xs_[4][64];
    __shared__ double xp_[4][64];
    __shared__ float ringA_[4][K * 64];
    __shared__ double ringP_[4][K * 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t unit = (int64_t)blockIdx.x * 4 + wv;
    const int tile = (int)(unit % ntile);
    const int64_t band = unit / ntile;
    const int64_t y0 = a.ylo + band * rb;
    if (y0 >= a.yhi) return;
    const int64_t y1 = min(a.yhi, y0 + rb);
    const int Wi = (int)g.W, WOi = (int)g.WO, Di = (int)g.D, hlo = (int)g.h_lo, hhi = (int)g.h_hi, Hi = (int)g.H;
    const int x0 = -R + tile * OWN;          // first output column of this wave
    const int w = x0 - R + lane;             // this lane's camera column (voxel column)
    const bool own = lane >= R && lane < 64 - R;  // lane's column is one of this wave's outputs
    const bool wok = w >= 0 && w < WOi;      // a voxel column of diagonal D
    const size_t slab = (size_t)g.WO * g.DO, plane = (size_t)g.H * g.W;
    const float cb = a.shift[0], pb = a.shift[1];
    const uint32_t pb4 = (uint32_t)(plane * 4);
    enum { kX = 0, kMc = 1, kC = 2, kY = 3, kMp = 4, kP = 5 };
    // gradient rows of this band: [y0 - R, y1 + R) clipped to [h_lo, h_hi); offsets relative to vb
    const int vb = (int)max((int64_t)hlo, y0 - R);
    const auto rG = make_rsrc(a.grad + (size_t)(vb - hlo) * slab, 0x7FFFFFF0u);
    const auto rP = make_rsrc(a.Xc, 0x7FFFFFF0u);
    const auto rBc = make_rsrc(a.sc.box, (uint32_t)min((size_t)0x7FFFFFF0u, plane * 8));
    const auto rBp = make_rsrc(a.sp.box, (uint32_t)min((size_t)0x7FFFFFF0u, plane * 8));
    constexpr uint32_t OOB = 0x80000000u;
    const uint32_t vcol = wok ? (uint32_t)((size_t)w * g.DO + Di) * 4u : OOB;  // voxel (., w, D) in a row
    const uint32_t vstride = (uint32_t)(slab * 4);
    const int64_t nvR = g.HV() * g.WO, nywR = (a.yhi - a.ylo) * g.W;
    const auto rT = make_rsrc(a.remT, (uint32_t)(4 * nvR * 4));
    const auto rT1 = make_rsrc(a.remT1, (uint32_t)(2 * nywR * 4));
    float* xs = xs_[wv];
    double* xp = xp_[wv];
    const double rk2 = 1.0 / (double)(K * K);
    struct Ld { float g, x, y, mp, mc, c, p, pv, cv; double bc, bp; };
    // loads of volume row h (zero outside the volume rows / columns: A_D = 0 there), the raw
    // images of row h + R (the product row that enters the patch sums at step h) and the raw
    // images of output row y = h - R (its T1 terms)
    auto load = [&](int h, Ld& b) {
        const bool hv = h >= hlo && h < hhi, hi = h >= 0 && h < Hi;
        const uint32_t vo = hv && vcol != OOB ? (uint32_t)(h - vb) * vstride + vcol : OOB;
        const uint32_t io = hi ? (uint32_t)(h * Wi) * 4u : OOB;
        b.g = ld_buf<float>(rG, vo);
        b.x = ld_buf<float>(rP, io != OOB && w >= 0 && w < Wi ? io + (uint32_t)w * 4u + kX * pb4 : OOB);
        b.y = ld_buf<float>(rP, io != OOB && wok ? io + (uint32_t)(w + Di) * 4u + kY * pb4 : OOB);
        const bool ow = io != OOB && wok && own;
        b.mp = ld_buf<float>(rP, ow ? io + (uint32_t)(w + Di) * 4u + kMp * pb4 : OOB);
        b.mc = ld_buf<float>(rP, ow ? io + (uint32_t)w * 4u + kMc * pb4 : OOB);
        b.bc = ld_buf_f64(rBc, ow ? (uint32_t)(h * Wi + w) * 8u : OOB);
        b.bp = ld_buf_f64(rBp, ow ? (uint32_t)(h * Wi + w + Di) * 8u : OOB);
        const int he = h + R;
        const bool ei = he >= 0 && he < Hi;
        const uint32_t eo = (uint32_t)(he * Wi) * 4u;
        b.c = ld_buf<float>(rP, ei && w >= 0 && w < Wi ? eo + (uint32_t)w * 4u + kC * pb4 : OOB);
        b.p = ld_buf<float>(rP, ei && w + Di >= 0 && w + Di < Wi ? eo + (uint32_t)(w + Di) * 4u + kP * pb4 : OOB);
        const int yo = h - R;
        const bool yi = own && yo >= 0 && yo < Hi;
        const uint32_t yb = (uint32_t)(yo * Wi) * 4u;
        b.pv = ld_buf<float>(rP, yi && w + Di >= 0 && w + Di < Wi ? yb + (uint32_t)(w + Di) * 4u + kP * pb4 : OOB);
        b.cv = ld_buf<float>(rP, yi && w >= 0 && w < Wi ? yb + (uint32_t)w * 4u + kC * pb4 : OOB);
    };
    // horizontal box over the lanes x - R .. x + R of a product row (own lanes)
    auto hbox = [&](double v) {
        xp[lane] = v;
        // other lanes' slots are read next: keep those loads after this store (a wave's LDS
        // accesses execute in program order; this pins the compiler's order)
        __builtin_amdgcn_wave_barrier();
        double c[2 * R + 1];
#pragma unroll
        for (int j = 0; j <= 2 * R; ++j) c[j] = xp[own ? lane - R + j : 0];
        return tree_sum<2 * R + 1>(c);
    };
    // the two K-deep rings in LDS (wave-private; a register ring needs the row loop unrolled K times,
    // and then the compiler keeps every step's horizontal-box operands live: 270+ VGPRs at k = 11)
    float* ring = ringA_[wv];    // [K][64] A_D of the last K rows (slot = step mod K)
    double* ringP = ringP_[wv];  // [K][64] horizontal box sums of c p of the last K product rows
#pragma unroll
    for (int i = 0; i < K; ++i) { ring[i * 64 + lane] = 0.f; ringP[i * 64 + lane] = 0.0; }
    float VS = 0.f;   // vertical sum of A_D over rows h - K + 1 .. h
    double SP = 0.0;  // patch sum of c p at (h, w): the product rows h - R .. h + R
    const int hs = (int)(y0 - R), he = (int)(y1 + R);  // rows walked; output y = h - R for y in [y0, y1)
    // warm-up: product rows hs - R .. hs + R - 1 into slots 1 .. K - 1 (step t puts row hs + t + R
    // into slot t mod K, evicting row hs + t - R - 1)
    for (int jj = 0; jj < K - 1; ++jj) {
        const int ry = hs - R + jj;
        const bool ei = ry >= 0 && ry < Hi;
        const uint32_t eo = (uint32_t)(ry * Wi) * 4u;
        const float c = ld_buf<float>(rP, ei && w >= 0 && w < Wi ? eo + (uint32_t)w * 4u + kC * pb4 : OOB);
        const float p = ld_buf<float>(rP, ei && w + Di >= 0 && w + Di < Wi ? eo + (uint32_t)(w + Di) * 4u + kP * pb4 : OOB);
        const double pe = hbox((double)c * (double)p);
        ringP[(jj + 1) * 64 + lane] = pe;
        SP += pe;
    }
    // Loads RP - 1 steps ahead in a ring of RP buffers indexed at compile time (the step loop unrolled RP
    // times), so that no register copy at the loop's back edge waits for the newest loads, and every load
    // of a step -- the strided gradient line included -- is issued RP - 1 steps before its use.  (Round 5:
    // one step ahead through a copy, with the T1 image loads issued and used inside the step, so each step
    // also waited for the next one's loads.)
    constexpr int RP = 4;
    Ld L[RP];
    int slot = 0;
    auto step = [&](Ld& cur, int h) {
        {  // product row h + R enters, row h - R - 1 leaves (the forward's sliding fp64 sums)
            const double pe = hbox((double)cur.c * (double)cur.p);
            SP = (SP + pe) - ringP[slot * 64 + lane];
            ringP[slot * 64 + lane] = pe;
        }
        const float rSD = __builtin_amdgcn_rsqf(__builtin_fmaf(cur.x, cur.y, kEps));
        const float AD = cur.g * rSD;
        VS += AD - ring[slot * 64 + lane];
        ring[slot * 64 + lane] = AD;
        slot = slot + 1 == K ? 0 : slot + 1;
        // per-voxel terms of (h, w): stored by the lanes that own column w
        if (own && wok && h >= hlo && h < hhi && h >= y0 && h < y1) {  // each row by one band
            // E + eps = sum c p - box_c box_p / k^2 + eps (the forward's fin_bc form)
            const double e = __builtin_fma(-cur.bc, cur.bp * rk2, SP + (double)kEps);
            const float VD = AD * ((float)e * rSD) * rSD;
            const uint32_t tv = (uint32_t)(((int64_t)(h - hlo) * WOi + w) * 4), tn = (uint32_t)(nvR * 4);
            st_buf(AD * cur.mp, rT, tv);           // camera Am at (h, w):  A mp'(h, w + D)
            st_buf(VD * cur.y, rT, tv + tn);       // camera B  at (h, w):  V Y(h, w + D)
            st_buf(AD * cur.mc, rT, tv + 2 * tn);  // projector Ac at (h, w + D): A mc'(h, w)
            st_buf(VD * cur.x, rT, tv + 3 * tn);   // projector Bp at (h, w + D): V X(h, w)
        }
        // output row y = h - R: BoxA_D(y, x) = sum of VS over the lanes x - R .. x + R
        const int y = h - R;
        if (y >= y0) {
            xs[lane] = VS;
            __builtin_amdgcn_wave_barrier();  // as in hbox: the cross-lane reads stay after the store
            float c[2 * R + 1];
#pragma unroll
            for (int j = 0; j <= 2 * R; ++j) c[j] = xs[own ? lane - R + j : 0];
            const float box = tree_sum<2 * R + 1>(c);
            const int x = w;  // output column of an own lane
            if (own) {
                const uint32_t ty = (uint32_t)((y - (int)a.ylo) * Wi * 4);
                // T1c at (y, x): p'(y, x + D) BoxA_D;  T1p at (y, x + D): c'(y, x) BoxA_D
                const int xd = x + Di;
                if (x >= 0 && x < Wi) st_buf((cur.pv - pb) * box, rT1, ty + (uint32_t)x * 4u);
                if (xd >= 0 && xd < Wi) st_buf((cur.cv - cb) * box, rT1, (uint32_t)(nywR * 4) + ty + (uint32_t)xd * 4u);
            }
        }
    };
    Unroll<0, RP - 1>::run([&](auto ic) { load(hs + decltype(ic)::value, L[decltype(ic)::value]); });
    int h = hs;
    for (; h + RP <= he; h += RP) {
        Unroll<0, RP>::run([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            load(h + i + RP - 1, L[(i + RP - 1) % RP]);  // past the band: in range or masked, unused
            step(L[i], h + i);
        });
    }
    Unroll<0, RP - 1>::run([&](auto ic) {  // the last < RP steps (their loads were issued above)
        constexpr int i = decltype(ic)::value;
        if (h + i < he) step(L[i], h + i);
    });
}

template <int K, bool WIN>
__global__ __launch_bounds__(64 * NWC) void k_bwd_coop(Geo g, BwdArgs a) {
    // XCD x owns row groups [x nRGx, (x+1) nRGx) (their halo rows are read on one XCD).
    // A wave's 256-byte gradient / volume row segment spans three 128-byte lines whose outer
    // parts the neighbouring diagonal chunk's workgroup reads at the same step; the order
    // decides whether those reads meet in the XCD's L2.
    // a.order 2 (window layouts): on an XCD, chunk rank fastest, then row group, then segment
    //   -- the few chunks of one (row group, segment) are dispatched together (C5 window:
    //   FETCH 140 -> 103 GB per launch, 37.1 -> 35.7 ms op).
    // a.order 1 (full layout, up to 2W/64 chunks of very different lengths): row group fastest,
    //   then chunk rank (longest first), then segment (C2 full: 4.36 -> 3.85-4.05 ms op).
    const int64_t hb = blockIdx.x, xi = hb / 8, x = hb % 8;
    const int nRGx = (a.nRG + 7) / 8;
    const int nU = a.nChunk;
    int j, sg, rg;
    if (a.order == 2) {
        const int jr = (int)(xi % nU);
        const int64_t rest = xi / nU;
        rg = (int)(x * nRGx + rest % nRGx);
        const int64_t sg64 = rest / nRGx;
        if (rg >= a.nRG || sg64 >= a.nsegMax) return;
        j = chunk_of_rank(jr, a.nChunk, a.jc);
        sg = (int)sg64;
    } else {
        const int64_t unit = xi / nRGx;
        rg = (int)(x * nRGx + xi % nRGx);
        if (rg >= a.nRG || unit >= (int64_t)nU * a.nsegMax) return;
        const int jr = (int)(unit % nU);
        j = chunk_of_rank(jr, a.nChunk, a.jc);
        sg = (int)(unit / nU);
    }
    if (sg >= chunk_nseg(chunk_geo(g, a.dlo, j), taps_of(g))) return;
    constexpr int NY = TRB + K - 1;
    __shared__ __attribute__((aligned(16))) float Abuf[2 * (NY + 1) * 64];  // + a spare row (halo A of no row)
    __shared__ __attribute__((aligned(16))) float ring[NWC * K * TRW * 64];
    constexpr int FBC = fbc_for<K>();
    __shared__ __attribute__((aligned(16))) float cbuf[NWC][FBC][12];
    __shared__ __attribute__((aligned(16))) float pbuf[NWC][FBC][12];
    constexpr int HPW = (K - 1 + NWC - 1) / NWC;
    __shared__ float camL[NWC][cam_lds_for<K>() ? (12 + (HPW > 0 ? HPW : 1)) * kCamP : 1];
    const int wv = threadIdx.x >> 6;
    bwd_coop_body<K, WIN>(g, a, j, sg, rg, Abuf, ring + wv * (K * TRW * 64), cbuf[wv], pbuf[wv], camL[wv]);
}

// Per (range class, column): the partial slots that hold the column (class 0 = camera
// T1c / Am / B, which share one range; 1 = projector T1p; 2 = projector Ac / Bp).
// cover layout: [3][W] counts, then [3][W][S] slot indices (uint16).
// k_bwd_cover counts every (chunk, segment) whose written range holds column x and lists the first S
// slot indices, in chunk order, then segment order.  plan_bwd's S bounds the count by construction
// (2 x the max chunk overlap, <= 2 segments per chunk); the device marks an over-full column with
// count -1, which k_bwd_gather turns into NaN gradients -- never a silently dropped slot.
// The slots of chunk j whose written range of class cls holds column x, in segment order (at most 2,
// adjacent segments; more are counted but not stored): their count, the first two into e.
__host__ __device__ inline int chunk_cover(const Geo& g, int64_t dlo, int Sj, int64_t x, int cls, int j,
                                           unsigned short* e) {
    const int t = cls == 0 ? 0 : cls == 1 ? 3 : 4;
    const ChunkGeo c = chunk_geo(g, dlo, j);
    int64_t lo, hi;
    type_range(c, taps_of(g), t, &lo, &hi);
    if (x < lo || x >= hi) return 0;
    const int ns = chunk_nseg(c, taps_of(g));
    const Taps tp = taps_of(g);
    const int64_t rel = x - (c.wlo - tp.r0) - (cls ? c.d0 : 0);
    // segments whose written range can hold x: relative to segment s's own first column
    // s seg, every range lies in [-k, seg + r0 + 63) (seg_range); checked exactly below
    auto fdiv = [](int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); };
    const int s_lo = (int)fdiv(rel - c.seg - tp.r0 - NLB, c.seg);
    const int s_hi = (int)fdiv(rel + g.k, c.seg);
    int n = 0;
    for (int sg = s_lo < 0 ? 0 : s_lo; sg <= s_hi; ++sg) {
        if (sg < 0 || sg >= ns) continue;
        seg_range(c, tp, sg, t, &lo, &hi);
        if (x >= lo && x < hi) {
            if (n < 2) e[n] = (unsigned short)(2 * (j % Sj) + (sg & 1));
            ++n;
        }
    }
    return n;
}
// One wave per (range class, column), lane = chunk (blocks of 64 chunks): each lane finds its chunk's slots
// and a ballot prefix places them after the lower chunks', so the list is in chunk order, then segment
// order -- the order k_bwd_gather sums in.  (Round 5: one thread per column ran the serial loop over
// every chunk and class, W threads in all: ~70-90 us at C2 full, where W / 256 = 4 workgroups.)
__global__ __launch_bounds__(256) void k_bwd_cover(Geo g, int64_t dlo, int nChunk, int S, int Sj, int* cover) {
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = (int)(threadIdx.x & 63);
    if (wid >= 3 * g.W) return;  // wave-uniform
    const int cls = (int)(wid / g.W);
    const int64_t x = wid - (int64_t)cls * g.W;
    unsigned short* list = (unsigned short*)(cover + 3 * g.W) + ((size_t)cls * g.W + x) * S;
    const uint64_t below = (1ull << lane) - 1;
    int n = 0;  // slots listed by the lower chunks (wave-uniform)
    for (int j0 = 0; j0 < nChunk; j0 += 64) {
        const int j = j0 + lane;
        unsigned short e[2] = {0, 0};
        const int c = j < nChunk ? chunk_cover(g, dlo, Sj, x, cls, j, e) : 0;
        const uint64_t b1 = __ballot(c >= 1), b2 = __ballot(c >= 2);
        const int pos = n + __popcll(b1 & below) + __popcll(b2 & below);
        if (c >= 1 && pos < S) list[pos] = e[0];
        if (c >= 2 && pos + 1 < S) list[pos + 1] = e[1];
        n += __popcll(b1) + __popcll(b2);
        // more than two segments of one chunk never hold a column (adjacent segments only); if one did,
        // the column reads as over-full (NaN gradients in k_bwd_gather), never as a dropped slot
        if (__ballot(c >= 3)) n = S + 1;
    }
    if (lane == 0) cover[cls * g.W + x] = n <= S ? n : -1;
}

// Sum of the partial slots of type 3 side + q at pixel p = (y, x) (fp64, even / odd slots in two
// accumulators, in the cover list's order), plus the remainder diagonal's term of that type
// (BwdArgs::remT / remT1, written by the last chunk's units).  The caller checks y in [ylo, yhi).
__device__ __forceinline__ double gather_sum(const Geo& g, const BwdArgs& a, const float* remT, const float* remT1,
                                             int side, int q, int64_t y, int64_t x, int64_t p) {
    const int64_t plane = g.H * g.W;
    const unsigned short* list = (const unsigned short*)(a.cover + 3 * g.W);
    const int t = 3 * side + q;
    const int cls = side == 0 ? 0 : (q == 0 ? 1 : 2);
    const int n = a.cover[cls * g.W + x];
    if (n < 0) return __builtin_nan("");  // more slots than planned (k_bwd_cover): fail loudly
    const unsigned short* sl = list + ((size_t)cls * g.W + x) * a.S;
    const float* base = a.part + (size_t)t * a.S * plane + p;
    double v0 = 0.0, v1 = 0.0;
    int i = 0;
    for (; i + 1 < n; i += 2) {
        v0 += (double)base[(size_t)sl[i] * plane];
        v1 += (double)base[(size_t)sl[i + 1] * plane];
    }
    if (i < n) v0 += (double)base[(size_t)sl[i] * plane];
    double s = v0 + v1;
    if (remT) {  // the remainder diagonal's terms (k_bwd_rem_rows)
        const int64_t nyw = (a.yhi - a.ylo) * g.W, nv = g.HV() * g.WO, yy = y - a.ylo, D = g.D;
        if (q == 0) {
            // written for camera columns x < WO + r (past them the box of diagonal D is empty) and
            // projector columns o >= D - r
            if (side == 0 ? x < g.WO + (g.k - 1 - g.r) : x >= D - g.r) s += (double)remT1[side * nyw + yy * g.W + x];
        } else {
            const int64_t w = side == 0 ? x : x - D;  // the voxel column of this pixel on diagonal D
            if (y >= g.h_lo && y < g.h_hi && w >= 0 && w < g.WO)
                s += (double)remT[(2 * side + q - 1) * nv + (y - g.h_lo) * g.WO + w];
        }
    }
    return s;
}

// The remainder diagonal's term of type 3 side + q at pixel (y, x) (BwdArgs::remT / remT1, k_bwd_rem_rows).
__device__ __forceinline__ double rem_term(const Geo& g, const BwdArgs& a, const float* remT, const float* remT1,
                                           int side, int q, int64_t y, int64_t x) {
    const int64_t nyw = (a.yhi - a.ylo) * g.W, nv = g.HV() * g.WO, yy = y - a.ylo, D = g.D;
    if (q == 0) {
        if (side == 0 ? x < g.WO + (g.k - 1 - g.r) : x >= D - g.r) return (double)remT1[side * nyw + yy * g.W + x];
        return 0.0;
    }
    const int64_t w = side == 0 ? x : x - D;
    if (y >= g.h_lo && y < g.h_hi && w >= 0 && w < g.WO) return (double)remT[(2 * side + q - 1) * nv + (y - g.h_lo) * g.WO + w];
    return 0.0;
}

// The three sums of one side at pixel p when every cover list holds <= 8 slots (a.S <= 8: window layouts
// up to four diagonal chunks): the lists first (4 dwords each; the camera side's three types share one
// list, the projector's Ac / Bp another), then every slot value of the three types at once (zero past a
// list's count), then the same fp64 sums in the same order as gather_sum (even / odd accumulators, list
// order; the zero terms leave them unchanged) -- three dependent memory round trips per pixel instead of
// one per slot pair.
__device__ __forceinline__ void gather_sums8(const Geo& g, const BwdArgs& a, const float* remT, const float* remT1,
                                             int side, int64_t y, int64_t x, int64_t p, double* s) {
    const int64_t plane = g.H * g.W;
    const unsigned short* list = (const unsigned short*)(a.cover + 3 * g.W);
    const int nw = a.S >> 1;  // dwords per list (S is even)
    int nq[3];
    uint32_t lw[3][4];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int cls = side == 0 ? 0 : (q == 0 ? 1 : 2);
        if (q > 0 && (side == 0 || q == 2)) {  // the same list as the previous type
            nq[q] = nq[q - 1];
#pragma unroll
            for (int w = 0; w < 4; ++w) lw[q][w] = lw[q - 1][w];
            continue;
        }
        nq[q] = a.cover[cls * g.W + x];
        const uint32_t* lp = (const uint32_t*)(list + ((size_t)cls * g.W + x) * a.S);
#pragma unroll
        for (int w = 0; w < 4; ++w) lw[q][w] = w < nw ? lp[w] : 0u;
    }
    // every slot load unconditional (a raw buffer load per type, past the list's count an out-of-range
    // offset reads 0): a bounds-tested load per slot was waited for one at a time.  A type's S slot
    // planes stay below 2 GiB (run_bwd picks this form only then), so a 32-bit offset reaches them.
    float v[3][8];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const uint64_t tb = (uint64_t)a.S * (uint64_t)plane * 4u;
        const auto rq = make_rsrc(a.part + (size_t)(3 * side + q) * a.S * plane, tb < 0x7FFFFFF0u ? (uint32_t)tb : 0x7FFFFFF0u);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t sl = (lw[q][i >> 1] >> (16 * (i & 1))) & 0xffffu;
            const uint32_t off = i < nq[q] ? (uint32_t)(((uint64_t)sl * (uint64_t)plane + (uint64_t)p) * 4u) : 0x80000000u;
            v[q][i] = ld_bufs<float>(rq, off, 0u);
        }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (nq[q] < 0) {  // more slots than planned (k_bwd_cover): fail loudly
            s[q] = __builtin_nan("");
            continue;
        }
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            v0 += (double)v[q][i];
            v1 += (double)v[q][i + 1];
        }
        s[q] = v0 + v1;
        if (remT) s[q] += rem_term(g, a, remT, remT1, side, q, y, x);
    }
}

// Per-pixel sums (k_bwd_gather -> k_bwd_combine3): fp64 sums of the fp32 chunk partials, stored as
// fp32 (one more rounding of values that are sums of fp32 partials already; the box filters and the
// final combination stay fp64).
typedef float acc_t;

// Sum the partial slots per pixel; out ([2 sides][3][H][W]): T1, Z = Am|Ac - m' B|Bp, B|Bp (k_bwd_combine3
// forms no patch sums: the gather forms m' B as it loads its tile -- the same product, one fp64 array less
// through HBM).
template <typename T, bool S8 = false>
__global__ __launch_bounds__(256) void k_bwd_gather(Geo g, BwdArgs a, acc_t* acc, const float* remT,
                                                    const float* remT1) {
    // blockIdx.y = the image row, x = the column, z = the side (no 64-bit division per thread)
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    const int64_t plane = g.H * g.W;
    if (x >= g.W) return;
    const int64_t p = y * g.W + x;
    const int side = blockIdx.z;
    double s[3] = {0.0, 0.0, 0.0};
    if (y >= a.ylo && y < a.yhi) {
        if constexpr (S8) {
            gather_sums8(g, a, remT, remT1, side, y, x, p, s);
        } else {
#pragma unroll
            for (int q = 0; q < 3; ++q) s[q] = gather_sum(g, a, remT, remT1, side, q, y, x, p);
        }
    }
    // Z = A - m' B (m' = box / k^2 - shift, the pixel's shifted patch mean): k_bwd_combine3 then
    // needs two box filters, Box[Z] = Box[A] - Box[m' B], and no patch sums
    const double* box = side == 0 ? a.sc.box : a.sp.box;
    s[1] -= s[2] * (box[p] / (double)(g.k * g.k) - (double)a.shift[side]);
    acc_t* o = acc + (size_t)side * 3 * plane;
    o[p] = (acc_t)s[0];
    o[plane + p] = (acc_t)s[1];
    o[2 * plane + p] = (acc_t)s[2];
}

// grad(y,x) = T1 - Box[Z] - img'(y,x) Box[B]   (k_bwd_gather2's Z = A - m' B; one side per blockIdx.z)
// TS x TS output tiles (TS = 32: the (TS + 2r)^2 input halo is 1.7x the tile, 2.6x at 16); inputs
// staged as fp32 (they are stored so), row sums and column sums in fp64, fixed order.
// KT > 0: the window size at compile time (the sweep's sizes: unrolled tap loops, constant tile
// pitch; C5 0.72 -> 0.58 ms); KT = 0: runtime k.
template <typename T, int TS, int KT = 0>
__global__ __launch_bounds__(256) void k_bwd_combine3(Geo g, const T* __restrict__ cam, const T* __restrict__ proj,
                                                      const float* __restrict__ shift, const acc_t* __restrict__ acc,
                                                      float* __restrict__ dcam, float* __restrict__ dproj) {
    extern __shared__ __attribute__((aligned(16))) double tl[];
    const int side = blockIdx.z;
    float* out = side == 0 ? dcam : dproj;
    if (!out) return;
    const T* img = side == 0 ? cam : proj;
    const int64_t plane = g.H * g.W;
    const acc_t* T1 = acc + (size_t)side * 3 * plane;
    const acc_t* Zz = T1 + plane;
    const acc_t* Bb = Zz + plane;
    // Box over rows y - r1 .. y + r0 and columns x - r1 .. x + r0 (r1 = k-1-k/2: the transpose of the forward's
    // patch); the tile's inputs start r1 rows / columns before the outputs
    const int k = KT > 0 ? KT : g.k, r = k - 1 - k / 2, L = TS + k - 1;
    double* hZ = tl;                 // [L][TS] row sums
    double* hB = hZ + L * TS;
    float* tZ = (float*)(hB + L * TS);  // [L][L] inputs
    float* tB = tZ + L * L;
    const int64_t y0 = (int64_t)blockIdx.y * TS, x0 = (int64_t)blockIdx.x * TS;
    const int Hi = (int)g.H, Wi = (int)g.W;
    // the input tile through unconditional raw buffer loads (outside the image: an out-of-range offset,
    // read as 0), four items per thread in flight together; a bounds-tested load per item was waited for
    // one at a time.  Each plane stays below 2 GiB (backward_supported: H W 24 < 2^31).
    const auto rZ = make_rsrc(Zz, (uint32_t)(plane * 4)), rB = make_rsrc(Bb, (uint32_t)(plane * 4));
    for (int e0 = 0; e0 < L * L; e0 += 4 * 256) {
        float z[4], bb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = e0 + (int)threadIdx.x + 256 * i, ee = e < L * L ? e : 0;
            const int y = (int)y0 + ee / L - r, x = (int)x0 + ee % L - r;
            const bool ok = e < L * L && y >= 0 && y < Hi && x >= 0 && x < Wi;
            const uint32_t off = ok ? (uint32_t)(((int64_t)y * Wi + x) * 4) : 0x80000000u;
            z[i] = ld_bufs<float>(rZ, off, 0u);
            bb[i] = ld_bufs<float>(rB, off, 0u);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = e0 + (int)threadIdx.x + 256 * i;
            if (e < L * L) {
                tZ[e] = z[i];
                tB[e] = bb[i];
            }
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < L * TS; e += 256) {
        const int ry = e / TS, cx = e % TS;
        double a = 0, b = 0;
#pragma unroll
        for (int jx = 0; jx < k; ++jx) {
            const int f = ry * L + cx + jx;
            a += (double)tZ[f];
            b += (double)tB[f];
        }
        hZ[e] = a;
        hB[e] = b;
    }
    __syncthreads();
    const double sh = (double)shift[side];
    // the pixels' T1 and image values first, all in flight together (out-of-range offsets past the image)
    static_assert(TS * TS % 256 == 0, "whole output items per thread");
    constexpr int NO = TS * TS / 256;
    const auto rT = make_rsrc(T1, (uint32_t)(plane * 4)), rI = make_rsrc(img, (uint32_t)(plane * sizeof(T)));
    float tv[NO], iv[NO];
#pragma unroll
    for (int j = 0; j < NO; ++j) {
        const int e = (int)threadIdx.x + 256 * j, ly = e / TS, lx = e % TS;
        const int64_t y = y0 + ly, x = x0 + lx;
        const bool ok = y < g.H && x < g.W;
        const int64_t q = y * g.W + x;
        tv[j] = ld_bufs<float>(rT, ok ? (uint32_t)(q * 4) : 0x80000000u, 0u);
        iv[j] = ld_bufs<T>(rI, ok ? (uint32_t)(q * (int64_t)sizeof(T)) : 0x80000000u, 0u);
    }
#pragma unroll
    for (int j = 0; j < NO; ++j) {
        const int e = (int)threadIdx.x + 256 * j, ly = e / TS, lx = e % TS;
        const int64_t y = y0 + ly, x = x0 + lx;
        if (y >= g.H || x >= g.W) continue;
        double sz = 0, sb = 0;
#pragma unroll
        for (int i = 0; i < k; ++i) {
            const int f = (ly + i) * TS + lx;
            sz += hZ[f];
            sb += hB[f];
        }
        const int64_t q = y * g.W + x;
        const double ip = (double)iv[j] - sh;
        out[q] = (float)((double)tv[j] - sz - ip * sb);
    }
}

// Image means (the global shifts cbar, pbar): per-block fp64 sums (blockIdx.y = the image; four
// independent loads in flight per thread -- one dependent load at a time left this HBM-latency
// bound: 103 us per image at 4096 x 8192), then one block.
template <typename T>
__global__ __launch_bounds__(256) void k_img_blocksum(const T* __restrict__ img0, const T* __restrict__ img1,
                                                      int64_t n, double* bsum) {
    __shared__ double red[256];
    const T* __restrict__ img = blockIdx.y ? img1 : img0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const float a = to_f(img[i]), b = to_f(img[i + stride]), c = to_f(img[i + 2 * stride]),
                    d = to_f(img[i + 3 * stride]);
        v0 += (double)a;
        v1 += (double)b;
        v2 += (double)c;
        v3 += (double)d;
    }
    for (; i < n; i += stride) v0 += (double)to_f(img[i]);
    double v = (v0 + v1) + (v2 + v3);
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}
__global__ __launch_bounds__(256) void k_img_shift(const double* __restrict__ bsum, int nb, int64_t n, float* shift) {
    __shared__ double red[256];
    for (int side = 0; side < 2; ++side) {
        double v = 0.0;
        for (int i = threadIdx.x; i < nb; i += 256) v += bsum[side * nb + i];
        red[threadIdx.x] = v;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
            __syncthreads();
        }
        if (threadIdx.x == 0) shift[side] = n > 0 ? (float)(red[0] / (double)n) : 0.f;
        __syncthreads();
    }
}

// fp32 images for the sweep (after the shifts are known; written by the statistics pass,
// stats.hip STATS_BWD_PREP): X = camera centred moment, mc' = camera patch mean - cbar,
// c = camera; Y, mp', p likewise for the projector.  The images stay unshifted so that a
// zero-padded (out-of-image) load minus the shift gives the shifted padding value -cbar / -pbar.

constexpr int kSumBlocks = 512;

// CUSTMA_BWD_GATHER8=0 keeps the per-slot-pair gather loop everywhere (same-box A/B)
inline bool gather8_enabled() {
    const char* e = getenv("CUSTMA_BWD_GATHER8");
    return !(e && e[0] == '0');
}

inline size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

struct BwdPlan {
    int nChunk, S, Sj, nRG, jc, nsegMax;
    bool ok;
    int64_t dlo, ylo, yhi;
    bool rem;  // window, D = 64 n: diagonal D handled by k_bwd_rem_rows, not a chunk
    size_t part_bytes, acc_bytes, cover_bytes, prep_bytes, misc_bytes, rem_bytes;
};

// The window form's in-range offsets must stay below kWinNR: the gradient / volume rows one unit
// reads (+ one row of columns and diagonals), and the six prepared images.
bool win_path_ok(const Geo& g) {
    const double slab = (double)g.WO * (double)g.DO * 4.0;
    return g.layout == CUSTMA_LAYOUT_WINDOW && slab * (TRB + g.k + 1) < (double)kWinNR &&
           (double)g.H * (double)g.W * 24.0 < (double)kWinNR;
}

BwdPlan plan_bwd_uncached(const Geo& g);

// plan_bwd runs from custma_workspace_bytes, backward_supported and the backward itself: the plans
// of the last few geometries are kept (the full layout's chunk sweep is 2W/64 chunk ranges)
BwdPlan plan_bwd(const Geo& g) {
    struct Entry {
        int64_t H, W, D, h_lo, h_hi;
        int k, layout, seg_min;
        BwdPlan p;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const Entry& e : cache)
            if (e.H == g.H && e.W == g.W && e.D == g.D && e.h_lo == g.h_lo && e.h_hi == g.h_hi && e.k == g.k &&
                e.layout == g.layout && e.seg_min == g.seg_min)
                return e.p;
    }
    const BwdPlan p = plan_bwd_uncached(g);
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 16) cache.erase(cache.begin());
    cache.push_back(Entry{g.H, g.W, g.D, g.h_lo, g.h_hi, g.k, g.layout, g.seg_min, p});
    return p;
}

BwdPlan plan_bwd_uncached(const Geo& g) {
    BwdPlan p;
    const Taps tp = taps_of(g);
    p.rem = false;
    if (g.layout == CUSTMA_LAYOUT_WINDOW) {
        p.dlo = 0;
        p.nChunk = (int)cdiv((int64_t)g.D + 1, NLB);
        p.jc = 0;
        // D = 64 n: the last diagonal alone would take a fifth chunk of sweeps with one live lane
        // in 64; k_bwd_rem_rows takes it instead (the window form only)
        if (g.D >= NLB && (g.D + 1) % NLB == 1 && win_path_ok(g) && g.k % 2 == 1) {
            p.rem = true;
            p.nChunk -= 1;
        }
    } else {
        p.dlo = -(g.W - 1);
        p.nChunk = (int)cdiv(2 * g.W - 1, NLB);
        const int64_t jc = (-32 - p.dlo) / NLB;
        p.jc = (int)(jc < 0 ? 0 : jc >= p.nChunk ? p.nChunk - 1 : jc);
    }
    // slots: 2 x the max number of chunks covering one column over the four range classes
    // (segment parity separates the overlapping projector ranges of adjacent segments): max
    // interval overlap by a sweep over the sorted range ends.  An allocation failure leaves
    // p.ok false, which backward_supported() reports (never a silently undersized S).
    p.S = 1;
    p.ok = true;
    try {
        const int64_t W = g.W;
        const int ts[4] = {0, 1, 3, 4};
        std::vector<std::pair<int64_t, int>> ev;
        ev.reserve(2 * (size_t)p.nChunk);
        for (int c = 0; c < 4; ++c) {
            ev.clear();
            for (int j = 0; j < p.nChunk; ++j) {
                int64_t lo, hi;
                type_range(chunk_geo(g, p.dlo, j), tp, ts[c], &lo, &hi);
                lo = lo < 0 ? 0 : lo;
                hi = hi > W ? W : hi;
                if (lo < hi) { ev.emplace_back(lo, 1); ev.emplace_back(hi, -1); }
            }
            std::sort(ev.begin(), ev.end());  // at equal positions the -1 (range end) comes first
            int run = 0;
            for (const auto& e : ev) {
                run += e.second;
                if (run > p.S) p.S = run;
            }
        }
    } catch (...) {
        p.ok = false;
    }
    // S = 2 x the max overlap bounds every column's cover count by construction (segment parity
    // separates adjacent segments' ranges); k_bwd_cover still marks a column that would exceed it
    // (count -1 -> NaN gradients in k_bwd_gather), the runtime guard that never drops a slot silently
    p.Sj = p.S;
    p.S = 2 * p.Sj;
    p.nsegMax = 1;
    for (int j = 0; j < p.nChunk; ++j) {
        const int ns = chunk_nseg(chunk_geo(g, p.dlo, j), tp);
        if (ns > p.nsegMax) p.nsegMax = ns;
    }
    // gradient rows: voxel row h feeds output rows h - r0 .. h + r1
    p.ylo = g.h_lo - tp.r0 > 0 ? g.h_lo - tp.r0 : 0;
    p.yhi = g.h_hi + tp.r1 < g.H ? g.h_hi + tp.r1 : g.H;
    p.nRG = (int)cdiv(p.yhi - p.ylo, TRB);
    const size_t plane = (size_t)g.H * g.W;
    p.part_bytes = (size_t)NTYPE * p.S * plane * sizeof(float);
    p.acc_bytes = 6 * plane * sizeof(acc_t);
    p.cover_bytes = 3 * (size_t)g.W * sizeof(int) + 3 * (size_t)g.W * p.S * sizeof(unsigned short);
    p.prep_bytes = 6 * plane * sizeof(float);
    p.misc_bytes = 2 * kSumBlocks * sizeof(double) + 256;
    // A of diagonal D [HV][WO] (fp32) and its vertical box [yhi - ylo][WO] (fp64)
    // remA [HV][WO] f32, its vertical box [yhi - ylo][WO] f64, remT [4][HV][WO] f32, remT1 [2][yhi - ylo][W] f64
    // remT [4][HV][WO] f32, remT1 [2][yhi - ylo][W] f32 (BwdArgs)
    p.rem_bytes = p.rem ? a256((size_t)4 * g.HV() * g.WO * 4) + (size_t)2 * (p.yhi - p.ylo) * g.W * 4 : 0;
    return p;
}


// Workgroups of k_bwd_coop resident at once on the current device (0 if unknown).
template <int K, bool WIN>
int coop_slots() {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_bwd_coop<K, WIN>, 64 * NWC, 0) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return per * cus;
}

// Filling the chip in k_bwd_coop's grid.  A launch of U units (chunk, column segment, row group) on `slots`
// resident workgroups of which U < slots leaves CUs idle (configs[2]'s window at 1024^2, D = 128: 256 units on
// 512 slots).  There, more and narrower column segments fill the chip at the price of their k - 1 halo steps
// each: pick the minimum segment count (Geo::seg_min) with the best estimate of
//     (U / slots) / ceil(U / slots) x (span / (span + nseg (k - 1))),
// changing the default only for a gain above 1 %: configs[2] window backward 0.62 -> 0.52 ms.  With a round or
// more of units the same estimate also predicted gains for a partial last round (a C5 rank band at N = 8:
// 33 row groups, 4.1 rounds), but narrower segments measured 2-3 % slower there and at C2 full (their loads,
// flushes and 64 extra projector columns per segment), so those grids keep the default (profiles/r06/h, i:
// C5 rank band 3.46 -> 3.38 ms with the restriction).  The partial slots and cover lists (BwdPlan::S) do not
// depend on the segmentation (a chunk's written ranges are the union of its segments'), so the workspace
// custma_workspace_bytes sized still fits; run_bwd checks that.
int tail_seg_min_uncached(const Geo& g, int slots);
int tail_seg_min(const Geo& g, int slots) {
    struct Entry {
        int64_t H, W, D, h_lo, h_hi;
        int k, layout, slots, seg_min;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const Entry& e : cache)
            if (e.H == g.H && e.W == g.W && e.D == g.D && e.h_lo == g.h_lo && e.h_hi == g.h_hi && e.k == g.k &&
                e.layout == g.layout && e.slots == slots)
                return e.seg_min;
    }
    const int n = tail_seg_min_uncached(g, slots);
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 16) cache.erase(cache.begin());
    cache.push_back(Entry{g.H, g.W, g.D, g.h_lo, g.h_hi, g.k, g.layout, slots, n});
    return n;
}
int tail_seg_min_uncached(const Geo& g, int slots) {
    if (slots <= 0) return 0;
    auto score = [&](int seg_min, int* nseg_out) -> double {
        Geo gg = g;
        gg.seg_min = seg_min;
        const BwdPlan p = plan_bwd(gg);
        if (!p.ok) return -1.0;
        int64_t units = 0, steps = 0, cols = 0;
        for (int j = 0; j < p.nChunk; ++j) {
            const ChunkGeo c = chunk_geo(gg, p.dlo, j);
            const int ns = chunk_nseg(c, taps_of(gg));
            units += (int64_t)ns * p.nRG;
            cols += c.whi - c.wlo;
            steps += (c.whi - c.wlo) + (int64_t)(ns + 1) * (g.k - 1);  // a segment sweeps its columns + k - 1 steps
        }
        if (units <= 0 || steps <= 0) return -1.0;
        *nseg_out = p.nsegMax;
        const double rounds = (double)units / slots;
        return rounds / std::ceil(rounds) * ((double)cols / (double)steps);
    };
    int n0 = 0;
    const double s0 = score(0, &n0);
    if (s0 <= 0.0) return 0;
    {
        const BwdPlan p = plan_bwd(g);
        int64_t units = 0;
        for (int j = 0; j < p.nChunk; ++j) units += (int64_t)chunk_nseg(chunk_geo(g, p.dlo, j), taps_of(g)) * p.nRG;
        if (units >= slots) return 0;  // the chip is full: narrower segments only add their overheads
    }
    double best = s0;
    int pick = 0;
    for (int n = n0 + 1; n <= n0 + 24; ++n) {
        int nn = 0;
        const double sc = score(n, &nn);
        if (nn < n) break;  // the slot-parity minimum width caps the count
        if (sc > best) { best = sc; pick = n; }
    }
    return best > s0 * 1.01 ? pick : 0;
}

template <typename T>
hipError_t run_bwd(const float* grad, const float* vol, const T* cam, const T* proj, const Geo& g_in, Stats sc,
                   Stats sp, float* dcam, float* dproj, void* ws, hipStream_t s) {
    Geo g = g_in;
    {
        int slots = 0;
        const bool win = win_path_ok(g);
        switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: slots = win ? coop_slots<KK, true>() : coop_slots<KK, false>(); break;
            CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
            default: break;
        }
#ifndef CUSTMA_NO_TAIL  // (A/B build: scripts/build_ablations.py no_tail)
        g.seg_min = tail_seg_min(g, slots);
#endif
        if (g.seg_min > 0 && plan_bwd(g).S != plan_bwd(g_in).S) g.seg_min = 0;  // (never: S is segmentation-free)
    }
    const BwdPlan p = plan_bwd(g);
    char* w = (char*)ws;
    float* part = (float*)w;
    w += a256(p.part_bytes);
    acc_t* acc = (acc_t*)w;
    w += a256(p.acc_bytes);
    int* cover = (int*)w;
    w += a256(p.cover_bytes);
    float* prep = (float*)w;
    w += a256(p.prep_bytes);
    double* bsum = (double*)w;
    float* shift = (float*)(bsum + 2 * kSumBlocks);
    const int64_t n = g.H * g.W;
    hipLaunchKernelGGL(k_img_blocksum<T>, dim3(kSumBlocks, 2), dim3(256), 0, s, cam, proj, n, bsum);
    hipLaunchKernelGGL(k_img_shift, dim3(1), dim3(256), 0, s, bsum, kSumBlocks, n, shift);
    hipLaunchKernelGGL(k_bwd_cover, dim3((unsigned)cdiv(3 * g.W * 64, 256)), dim3(256), 0, s, g, p.dlo, p.nChunk, p.S, p.Sj,
                       cover);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the patch sums (box, fp64, for k_bwd_gather) and the six prepared fp32 images in one pass
    // (stats.hip STATS_BWD_PREP; was box + sqt, then a separate k_bwd_prep pass over them)
    if ((e = launch_stats(cam, proj, std::is_same<T, __half>::value ? CUSTMA_F16 : CUSTMA_F32, g, sc, sp, s,
                          STATS_BWD_PREP, prep, shift)) != hipSuccess)
        return e;
    BwdArgs a;
    a.cam = cam; a.proj = proj; a.sc = sc; a.sp = sp;
    a.grad = grad; a.vol = vol; a.shift = shift; a.part = part; a.cover = cover;
    a.Xc = prep; a.mcc = prep + n; a.cc = prep + 2 * n; a.Yp = prep + 3 * n; a.mpp = prep + 4 * n; a.pp = prep + 5 * n;
    a.S = p.S; a.Sj = p.Sj; a.nChunk = p.nChunk; a.nRG = p.nRG; a.jc = p.jc; a.nsegMax = p.nsegMax;
    a.dlo = p.dlo; a.ylo = p.ylo; a.yhi = p.yhi;
    a.order = g.layout == CUSTMA_LAYOUT_WINDOW ? 2 : 1;
    a.remT = nullptr;
    a.remT1 = nullptr;
    if (p.rem) {
        char* rw = (char*)bsum + a256(p.misc_bytes);  // the plan's rem_bytes follow misc_bytes
        a.remT = (float*)rw;
        a.remT1 = (float*)(rw + a256((size_t)4 * g.HV() * g.WO * 4));
    }
    const int nU = p.nChunk;  // chunk ranks of units (p.rem: diagonal D by k_bwd_rem_rows)
    const int64_t units = (int64_t)nU * p.nsegMax * p.nRG;
    const unsigned blocks = (unsigned)(8 * (int64_t)nU * p.nsegMax * cdiv(p.nRG, 8));
    // k_bwd_rem_rows: one wave per (column tile of 64 - 2r owned columns over [-r, WO + r), row band)
    const int rem_tiles = (int)cdiv(g.WO + 2 * g.r, 64 - 2 * g.r);
    // Row bands of kRemRB rows, halved while the grid has fewer than kRemWaves waves: a wave walks its band
    // row by row with one strided gradient line per step, so a small grid (C3: 1088 waves of 64 rows, about
    // one per SIMD) is latency-bound; shorter bands walk more warm-up rows (K - 1 per band) in parallel.
    int rem_rb = kRemRB;
    while (rem_rb > 8 && (int64_t)rem_tiles * cdiv(p.yhi - p.ylo, rem_rb) < kRemWaves) rem_rb /= 2;
    const int64_t rem_units = (int64_t)rem_tiles * cdiv(p.yhi - p.ylo, rem_rb);
    if (units > 0) {
        const bool win = win_path_ok(g);
        prof_begin(PROF_BWD, s);
        switch (g.k) {
#define CUSTMA_K(KK)                                                                              \
    case KK:                                                                                             \
        if (win)                                                                                         \
            hipLaunchKernelGGL((k_bwd_coop<KK, true>), dim3(blocks), dim3(64 * NWC), 0, s, g, a);        \
        else                                                                                             \
            hipLaunchKernelGGL((k_bwd_coop<KK, false>), dim3(blocks), dim3(64 * NWC), 0, s, g, a);       \
        break;
            CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
            default: return hipErrorInvalidValue;
        }
        prof_end(PROF_BWD, s);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (p.rem) {
        switch (g.k) {
#define CUSTMA_K(KK)                                                                                             \
    case KK:                                                                                                            \
        hipLaunchKernelGGL((k_bwd_rem_rows<KK>), dim3((unsigned)cdiv(rem_units, 4)), dim3(256), 0, s, g, a, rem_tiles, \
                           rem_rb);                                                                                     \
        break;
            CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
            default: return hipErrorInvalidValue;
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // (gather and combine fused into one tiled pass -- the slot sums recomputed for each tile's r
    // halo -- measured slower: C5 backward op 29.5 -> 31.1 ms, C2 full 3.82 -> 3.95 ms)
    // (a column-wise form, cover lists staged in LDS once per 64 columns and each slot read for 4-8 rows at
    // once, measured slower: C5 1.82 -> 2.52-2.74 ms at 122-134 VGPRs against this kernel's 30)
    {
        const dim3 ggrid((unsigned)cdiv(g.W, 256), (unsigned)g.H, 2);
        // (the batched form's 32-bit buffer offsets reach one type's S partial planes while they stay
        // below 2 GiB; larger images take the per-slot-pair form)
        if (p.S <= 8 && gather8_enabled() && (double)p.S * (double)n * 4.0 < 2147483648.0)
            hipLaunchKernelGGL((k_bwd_gather<T, true>), ggrid, dim3(256), 0, s, g, a, acc, a.remT, a.remT1);
        else
            hipLaunchKernelGGL((k_bwd_gather<T, false>), ggrid, dim3(256), 0, s, g, a, acc, a.remT, a.remT1);
    }
    {
        constexpr int TS3 = 32;
        const int L3 = TS3 + g.k - 1;
        const size_t lds3 = sizeof(double) * 2 * L3 * TS3 + sizeof(float) * 2 * L3 * L3;
        const dim3 cgrid((unsigned)cdiv(g.W, TS3), (unsigned)cdiv(g.H, TS3), 2);
        auto go = [&](auto kc) {
            constexpr int KK = decltype(kc)::value;
            if ((e = allow_lds(k_bwd_combine3<T, TS3, KK>, lds3)) != hipSuccess) return;
            hipLaunchKernelGGL((k_bwd_combine3<T, TS3, KK>), cgrid, dim3(256), lds3, s, g, cam, proj, shift, acc, dcam,
                               dproj);
        };
        switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: go(std::integral_constant<int, KK>{}); break;
            CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
            default: go(std::integral_constant<int, 0>{});
        }
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

}  // namespace

size_t backward_workspace_bytes(const Geo& g) {
    const BwdPlan p = plan_bwd(g);
    return a256(p.part_bytes) + a256(p.acc_bytes) + a256(p.cover_bytes) + a256(p.prep_bytes) + a256(p.misc_bytes) +
           a256(p.rem_bytes);
}

bool backward_supported(const Geo& g) {
    // the six prepared fp32 images are addressed through one 32-bit buffer range
    if ((double)g.H * (double)g.W * 24.0 >= 2147483648.0) return false;
    // 32-bit buffer offsets: the volume rows one wave reads (16 + 2r + 1 row slabs) and one fp64
    // image must stay below 2 GiB
    if (!plan_bwd(g).ok) return false;
    const double slab = (double)g.WO * (double)g.DO * 4.0;
    return slab * (TRB + g.k) < 2147483648.0 && (double)g.H * (double)g.W * 8.0 < 2147483648.0;
}

hipError_t launch_backward(const float* grad, const float* vol, const void* cam, const void* proj, int dtype,
                           const Geo& g, Stats sc, Stats sp, float* dcam, float* dproj, void* ws, hipStream_t s) {
    if (dtype == CUSTMA_F16)
        return run_bwd(grad, vol, (const __half*)cam, (const __half*)proj, g, sc, sp, dcam, dproj, ws, s);
    return run_bwd(grad, vol, (const float*)cam, (const float*)proj, g, sc, sp, dcam, dproj, ws, s);
}

}  // namespace custma
