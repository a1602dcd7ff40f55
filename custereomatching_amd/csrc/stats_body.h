// Per-pixel patch statistics: the tile body of stats.hip's k_stats, also run by the fused forward's
// statistics workgroups (sweep_wave.hip).  See stats.hip for what each mode writes.
#pragma once
#include <type_traits>

#include "common.h"

namespace custma {
namespace stats_detail {
// A workgroup (256 threads) covers TX x TY pixels; a thread owns a PR x PC micro-tile (PR rows,
// PC = 2 adjacent columns), so every tap row it reads from LDS (k + 1 values, float2 reads)
// feeds up to 8 pixels -- 2 horizontally, 4 vertically.  Round 4: 1 x 4 micro-tiles read
// (k + 3) k single floats per 4 pixels (C3 forward statistics 0.106 ms, ~4x its VALU floor).
// The box-only modes (no fp32 chains) take PR = 2, and the modes with sums of squares 4-column row-sum
// items, to keep their LDS and registers at the old kernel's occupancy.
constexpr int TX = 32, PC = 2, NQC = TX / PC;
__host__ __device__ constexpr int pr_for(int mode) { return mode == STATS_BOX || mode == STATS_BWD_PREP ? 2 : 4; }
__host__ __device__ constexpr int ty_for(int mode) { return 256 / NQC * pr_for(mode); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// LDS image pitch (floats): >= TX + k (a tap row's float2 reads may take one value past the
// TX + k - 1 loaded ones) and = 8 (mod 16), so the four 16-lane groups of a wave (PR rows apart)
// start their float2 reads 32 banks apart
__host__ __device__ constexpr int lx_for(int k) {
    const int lx = TX + k;
    return lx + (24 - lx % 16) % 16;
}

// KT > 0: the window size as a compile-time constant (the sweep's instantiations), so the
// k^2 tap loops unroll and a tap row lives in registers; KT = 0: runtime k (taps read from LDS).
// MODE (StatsMode): which outputs are written.
//   STATS_FULL      mean, sq, box, sqt
//   STATS_BOX       box, sqt                  (the generic backward's statistics)
//   STATS_BWD_PREP  box and the fused sweep's prepared fp32 images (bwd_fused.hip k_bwd_prep's
//                   X = sqt, m' = box / k^2 - shift, raw image; image z at prep + 3 z planes)
//   STATS_FWD       sq, box                   (what the fast forward sweeps read)
//   STATS_MSB       mean, sq, box             (the disparity: its sweep reads sq, box, the exact
//                                              recheck mean, sq; the exact forward: mean, sq)
// One statistics tile (TX x TY pixels of image bz, tile (tbx, tby) of the row range [ybeg, yend)) by the 256
// threads of a workgroup; `lds_d` = the dynamic LDS of stats_lds_bytes().
template <typename V>
__device__ __forceinline__ void stats_put(V* p, V v) {
    *p = v;
}
template <typename T, int KT, int MODE>
__device__ __forceinline__ void stats_tile(const T* __restrict__ img0, const T* __restrict__ img1, const Geo& g,
                                           const Stats& st0, const Stats& st1, float* __restrict__ prep,
                                           const float* __restrict__ shift, int64_t ybeg, int64_t yend, int tbx,
                                           int tby, int bz, double* lds_d) {
    constexpr bool BOX_ONLY = MODE == STATS_BOX || MODE == STATS_BWD_PREP;
    constexpr bool SQT = MODE != STATS_FWD && MODE != STATS_MSB;  // the fp64 sums of squares only feed sqt
    constexpr int PR = pr_for(MODE), TY = ty_for(MODE);
    constexpr int RSEG = SQT ? 4 : 8;  // row-sum items: RSEG consecutive columns of one tile row per thread
    static_assert(PR % 2 == 0 && TX % RSEG == 0, "vertical pixel pairs; whole row-sum items");
    // bz: 0 = camera, 1 = projector (one launch for both images)
    const T* __restrict__ img = bz ? img1 : img0;
    const Stats& st = bz ? st1 : st0;
    const int k = KT > 0 ? KT : g.k, r0 = k / 2, LX = lx_for(k), LY = TY + k - 1;
    double* rs = lds_d;                               // [LY][TX] fp64 k-tap row sums
    double* rs2 = rs + (SQT ? LY * TX : 0);           // [LY][TX] fp64 k-tap row sums of squares
    float* tile = (float*)(rs2 + LY * TX);             // [LY][LX] zero-padded image tile
    // pixel rows [ybeg, yend) (STATS_BAND_ROWS: the volume rows only); taps rows / columns
    // -k/2 .. k-1-k/2 (the reference's kernel_size / 2 origin, stereo_matching_kernel.cu:44)
    const int64_t y0 = ybeg + (int64_t)tby * TY, x0 = (int64_t)tbx * TX;
    const int tid = threadIdx.x;
    const int TXK = TX + k - 1;
    // The tile through raw buffer loads over the image rows from ybase on: an element outside the image
    // takes an out-of-range offset and reads 0 (the reference's zero padding), so every load is
    // unconditional and the loads of all NIT items are in flight together (an exec-masked load per
    // element waited for each one: the pass was latency-bound, ~0.1 ms at C3 for 0.12 GB).
    {
        const int64_t ybase = y0 - r0 > 0 ? y0 - r0 : 0;
        const uint64_t nb = (uint64_t)(g.H > ybase ? g.H - ybase : 0) * (uint64_t)g.W * sizeof(T);
        const auto rimg = make_rsrc(img + ybase * g.W, nb < 0x7FFFFFF0u ? (uint32_t)nb : 0x7FFFFFF0u);
        const int total = LY * TXK;
        auto item = [&](int e, float& v) {
            const int ee = e < total ? e : 0;
            const int ty = ee / TXK, tx = ee - ty * TXK;
            const int64_t y = y0 + ty - r0, x = x0 + tx - r0;
            const bool in = e < total && y >= 0 && y < g.H && x >= 0 && x < g.W;
            v = ld_bufs<T>(rimg, in ? (uint32_t)(((y - ybase) * g.W + x) * (int64_t)sizeof(T)) : 0x80000000u, 0u);
        };
        auto put = [&](int e, float v) {
            if (e < total) {
                const int ty = e / TXK, tx = e - ty * TXK;
                tile[ty * LX + tx] = v;
            }
        };
        if constexpr (KT > 0) {
            constexpr int NIT = ((ty_for(MODE) + KT - 1) * (TX + KT - 1) + 255) / 256;
            float v[NIT];
#pragma unroll
            for (int i = 0; i < NIT; ++i) item(tid + 256 * i, v[i]);
#pragma unroll
            for (int i = 0; i < NIT; ++i) put(tid + 256 * i, v[i]);
        } else {
            for (int e0 = 0; e0 < total; e0 += 4 * 256) {
                float v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) item(e0 + tid + 256 * i, v[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) put(e0 + tid + 256 * i, v[i]);
            }
        }
    }
    __syncthreads();
    // row sums: RSEG columns of one tile row per item, each a k-long fp64 sum in tap order (exact
    // for fp32 inputs within a 2^29 dynamic range, so the order does not change the value)
#pragma unroll 1
    for (int it = tid; it < LY * (TX / RSEG); it += 256) {
        const int ty = it / (TX / RSEG), c0 = (it % (TX / RSEG)) * RSEG;
        const float* t = tile + ty * LX + c0;
        double a[RSEG], b[RSEG];
#pragma unroll
        for (int c = 0; c < RSEG; ++c) a[c] = b[c] = 0.0;
        if constexpr (KT > 0) {
            double v[KT + RSEG - 1];
#pragma unroll
            for (int j = 0; j < KT + RSEG - 1; ++j) v[j] = (double)t[j];
#pragma unroll
            for (int c = 0; c < RSEG; ++c)
#pragma unroll
                for (int j = 0; j < KT; ++j) {
                    a[c] += v[c + j];
                    if constexpr (SQT) b[c] = fma(v[c + j], v[c + j], b[c]);
                }
        } else {
            for (int j = 0; j < k; ++j)
#pragma unroll
                for (int c = 0; c < RSEG; ++c) {
                    const double v = (double)t[c + j];
                    a[c] += v;
                    if constexpr (SQT) b[c] = fma(v, v, b[c]);
                }
        }
        f64x2* o = (f64x2*)(rs + ty * TX + c0);
        f64x2* o2 = (f64x2*)(rs2 + ty * TX + c0);
#pragma unroll
        for (int c = 0; c < RSEG; c += 2) {
            o[c / 2] = f64x2{a[c], a[c + 1]};
            if constexpr (SQT) o2[c / 2] = f64x2{b[c], b[c + 1]};
        }
    }
    __syncthreads();
    const int qc = tid % NQC, qr = tid / NQC;  // pixel rows PR qr .. PR qr + PR-1, columns PC qc, PC qc + 1
    const int ly0 = PR * qr, lx0 = PC * qc;
    const float rk2 = (float)(k * k);
    // fp64 patch sums (k row sums down the column, tap order) and sums of squares (after the
    // fp32 chains, so that they are not live across them)
    double bx[PR][PC], b2[PR][PC];
    auto box_sums = [&]() {
#pragma unroll
        for (int p = 0; p < PR; ++p)
#pragma unroll
            for (int c = 0; c < PC; ++c) bx[p][c] = b2[p][c] = 0.0;
        // (partly unrolled: fully unrolled, every row's f64x2 reads are hoisted -- 114-120 VGPRs in the
        // box-only modes)
#pragma unroll 2
        for (int i2 = 0; i2 < k + PR - 1; ++i2) {
            const f64x2 u = *(const f64x2*)(rs + (ly0 + i2) * TX + lx0);
            f64x2 u2 = {0.0, 0.0};
            if constexpr (SQT) u2 = *(const f64x2*)(rs2 + (ly0 + i2) * TX + lx0);
#pragma unroll
            for (int p = 0; p < PR; ++p)
                if (i2 - p >= 0 && i2 - p < k) {
                    bx[p][0] += u.x;
                    bx[p][1] += u.y;
                    if constexpr (SQT) {
                        b2[p][0] += u2.x;
                        b2[p][1] += u2.y;
                    }
                }
        }
    };
    if constexpr (BOX_ONLY) {
        box_sums();
#pragma unroll
        for (int p = 0; p < PR; ++p) {
            const int64_t y = y0 + ly0 + p;
            if (y >= yend) break;
#pragma unroll
            for (int c = 0; c < PC; ++c) {
                const int64_t x = x0 + lx0 + c;
                if (x >= g.W) break;
                const double b = bx[p][c];
                const int64_t o = y * g.W + x;
                stats_put(st.box + o, b);
                const double c2 = b2[p][c] - b * b / (double)(k * k);
                const float sqt = (float)(c2 > 0.0 ? c2 : 0.0);
                if constexpr (MODE == STATS_BWD_PREP) {
                    const int64_t n = g.H * g.W;
                    float* pz = prep + 3 * n * bz;
                    stats_put(pz + o, sqt);
                    stats_put(pz + n + o, (float)(b / (double)(k * k) - (double)shift[bz]));
                    // raw: the sweep subtracts the shift after a zero-padded load
                    stats_put(pz + 2 * n + o, tile[(ly0 + p + r0) * LX + lx0 + c + r0]);
                } else {
                    stats_put(st.sqt + o, sqt);
                }
            }
        }
        return;
    }
    // The reference's fp32 mean and centred squares (custma/src/stereo_matching_kernel.cu:40-54,
    // :56-69): per pixel the taps arrive in (i, j) row-major order, each an IEEE add / fma on a
    // running fp32 value; a tap row read once feeds every pixel of the micro-tile whose patch
    // holds it.  Pixels (p, c), (p + 1, c) share the tap value: packed fp32 ops (the same IEEE
    // operation per half).
    const float* t = tile + ly0 * LX + lx0;
    float m[PR][PC], sq[PR][PC];
#pragma unroll
    for (int p = 0; p < PR; ++p)
#pragma unroll
        for (int c = 0; c < PC; ++c) m[p][c] = sq[p][c] = 0.f;
    // pass 0: sums; pass 1: centred squares (m = the pass-0 sum / k^2)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {
#pragma unroll
            for (int p = 0; p < PR; ++p)
#pragma unroll
                for (int c = 0; c < PC; ++c) m[p][c] = m[p][c] / rk2;
        }
        auto tap = [&](float& acc, float v, float mv) {
            if (pass == 0) acc = acc + v;
            else {
                const float d = v - mv;
                acc = __builtin_fmaf(d, d, acc);
            }
        };
        // tap rows one at a time (not unrolled: the row's k + 1 values stay the only live tap registers)
#pragma unroll 1
        for (int i2 = 0; i2 < k + PR - 1; ++i2) {
            if constexpr (KT > 0) {
                constexpr int NV = KT + PC - 1, NV2 = (NV + 1) / 2;
                float v[2 * NV2];
                const f32x2* tr = (const f32x2*)(t + i2 * LX);
#pragma unroll
                for (int j = 0; j < NV2; ++j) {
                    const f32x2 w = tr[j];
                    v[2 * j] = w.x;
                    v[2 * j + 1] = w.y;
                }
                // per vertical pixel pair: both patches hold the row -> packed; one -> scalar
#pragma unroll
                for (int pp = 0; pp < PR / 2; ++pp) {
                    const int pa = 2 * pp, pb = 2 * pp + 1;
                    const bool ina = i2 - pa >= 0 && i2 - pa < k, inb = i2 - pb >= 0 && i2 - pb < k;
                    if (ina && inb) {
#pragma unroll
                        for (int c = 0; c < PC; ++c) {
                            f32x2 a = pass == 0 ? f32x2{m[pa][c], m[pb][c]} : f32x2{sq[pa][c], sq[pb][c]};
                            const f32x2 mm = {m[pa][c], m[pb][c]};
#pragma unroll
                            for (int j = 0; j < KT; ++j) {
                                const f32x2 vv = {v[c + j], v[c + j]};
                                if (pass == 0) a = a + vv;
                                else {
                                    const f32x2 d = vv - mm;
                                    a = __builtin_elementwise_fma(d, d, a);
                                }
                            }
                            if (pass == 0) { m[pa][c] = a.x; m[pb][c] = a.y; }
                            else { sq[pa][c] = a.x; sq[pb][c] = a.y; }
                        }
                    } else if (ina || inb) {
                        const int p1 = ina ? pa : pb;
#pragma unroll
                        for (int c = 0; c < PC; ++c) {
                            float acc = pass == 0 ? m[p1][c] : sq[p1][c];
                            const float mv = m[p1][c];
#pragma unroll
                            for (int j = 0; j < KT; ++j) tap(acc, v[c + j], mv);
                            if (pass == 0) m[p1][c] = acc;
                            else sq[p1][c] = acc;
                        }
                    }
                }
            } else {
                for (int j = 0; j < k; ++j)
#pragma unroll
                    for (int c = 0; c < PC; ++c) {
                        const float u = t[i2 * LX + c + j];
#pragma unroll
                        for (int p = 0; p < PR; ++p)
                            if (i2 - p >= 0 && i2 - p < k) tap(pass == 0 ? m[p][c] : sq[p][c], u, m[p][c]);
                    }
            }
        }
    }
    box_sums();
#pragma unroll
    for (int p = 0; p < PR; ++p) {
        const int64_t y = y0 + ly0 + p;
        if (y >= yend) break;
        // the thread's two columns as one 8- / 16-byte store where both lie in the image and the
        // addresses are aligned (W even and 256-byte aligned planes, as the library carves them): half
        // the store instructions, each lane's bytes contiguous
        const int64_t xp = x0 + lx0, op = y * g.W + xp;
        const bool al = (((uintptr_t)(st.sq + op) | (uintptr_t)(st.mean + op) | (uintptr_t)(st.sqt + op)) & 7) == 0 &&
                        ((uintptr_t)(st.box + op) & 15) == 0;
        if ((g.W & 1) == 0 && xp + 1 < g.W && al) {
            static_assert(PC == 2, "column pairs");
            if constexpr (MODE == STATS_FULL || MODE == STATS_MSB) *(f32x2*)(st.mean + op) = f32x2{m[p][0], m[p][1]};
            *(f32x2*)(st.sq + op) = f32x2{sq[p][0], sq[p][1]};
            *(f64x2*)(st.box + op) = f64x2{bx[p][0], bx[p][1]};
            if constexpr (MODE == STATS_FULL) {
                float t[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const double c2 = b2[p][c] - bx[p][c] * bx[p][c] / (double)(k * k);
                    t[c] = (float)(c2 > 0.0 ? c2 : 0.0);
                }
                *(f32x2*)(st.sqt + op) = f32x2{t[0], t[1]};
            }
            continue;
        }
#pragma unroll
        for (int c = 0; c < PC; ++c) {
            const int64_t x = x0 + lx0 + c;
            if (x >= g.W) break;
            const int64_t o = y * g.W + x;
            const double b = bx[p][c];
            if constexpr (MODE == STATS_FULL || MODE == STATS_MSB) stats_put(st.mean + o, m[p][c]);
            stats_put(st.sq + o, sq[p][c]);
            stats_put(st.box + o, b);
            if constexpr (MODE == STATS_FULL) {
                const double c2 = b2[p][c] - b * b / (double)(k * k);
                stats_put(st.sqt + o, (float)(c2 > 0.0 ? c2 : 0.0));
            }
        }
    }
}

// dynamic LDS bytes of one statistics tile (mode, k)
inline size_t stats_lds_bytes(int mode, int k) {
    const int LX = lx_for(k), LY = ty_for(mode) + k - 1;
    return sizeof(double) * (mode == STATS_FWD || mode == STATS_MSB ? 1 : 2) * LY * TX + sizeof(float) * LY * LX;
}
}  // namespace stats_detail
}  // namespace custma
