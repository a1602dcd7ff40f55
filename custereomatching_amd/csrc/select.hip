// Disparity selection.
//
//  * k_argmax: first-index argmax over the volume's last axis -- what the
//    reference's callers do with torch.max / torch.argmax on the returned
//    volume (examples/verify.py:72, examples/test.py:78-83).
//  * fused, certified disparity (no volume): the fast sweep writes per
//    disparity-chunk (best, second, index) partials; k_disp_merge combines
//    them and CERTIFIES a pixel when its top-2 gap exceeds twice the fast
//    path's error bound (then the fast argmax is provably the exact argmax);
//    every other pixel is queued and k_disp_recheck re-decides it with the
//    reference arithmetic (exact k*k fma chain, stereo_matching_kernel.cu:39-71).
//    The reported best cost is always recomputed exactly.  So the index map is
//    bit-identical to argmax of the exact volume.
#include <float.h>

#include <type_traits>

#include "common.h"
#include "sweep.h"

namespace custma {

namespace {

// torch.argmax semantics: NaN is the maximum, first index on ties.
// Start from (-inf, INT64_MAX) so the first element always wins.
__device__ __forceinline__ void amax_merge(float& bv, int64_t& bi, float ov, int64_t oi) {
    bool take;
    if (bv != bv) take = (ov != ov) && oi < bi;
    else if (ov != ov) take = true;
    else take = ov > bv || (ov == bv && oi < bi);
    if (take) { bv = ov; bi = oi; }
}

__global__ __launch_bounds__(256) void k_argmax(const float* __restrict__ vol, int64_t rows, int64_t n,
                                                int64_t* __restrict__ idx, float* __restrict__ best) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t row = wave; row < rows; row += nwaves) {
        float bv = -INFINITY;
        int64_t bi = INT64_MAX;
        if (n > 512) {
            // long rows (n < 2^29, checked at launch): 8 loads per lane in flight together through one raw
            // buffer (past the row's end an out-of-range offset, not merged): C2 full 1.65 -> 1.43 ms
            const auto r = make_rsrc(vol + row * n, (uint32_t)(n * 4));
            for (int64_t s0 = 0; s0 < n; s0 += 64 * 8) {
                float x[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int64_t s = s0 + lane + 64 * j;
                    x[j] = ld_bufs<float>(r, s < n ? (uint32_t)(s * 4) : 0x80000000u, 0u);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int64_t s = s0 + lane + 64 * j;
                    if (s < n) amax_merge(bv, bi, x[j], s);
                }
            }
        } else {  // short rows (window layouts): the batched form measured slower (C3 2.43 -> 2.50 ms)
            const float* v = vol + row * n;
            for (int64_t s = lane; s < n; s += 64) amax_merge(bv, bi, v[s], s);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float ov = __shfl_xor(bv, off);
            const int64_t oi = __shfl_xor(bi, off);
            amax_merge(bv, bi, ov, oi);
        }
        if (lane == 0) {
            idx[row] = bi;
            if (best) best[row] = bv;
        }
    }
}

// Exact reference cost of one voxel (stereo_matching_kernel.cu:39-71, nvcc
// -fmad=true), using the stats pass's bit-identical means and moments.
// KT > 0: compile-time window; patches fully inside the image take unguarded row loads.
template <typename T, int KT = 0>
__device__ float exact_cost(const T* cam, const T* proj, const Geo& g, const Stats& sc, const Stats& sp, int64_t h,
                            int64_t w, int64_t d) {
    const float mc = sc.mean[h * g.W + w], mp = sp.mean[h * g.W + d];
    float e = 0.f;
    const int k = KT > 0 ? KT : g.k, r = k / 2;
    if (KT > 0 && h >= r && h + r < g.H && w >= r && w + r < g.W && d >= r && d + r < g.W) {
        const T* cr = cam + (h - r) * g.W + (w - r);
        const T* pr = proj + (h - r) * g.W + (d - r);
#pragma unroll
        for (int i = 0; i < k; ++i) {
#pragma unroll
            for (int j = 0; j < k; ++j) {
                const float c = to_f(cr[j]) - mc;
                const float p = to_f(pr[j]) - mp;
                e = __builtin_fmaf(c, p, e);
            }
            cr += g.W;
            pr += g.W;
        }
    } else {
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j) {
                const float c = ldpad(cam, g.H, g.W, h + i - r, w + j - r) - mc;
                const float p = ldpad(proj, g.H, g.W, h + i - r, d + j - r) - mp;
                e = __builtin_fmaf(c, p, e);
            }
    }
    const float den = sqrtf(__builtin_fmaf(sc.sq[h * g.W + w], sp.sq[h * g.W + d], kEps));
    return (e + kEps) / den;
}

// exact_cost for any k with the patch loads batched: per patch row, 8 camera and 8 projector values
// through unconditional raw buffer loads (out-of-image offsets read 0, as ldpad) in flight together,
// then the same fma chain in the same order (the taps past k are loaded but not used).  A bounds-tested
// load per tap was waited for one at a time: 2 k^2 round trips per voxel in k_disp_recheck.
template <typename T>
__device__ float exact_cost_batched(const T* cam, const T* proj, const Geo& g, const Stats& sc, const Stats& sp,
                                    int64_t h, int64_t w, int64_t d) {
    const uint64_t nb = (uint64_t)g.H * (uint64_t)g.W * sizeof(T);
    if (nb >= 0x7FFFFFF0u) return exact_cost<T>(cam, proj, g, sc, sp, h, w, d);
    const auto rc = make_rsrc(cam, (uint32_t)nb), rp = make_rsrc(proj, (uint32_t)nb);
    const float mc = sc.mean[h * g.W + w], mp = sp.mean[h * g.W + d];
    float e = 0.f;
    const int k = g.k, r = k / 2;
    for (int i = 0; i < k; ++i) {
        const int64_t y = h + i - r;
        const bool yin = y >= 0 && y < g.H;
        for (int j0 = 0; j0 < k; j0 += 8) {
            float cv[8], pv[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const int64_t xc = w + j0 + jj - r, xp = d + j0 + jj - r;
                const bool cin = yin && xc >= 0 && xc < g.W, pin = yin && xp >= 0 && xp < g.W;
                cv[jj] = ld_bufs<T>(rc, cin ? (uint32_t)((y * g.W + xc) * (int64_t)sizeof(T)) : 0x80000000u, 0u);
                pv[jj] = ld_bufs<T>(rp, pin ? (uint32_t)((y * g.W + xp) * (int64_t)sizeof(T)) : 0x80000000u, 0u);
            }
#pragma unroll
            for (int jj = 0; jj < 8; ++jj)
                if (j0 + jj < k) e = __builtin_fmaf(cv[jj] - mc, pv[jj] - mp, e);
        }
    }
    const float den = sqrtf(__builtin_fmaf(sc.sq[h * g.W + w], sp.sq[h * g.W + d], kEps));
    return (e + kEps) / den;
}

__device__ __forceinline__ int64_t d_of_s(const Geo& g, int64_t w, int64_t s) {
    return g.layout == CUSTMA_LAYOUT_WINDOW ? w + s : s;
}

// Optional outputs of the fused disparity beyond (index, best): soft-argmax with beta
// (examples/verify.py:31-39) and the max-cost confidence mask (verify.py:72-74).
struct SoftOut {
    float* soft;  // [HV][WO] or null
    float* mask;  // [HV][WO] or null: 1 where best > threshold, else 0
    float kb;     // beta * log2(e)
    float threshold;
};

template <typename T, int KT>
__global__ __launch_bounds__(256) void k_disp_merge(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                    Stats sc, Stats sp, DispPartial part, int nChunk, float tau,
                                                    int64_t* __restrict__ idx, float* __restrict__ best,
                                                    int32_t* __restrict__ counter, int64_t* __restrict__ queue,
                                                    SoftOut so) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t npix = g.HV() * g.WO;
    if (p >= npix) return;
    float b = -FLT_MAX, sec = -FLT_MAX, q0 = 0.f, q1 = 0.f;
    int64_t bi = INT64_MAX;
    for (int c = 0; c < nChunk; ++c) {
        const int64_t q = (int64_t)c * npix + p;
        const int32_t oi = part.index[q];
        if (oi < 0) continue;
        const float ob = part.best[q], os = part.second[q];
        if (so.soft) soft_merge(b, ob, part.s0[q], part.s1[q], so.kb, q0, q1);
        if (ob > b || (ob == b && oi < bi)) {
            sec = fmaxf(os, b); b = ob; bi = oi;
        } else {
            sec = fmaxf(sec, ob);
        }
    }
    const int64_t h = g.h_lo + p / g.WO, w = p % g.WO;
    if (bi != INT64_MAX && (sec == -FLT_MAX || b - sec > tau)) {
        idx[p] = bi;
        const float eb = exact_cost<T, KT>(cam, proj, g, sc, sp, h, w, d_of_s(g, w, bi));
        if (best) best[p] = eb;
        if (so.mask) so.mask[p] = eb > so.threshold ? 1.f : 0.f;
        if (so.soft) so.soft[p] = q1 / q0;
    } else {
        const int32_t slot = atomicAdd(counter, 1);
        queue[slot] = p;
    }
}

// k_disp_merge for window layouts with a compile-time window: one workgroup per 4 x 64 pixel tile
// stages the camera tile and the projector strip its D + 1 diagonals reach (zero-padded, as float)
// in LDS, so a certified pixel's exact best cost reads its two k x k patches from LDS instead of
// 2 k^2 global loads (the projector patch at a per-pixel disparity).  Same fp32 operations in the
// same order as exact_cost (bit-identical).
// Tile rows (one wave each) x columns: 8 rows stage 18 / 8 projector-strip rows per pixel row at k = 11 where
// 4 rows staged 14 / 4 -- the staging is the kernel's cost: C5 merge 0.85 -> 0.66 ms, C3 disparity 1.200 ->
// 1.178 ms; 16 rows 0.78 ms (fewer resident workgroups), profiles/r06/q.  (Reading the patches as 8-byte pairs
// from two staggered LDS copies doubled the kernel's time: twice the LDS, a third of the workgroups per CU,
// profiles/r06/p.)
#ifndef CUSTMA_MTY
#define CUSTMA_MTY 8
#endif
constexpr int kMTY = CUSTMA_MTY, kMTX = 64;
template <typename T, int KT>
__global__ __launch_bounds__(64 * kMTY) void k_disp_merge_tile(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                         Stats sc, Stats sp, DispPartial part, int nChunk, float tau,
                                                         int64_t* __restrict__ idx, float* __restrict__ best,
                                                         int32_t* __restrict__ counter, int64_t* __restrict__ queue,
                                                         SoftOut so, int ntx) {
    constexpr int R = KT / 2, CY = kMTY + 2 * R, CX = kMTX + 2 * R;
    extern __shared__ float tl[];
    const int PX = kMTX + (int)g.D + 2 * R;  // projector strip width
    float* tc = tl;
    float* tp = tl + CY * CX;
    const int64_t x0 = (int64_t)(blockIdx.x % ntx) * kMTX, hy0 = g.h_lo + (int64_t)(blockIdx.x / ntx) * kMTY;
    tile_to_lds<T>(cam, g.H, g.W, hy0 - R, x0 - R, CY, CX, tc, CX, (int)threadIdx.x, 64 * kMTY);
    tile_to_lds<T>(proj, g.H, g.W, hy0 - R, x0 - R, CY, PX, tp, PX, (int)threadIdx.x, 64 * kMTY);
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int64_t h = hy0 + ty, w = x0 + tx;
    if (h >= g.h_hi || w >= g.WO) return;
    const int64_t npix = g.HV() * g.WO, p = (h - g.h_lo) * g.WO + w;
    float b = -FLT_MAX, sec = -FLT_MAX, q0 = 0.f, q1 = 0.f;
    int64_t bi = INT64_MAX;
    for (int c = 0; c < nChunk; ++c) {
        const int64_t q = (int64_t)c * npix + p;
        const int32_t oi = part.index[q];
        if (oi < 0) continue;
        const float ob = part.best[q], os = part.second[q];
        if (so.soft) soft_merge(b, ob, part.s0[q], part.s1[q], so.kb, q0, q1);
        if (ob > b || (ob == b && oi < bi)) {
            sec = fmaxf(os, b); b = ob; bi = oi;
        } else {
            sec = fmaxf(sec, ob);
        }
    }
    if (bi != INT64_MAX && (sec == -FLT_MAX || b - sec > tau)) {
        idx[p] = bi;
        const int64_t d = w + bi;  // window layout: d = w + s
        const float mc = sc.mean[h * g.W + w], mp = sp.mean[h * g.W + d];
        float e = 0.f;
        const float* cr = tc + ty * CX + tx;
        const float* pr = tp + ty * PX + tx + (int)bi;
#pragma unroll
        for (int i = 0; i < KT; ++i) {
#pragma unroll
            for (int j = 0; j < KT; ++j) e = __builtin_fmaf(cr[j] - mc, pr[j] - mp, e);
            cr += CX;
            pr += PX;
        }
        const float den = sqrtf(__builtin_fmaf(sc.sq[h * g.W + w], sp.sq[h * g.W + d], kEps));
        const float eb = (e + kEps) / den;
        if (best) best[p] = eb;
        if (so.mask) so.mask[p] = eb > so.threshold ? 1.f : 0.f;
        if (so.soft) so.soft[p] = q1 / q0;
    } else {
        const int32_t slot = atomicAdd(counter, 1);
        queue[slot] = p;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_disp_recheck(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                      Stats sc, Stats sp, const int32_t* __restrict__ counter,
                                                      const int64_t* __restrict__ queue, int64_t* __restrict__ idx,
                                                      float* __restrict__ best, SoftOut so) {
    __shared__ float rv[4], r0[4], r1[4];
    __shared__ int64_t ri[4];
    const int n = *counter;
    for (int64_t e = blockIdx.x; e < n; e += gridDim.x) {
        const int64_t p = queue[e];
        const int64_t h = g.h_lo + p / g.WO, w = p % g.WO;
        float bv = -INFINITY, q0 = 0.f, q1 = 0.f;
        int64_t bi = INT64_MAX;
        for (int64_t s = threadIdx.x; s < g.DO; s += blockDim.x) {
            const int64_t d = d_of_s(g, w, s);
            if (!voxel_valid(g, w, d)) continue;
            const float c = exact_cost_batched(cam, proj, g, sc, sp, h, w, d);
            if (so.soft) soft_add(c, (float)s, bv, so.kb, q0, q1);
            amax_merge(bv, bi, c, s);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float ov = __shfl_xor(bv, off);
            const int64_t oi = __shfl_xor(bi, off);
            if (so.soft) {
                const float o0 = __shfl_xor(q0, off), o1 = __shfl_xor(q1, off);
                soft_merge(bv, ov, o0, o1, so.kb, q0, q1);
            }
            amax_merge(bv, bi, ov, oi);
        }
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { rv[wave] = bv; ri[wave] = bi; r0[wave] = q0; r1[wave] = q1; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int q = 1; q < (int)(blockDim.x >> 6); ++q) {
                if (so.soft) soft_merge(bv, rv[q], r0[q], r1[q], so.kb, q0, q1);
                amax_merge(bv, bi, rv[q], ri[q]);
            }
            idx[p] = bi;
            if (best) best[p] = bv;
            if (so.mask) so.mask[p] = bv > so.threshold ? 1.f : 0.f;
            if (so.soft) so.soft[p] = q1 / q0;
        }
        __syncthreads();
    }
}

// k_disp_recheck with the queued pixel's k x k camera patch and its k x (DO + k - 1) projector strip staged in
// LDS once (zero-padded, as float: tile_to_lds), so each of its DO diagonals runs the exact_cost chain from LDS
// instead of 2 k^2 global loads (batched by 8 per patch row, each batch a round trip: the kernel was latency-
// bound, ~40-60 us for ~150 pixels).  Same fp32 operations in the same order as exact_cost (bit-identical).
template <typename T>
__global__ __launch_bounds__(256) void k_disp_recheck_lds(const T* __restrict__ cam, const T* __restrict__ proj, Geo g,
                                                          Stats sc, Stats sp, const int32_t* __restrict__ counter,
                                                          const int64_t* __restrict__ queue, int64_t* __restrict__ idx,
                                                          float* __restrict__ best, SoftOut so, int PX) {
    extern __shared__ float rl[];
    __shared__ float rv[4], r0[4], r1[4];
    __shared__ int64_t ri[4];
    const int k = g.k, r = k / 2;
    float* tc = rl;          // [k][k]
    float* tp = rl + k * k;  // [k][PX]: projector columns dmin - r .. dmin - r + PX - 1
    const int n = *counter;
    for (int64_t e = blockIdx.x; e < n; e += gridDim.x) {
        const int64_t p = queue[e];
        const int64_t h = g.h_lo + p / g.WO, w = p % g.WO;
        const int64_t dmin = d_of_s(g, w, 0);
        tile_to_lds<T>(cam, g.H, g.W, h - r, w - r, k, k, tc, k, (int)threadIdx.x, 256);
        tile_to_lds<T>(proj, g.H, g.W, h - r, dmin - r, k, PX, tp, PX, (int)threadIdx.x, 256);
        __syncthreads();
        const float mc = sc.mean[h * g.W + w], qc = sc.sq[h * g.W + w];
        float bv = -INFINITY, q0 = 0.f, q1 = 0.f;
        int64_t bi = INT64_MAX;
        for (int64_t s = threadIdx.x; s < g.DO; s += blockDim.x) {
            const int64_t d = d_of_s(g, w, s);
            if (!voxel_valid(g, w, d)) continue;
            const float mp = sp.mean[h * g.W + d];
            float acc = 0.f;
            for (int i = 0; i < k; ++i) {
                const float* cr = tc + i * k;
                const float* pr = tp + i * PX + (int)(d - dmin);
                for (int j = 0; j < k; ++j) acc = __builtin_fmaf(cr[j] - mc, pr[j] - mp, acc);
            }
            const float den = sqrtf(__builtin_fmaf(qc, sp.sq[h * g.W + d], kEps));
            const float c = (acc + kEps) / den;
            if (so.soft) soft_add(c, (float)s, bv, so.kb, q0, q1);
            amax_merge(bv, bi, c, s);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float ov = __shfl_xor(bv, off);
            const int64_t oi = __shfl_xor(bi, off);
            if (so.soft) {
                const float o0 = __shfl_xor(q0, off), o1 = __shfl_xor(q1, off);
                soft_merge(bv, ov, o0, o1, so.kb, q0, q1);
            }
            amax_merge(bv, bi, ov, oi);
        }
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { rv[wave] = bv; ri[wave] = bi; r0[wave] = q0; r1[wave] = q1; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int q = 1; q < (int)(blockDim.x >> 6); ++q) {
                if (so.soft) soft_merge(bv, rv[q], r0[q], r1[q], so.kb, q0, q1);
                amax_merge(bv, bi, rv[q], ri[q]);
            }
            idx[p] = bi;
            if (best) best[p] = bv;
            if (so.mask) so.mask[p] = bv > so.threshold ? 1.f : 0.f;
            if (so.soft) so.soft[p] = q1 / q0;
        }
        __syncthreads();  // (the next pixel's tiles overwrite this one's)
    }
}

}  // namespace

hipError_t launch_argmax(const float* vol, int64_t rows, int64_t n, int64_t* idx, float* best, hipStream_t s) {
    if (n >= ((int64_t)1 << 29)) return hipErrorInvalidValue;  // one row through one 32-bit buffer range
    const int64_t waves = rows < 2048 * 4 ? rows : 2048 * 4;
    const int64_t blocks = cdiv(waves, 4);
    hipLaunchKernelGGL(k_argmax, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(256), 0, s, vol, rows, n, idx, best);
    return hipGetLastError();
}

size_t disparity_partial_bytes(const Geo& g) {
    const SweepGrid sg = sweep_grid(g);
    const size_t n = (size_t)sg.nChunk * g.HV() * g.WO;
    return n * (4 + 4 + 4 + 4 + 4) + (size_t)g.HV() * g.WO * 8 + 256;
}

hipError_t launch_disparity(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            int64_t* idx, float* best, int32_t* n_rechecked, void* ws, hipStream_t s, float* soft,
                            float beta, float* mask, float threshold) {
    SoftOut so;
    so.soft = soft;
    so.mask = mask;
    so.kb = beta * 1.4426950408889634f;
    so.threshold = threshold;
    const SweepGrid sg = sweep_grid(g);
    const size_t n = (size_t)sg.nChunk * g.HV() * g.WO;
    char* p = (char*)ws;
    int32_t* counter = (int32_t*)p;  // 256 B header
    p += 256;
    int64_t* queue = (int64_t*)p;
    p += (size_t)g.HV() * g.WO * 8;
    DispPartial part;
    part.best = (float*)p;
    part.second = part.best + n;
    part.index = (int32_t*)(part.second + n);
    part.s0 = soft ? (float*)(part.index + n) : nullptr;
    part.s1 = soft ? part.s0 + n : nullptr;
    part.kb = so.kb;
    hipError_t e = hipMemsetAsync(counter, 0, 4, s);
    if (e != hipSuccess) return e;
    // kernel sizes without a sweep instantiation: every pixel is decided exactly
    // window layout with D + 1 <= 257: the tile kernel reduces all diagonals of a pixel in
    // one workgroup (one partial per pixel); otherwise per-chunk partials from k_sweep_fwd
    const bool tile = fast_supported(g.k) && disp_tile_ok(g);
    const int nChunk = !fast_supported(g.k) ? 0 : tile ? 1 : sg.nChunk;
    if (nChunk) {
        e = tile ? launch_disp_tile(cam, proj, dtype, g, sc, sp, part, s)
                 : launch_disp_partials(cam, proj, dtype, g, sc, sp, part, s);
        if (e != hipSuccess) return e;
    }
    // certification margin: 2 x twice the fast path's worst-case error
    const float tau = (float)(8.0 * (g.k * g.k + 6) * 5.9604644775390625e-08);
    const int64_t npix = g.HV() * g.WO;
    const unsigned mb = (unsigned)cdiv(npix, 256);
    // window layouts: the LDS-tiled merge while the projector strip fits
    const int ntx = (int)cdiv(g.WO, kMTX);
    const size_t mlds = sizeof(float) * (size_t)(kMTY + 2 * g.r) * (kMTX + 2 * g.r + (kMTX + g.D + 2 * g.r));
    const bool mtile = g.layout == CUSTMA_LAYOUT_WINDOW && mlds <= 64 * 1024;
    const unsigned mtb = (unsigned)(ntx * cdiv(g.HV(), kMTY));
    auto merge = [&](auto kc) {
        constexpr int KT = decltype(kc)::value;
        if constexpr (KT > 0) {
            if (mtile) {
                if (dtype == CUSTMA_F16)
                    hipLaunchKernelGGL((k_disp_merge_tile<__half, KT>), dim3(mtb), dim3(64 * kMTY), mlds, s,
                                       (const __half*)cam, (const __half*)proj, g, sc, sp, part, nChunk, tau, idx,
                                       best, counter, queue, so, ntx);
                else
                    hipLaunchKernelGGL((k_disp_merge_tile<float, KT>), dim3(mtb), dim3(64 * kMTY), mlds, s,
                                       (const float*)cam, (const float*)proj, g, sc, sp, part, nChunk, tau, idx,
                                       best, counter, queue, so, ntx);
                return;
            }
        }
        if (dtype == CUSTMA_F16)
            hipLaunchKernelGGL((k_disp_merge<__half, KT>), dim3(mb), dim3(256), 0, s, (const __half*)cam,
                               (const __half*)proj, g, sc, sp, part, nChunk, tau, idx, best, counter, queue, so);
        else
            hipLaunchKernelGGL((k_disp_merge<float, KT>), dim3(mb), dim3(256), 0, s, (const float*)cam,
                               (const float*)proj, g, sc, sp, part, nChunk, tau, idx, best, counter, queue, so);
    };
    switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: merge(std::integral_constant<int, KK>{}); break;
        CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
        default: merge(std::integral_constant<int, 0>{});
    }
    // the exact re-decision of the queued pixels: from LDS tiles while the projector strip fits 64 KiB
    const int PX = (int)g.DO + g.k - 1;
    const size_t rlds = sizeof(float) * (size_t)g.k * (size_t)(g.k + PX);
    if (rlds <= 65536) {
        if (dtype == CUSTMA_F16)
            hipLaunchKernelGGL(k_disp_recheck_lds<__half>, dim3(2048), dim3(256), rlds, s, (const __half*)cam,
                               (const __half*)proj, g, sc, sp, counter, queue, idx, best, so, PX);
        else
            hipLaunchKernelGGL(k_disp_recheck_lds<float>, dim3(2048), dim3(256), rlds, s, (const float*)cam,
                               (const float*)proj, g, sc, sp, counter, queue, idx, best, so, PX);
    } else if (dtype == CUSTMA_F16) {
        hipLaunchKernelGGL(k_disp_recheck<__half>, dim3(2048), dim3(256), 0, s, (const __half*)cam,
                           (const __half*)proj, g, sc, sp, counter, queue, idx, best, so);
    } else {
        hipLaunchKernelGGL(k_disp_recheck<float>, dim3(2048), dim3(256), 0, s, (const float*)cam,
                           (const float*)proj, g, sc, sp, counter, queue, idx, best, so);
    }
    e = hipGetLastError();
    if (e == hipSuccess && n_rechecked) e = hipMemcpyAsync(n_rechecked, counter, 4, hipMemcpyDeviceToDevice, s);
    return e;
}

}  // namespace custma
