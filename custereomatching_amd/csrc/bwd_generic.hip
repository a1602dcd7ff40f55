// Backward for every kernel size the fused sweep (bwd_fused.hip) has no
// instantiation for: even k (taps at offsets -k/2 .. k-1-k/2, the reference's
// `kernel_size / 2` origin, custma/src/stereo_matching_kernel.cu:103-105, 172-173)
// and odd k > 17.  Same decomposition as the fused path, every sum in fp64:
//
//   dC(y,x) = T1c(y,x) - sum_box [Am + c(y,x) B - mc B]
//   dP(y,o) = T1p(y,o) - sum_box [Ac + p(y,o) Bp - mp Bp]
//
//   A = g / S, V = A cost / S  (S = sqrt(X Y + eps); per voxel of the volume)
//   Am(h,w) = sum_d A mp(h,d)    B(h,w)  = sum_d V Y(h,d)      (volume-row sums)
//   Ac(h,d) = sum_w A mc(h,w)    Bp(h,d) = sum_w V X(h,w)      (volume-column sums)
//   BoxA(y,x,dl) = sum of A(h, w, w+dl) over volume rows h whose patch holds row y
//                  and camera columns w whose patch holds column x (fixed diagonal dl)
//   T1c(y,x) = sum_dl p(y,x+dl) BoxA(y,x,dl)     T1p(y,o) = sum_dl c(y,o-dl) BoxA(y,o-dl,dl)
//
// Reference: get_patches_grad_kernel (.cu:75-152) forms, per voxel and tap,
// g (y~/S - Y x~ (E+eps)/S^3) and patches_grad_to_image_kernel (.cu:155-179)
// scatters it with float atomics; summed over voxels that is the identity above
// (the centring Jacobian vanishes because centred patches sum to zero).
// Deterministic: fixed per-thread loops and fixed-shape wave reductions.
//
// Bounded for any image size: the volume-shaped fp64 passes (A, its vertical box VA and
// horizontal box BA) run over bands of output rows whose buffers fit kGenBandBytes (A of a
// band's rows plus its k - 1 halo rows is recomputed per band), every kernel is grid-stride
// (no grid past 2^32 work-items), and the per-pixel k x k box sums are separable (2k adds
// per pixel).  Workspace: 6 fp64 images + 3 fp64 images of row sums + the band buffers.
#include <stdlib.h>

#include "common.h"

namespace custma {

namespace {

constexpr int kGT = 256;                        // threads per block
constexpr unsigned kGridCap = 8192;             // grid-stride kernels: at most this many blocks
constexpr size_t kGenBandBytes = (size_t)2 << 30;  // A / VA / BA band buffers (at least one row)

struct GenArgs {
    const float* grad;  // [HV][WO][DO]
    const float* vol;   // forward output for the same images
    Stats sc, sp;
    double* A;          // [band rows + k - 1][WO][DO]: volume rows [ha, hb)
    double* VA;         // [band rows][WO][DO]   vertical box of A
    double* BA;         // [band rows][W][DO]    horizontal box of VA (camera column x, not w)
    double* Am;         // [H][W] (the volume rows; zero elsewhere)
    double* Bc;         // [H][W]
    double* Ac;         // [H][W]
    double* Bp;         // [H][W]
    double* T1c;        // [yhi - ylo][W]
    double* T1p;        // [yhi - ylo][W]
    double* hs;         // [3][H][W] horizontal k-sums of the box terms (one side at a time)
    int64_t ylo, yhi;   // image rows whose gradient can be nonzero
    int64_t y0, y1;     // this band's output rows
    int64_t ha, hb;     // volume rows held in A for this band
    int o, a;           // tap offsets: rows/cols [h - o, h + a] (o = k/2, a = k-1-o)
};

__device__ __forceinline__ int64_t gdo(const Geo& g, int64_t w, int64_t s) {
    return g.layout == CUSTMA_LAYOUT_WINDOW ? w + s : s;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ double gen_S(const Geo& g, const GenArgs& a, int64_t h, int64_t w, int64_t d) {
    const double X = (double)a.sc.sqt[h * g.W + w], Y = (double)a.sp.sqt[h * g.W + d];
    return sqrt(X * Y + (double)kEps);
}

// One wave per volume row (h, w), grid-stride: Am and B (sums over the row's diagonals).
__global__ __launch_bounds__(kGT) void k_gen_row(Geo g, GenArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (kGT / 64);
    const double rk2 = 1.0 / ((double)g.k * g.k);
    for (int64_t row = (int64_t)blockIdx.x * (kGT / 64) + (threadIdx.x >> 6); row < g.HV() * g.WO; row += nw) {
        const int64_t hv = row / g.WO, w = row % g.WO, h = g.h_lo + hv;
        const double X = (double)a.sc.sqt[h * g.W + w];
        double am = 0.0, b = 0.0;
        for (int64_t s = lane; s < g.DO; s += 64) {
            const int64_t d = gdo(g, w, s);
            if (d >= g.W) continue;
            const int64_t e = row * g.DO + s;
            const double Y = (double)a.sp.sqt[h * g.W + d];
            const double S = sqrt(X * Y + (double)kEps);
            const double A = (double)a.grad[e] / S;
            const double V = A * (double)a.vol[e] / S;
            am += A * (a.sp.box[h * g.W + d] * rk2);
            b += V * Y;
        }
        am = wave_sum(am);
        b = wave_sum(b);
        if (lane == 0) {
            a.Am[h * g.W + w] = am;
            a.Bc[h * g.W + w] = b;
        }
    }
}

// One thread per (volume row h, projector column d), grid-stride: Ac and Bp (sums over the
// camera columns of the voxels at projector column d).
__global__ __launch_bounds__(kGT) void k_gen_col(Geo g, GenArgs a) {
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    const double rk2 = 1.0 / ((double)g.k * g.k);
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < g.HV() * g.W; t += (int64_t)gridDim.x * kGT) {
        const int64_t hv = t / g.W, d = t % g.W, h = g.h_lo + hv;
        const double Y = (double)a.sp.sqt[h * g.W + d];
        int64_t wlo = 0, whi = g.WO;  // camera columns with a voxel at projector column d
        if (window) {
            wlo = d - g.D > 0 ? d - g.D : 0;
            whi = d + 1 < g.WO ? d + 1 : g.WO;
        }
        double ac = 0.0, bp = 0.0;
        for (int64_t w = wlo; w < whi; ++w) {
            const int64_t e = (hv * g.WO + w) * g.DO + (window ? d - w : d);
            const double X = (double)a.sc.sqt[h * g.W + w];
            const double S = sqrt(X * Y + (double)kEps);
            const double A = (double)a.grad[e] / S;
            ac += A * (a.sc.box[h * g.W + w] * rk2);
            bp += A * (double)a.vol[e] / S * X;
        }
        a.Ac[h * g.W + d] = ac;
        a.Bp[h * g.W + d] = bp;
    }
}

// A of the volume rows [ha, hb) (this band's rows and their halo), grid-stride.
__global__ __launch_bounds__(kGT) void k_gen_a(Geo g, GenArgs a) {
    const int64_t slab = g.WO * g.DO, n = (a.hb - a.ha) * slab;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < n; t += (int64_t)gridDim.x * kGT) {
        const int64_t h = a.ha + t / slab, e = t % slab, w = e / g.DO, s = e % g.DO, d = gdo(g, w, s);
        double A = 0.0;
        if (d < g.W) A = (double)a.grad[(h - g.h_lo) * slab + e] / gen_S(g, a, h, w, d);
        a.A[t] = A;
    }
}

// VA(y, w, s) = sum of A(h, w, s) over the volume rows h in [y - a, y + o], y in the band.
__global__ __launch_bounds__(kGT) void k_gen_vbox(Geo g, GenArgs a) {
    const int64_t slab = g.WO * g.DO, n = (a.y1 - a.y0) * slab;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < n; t += (int64_t)gridDim.x * kGT) {
        const int64_t y = a.y0 + t / slab, e = t % slab;
        int64_t h0 = y - a.a, h1 = y + a.o;
        h0 = h0 > a.ha ? h0 : a.ha;
        h1 = h1 < a.hb - 1 ? h1 : a.hb - 1;
        double v = 0.0;
        for (int64_t h = h0; h <= h1; ++h) v += a.A[(h - a.ha) * slab + e];
        a.VA[t] = v;
    }
}

// BA(y, x, s) = sum of VA(y, w, s_w) over camera columns w in [x - a, x + o] on the same diagonal
// (window: s_w = s; full: projector column d_w = s + w - x).
__global__ __launch_bounds__(kGT) void k_gen_hbox(Geo g, GenArgs a) {
    const int64_t slab = g.W * g.DO, n = (a.y1 - a.y0) * slab;
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < n; t += (int64_t)gridDim.x * kGT) {
        const int64_t yy = t / slab, e = t % slab, x = e / g.DO, s = e % g.DO;
        int64_t w0 = x - a.a, w1 = x + a.o;
        w0 = w0 > 0 ? w0 : 0;
        w1 = w1 < g.WO - 1 ? w1 : g.WO - 1;
        double v = 0.0;
        const double* va = a.VA + yy * g.WO * g.DO;
        for (int64_t w = w0; w <= w1; ++w) {
            const int64_t sw = window ? s : s + (w - x);
            if (sw >= 0 && sw < g.DO) v += va[w * g.DO + sw];
        }
        a.BA[t] = v;
    }
}

// One wave per pixel (y, x) of the band, grid-stride: T1c = sum_s p(y, d(x, s)) BA(y, x, s).
template <typename T>
__global__ __launch_bounds__(kGT) void k_gen_t1c(Geo g, GenArgs a, const T* __restrict__ proj) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (kGT / 64), np = (a.y1 - a.y0) * g.W;
    for (int64_t p = (int64_t)blockIdx.x * (kGT / 64) + (threadIdx.x >> 6); p < np; p += nw) {
        const int64_t yy = p / g.W, x = p % g.W, y = a.y0 + yy;
        const double* ba = a.BA + p * g.DO;
        double v = 0.0;
        for (int64_t s = lane; s < g.DO; s += 64) {
            const int64_t d = gdo(g, x, s);
            if (d < g.W) v += (double)to_f(proj[y * g.W + d]) * ba[s];
        }
        v = wave_sum(v);
        if (lane == 0) a.T1c[(y - a.ylo) * g.W + x] = v;
    }
}

// One thread per pixel (y, o) of the band, grid-stride: T1p = sum_x c(y, x) BA(y, x, s) at
// projector column o.
template <typename T>
__global__ __launch_bounds__(kGT) void k_gen_t1p(Geo g, GenArgs a, const T* __restrict__ cam) {
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    const int64_t np = (a.y1 - a.y0) * g.W;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < np; t += (int64_t)gridDim.x * kGT) {
        const int64_t yy = t / g.W, o = t % g.W, y = a.y0 + yy;
        int64_t x0 = 0, x1 = g.W;
        if (window) {
            x0 = o - g.D > 0 ? o - g.D : 0;
            x1 = o + 1;
        }
        double v = 0.0;
        for (int64_t x = x0; x < x1; ++x)
            v += (double)to_f(cam[y * g.W + x]) * a.BA[(yy * g.W + x) * g.DO + (window ? o - x : o)];
        a.T1p[(y - a.ylo) * g.W + o] = v;
    }
}

// Horizontal k-sums (columns [x - a, x + o], clipped) of one side's three box terms:
// hs[0] = row sums of Am|Ac, hs[1] of B|Bp, hs[2] of m B|m Bp (m = the patch mean).
__global__ __launch_bounds__(kGT) void k_gen_hsum(Geo g, GenArgs a, int side) {
    const double rk2 = 1.0 / ((double)g.k * g.k);
    const double* R = side == 0 ? a.Am : a.Ac;
    const double* B = side == 0 ? a.Bc : a.Bp;
    const double* box = side == 0 ? a.sc.box : a.sp.box;
    const int64_t n = g.H * g.W;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < n; t += (int64_t)gridDim.x * kGT) {
        const int64_t y = t / g.W, x = t % g.W;
        const int64_t w0 = x - a.a > 0 ? x - a.a : 0, w1 = x + a.o < g.W - 1 ? x + a.o : g.W - 1;
        double sr = 0.0, sb = 0.0, sm = 0.0;
        for (int64_t w = w0; w <= w1; ++w) {
            const int64_t q = y * g.W + w;
            sr += R[q];
            sb += B[q];
            sm += box[q] * rk2 * B[q];
        }
        a.hs[t] = sr;
        a.hs[n + t] = sb;
        a.hs[2 * n + t] = sm;
    }
}

// Vertical k-sums of the row sums and the gradient of one side (zero outside [ylo, yhi)).
template <typename T>
__global__ __launch_bounds__(kGT) void k_gen_combine(Geo g, GenArgs a, const T* __restrict__ img, int side,
                                                     float* __restrict__ out) {
    const int64_t n = g.H * g.W;
    const double* T1 = side == 0 ? a.T1c : a.T1p;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < n; t += (int64_t)gridDim.x * kGT) {
        const int64_t y = t / g.W, x = t % g.W;
        if (y < a.ylo || y >= a.yhi) {
            out[t] = 0.f;
            continue;
        }
        const int64_t h0 = y - a.a > 0 ? y - a.a : 0, h1 = y + a.o < g.H - 1 ? y + a.o : g.H - 1;
        double sr = 0.0, sb = 0.0, sm = 0.0;
        for (int64_t h = h0; h <= h1; ++h) {
            const int64_t q = h * g.W + x;
            sr += a.hs[q];
            sb += a.hs[n + q];
            sm += a.hs[2 * n + q];
        }
        out[t] = (float)(T1[(y - a.ylo) * g.W + x] - sr - (double)to_f(img[t]) * sb + sm);
    }
}

struct GenPlan {
    int64_t ylo, yhi, band;      // output rows with a gradient; output rows per band
    size_t A, VA, BA, img, t1;   // bytes of each buffer
};

GenPlan plan_gen(const Geo& g) {
    GenPlan p;
    const int o = g.k / 2, a = g.k - 1 - o;
    p.ylo = g.h_lo - o > 0 ? g.h_lo - o : 0;
    p.yhi = g.h_hi + a < g.H ? g.h_hi + a : g.H;
    const int64_t ny = p.yhi - p.ylo;
    const size_t vrow = (size_t)g.WO * g.DO * 8, brow = (size_t)g.W * g.DO * 8;
    // rows per band: A holds band + k - 1 rows, VA and BA band rows each
    const size_t fixed = (size_t)(g.k - 1) * vrow, per = 2 * vrow + brow;
    int64_t band = kGenBandBytes > fixed + per ? (int64_t)((kGenBandBytes - fixed) / per) : 1;
    if (const char* e = getenv("CUSTMA_GEN_BAND_ROWS")) {  // testing: force small bands
        const int64_t v = atoll(e);
        if (v > 0) band = v;
    }
    band = band < ny ? band : ny;
    p.band = band > 0 ? band : 1;
    p.A = (size_t)(p.band + g.k - 1) * vrow;
    p.VA = (size_t)p.band * vrow;
    p.BA = (size_t)p.band * brow;
    p.img = (size_t)g.H * g.W * 8;
    p.t1 = (size_t)(ny > 0 ? ny : 0) * g.W * 8;
    return p;
}

inline size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

unsigned grid_for(int64_t n, int per_block = kGT) {
    const int64_t b = cdiv(n, per_block);
    return (unsigned)(b < (int64_t)kGridCap ? (b > 0 ? b : 1) : kGridCap);
}

template <typename T>
hipError_t run_gen(const float* grad, const float* vol, const T* cam, const T* proj, const Geo& g, Stats sc,
                   Stats sp, float* dcam, float* dproj, void* ws, hipStream_t s) {
    const GenPlan p = plan_gen(g);
    GenArgs a;
    a.grad = grad; a.vol = vol; a.sc = sc; a.sp = sp;
    a.ylo = p.ylo; a.yhi = p.yhi;
    a.o = g.k / 2; a.a = g.k - 1 - a.o;
    char* w = (char*)ws;
    a.A = (double*)w; w += al(p.A);
    a.VA = (double*)w; w += al(p.VA);
    a.BA = (double*)w; w += al(p.BA);
    double* imgs = (double*)w;
    a.Am = (double*)w; w += al(p.img);
    a.Bc = (double*)w; w += al(p.img);
    a.Ac = (double*)w; w += al(p.img);
    a.Bp = (double*)w; w += al(p.img);
    a.T1c = (double*)w; w += al(p.t1);
    a.T1p = (double*)w; w += al(p.t1);
    a.hs = (double*)w;
    // rows outside the volume band hold no row / column terms
    hipError_t e = hipMemsetAsync(imgs, 0, 4 * al(p.img), s);
    if (e != hipSuccess) return e;
    prof_begin(PROF_BWD, s);
    hipLaunchKernelGGL(k_gen_row, dim3(grid_for(g.HV() * g.WO, kGT / 64)), dim3(kGT), 0, s, g, a);
    hipLaunchKernelGGL(k_gen_col, dim3(grid_for(g.HV() * g.W)), dim3(kGT), 0, s, g, a);
    for (int64_t y0 = p.ylo; y0 < p.yhi; y0 += p.band) {
        a.y0 = y0;
        a.y1 = y0 + p.band < p.yhi ? y0 + p.band : p.yhi;
        a.ha = a.y0 - a.a > g.h_lo ? a.y0 - a.a : g.h_lo;
        a.hb = a.y1 + a.o < g.h_hi ? a.y1 + a.o : g.h_hi;  // rows [y1 - 1 - a, y1 - 1 + o] end at y1 - 1 + o
        if (a.hb < a.ha) a.hb = a.ha;
        hipLaunchKernelGGL(k_gen_a, dim3(grid_for((a.hb - a.ha) * g.WO * g.DO)), dim3(kGT), 0, s, g, a);
        hipLaunchKernelGGL(k_gen_vbox, dim3(grid_for((a.y1 - a.y0) * g.WO * g.DO)), dim3(kGT), 0, s, g, a);
        hipLaunchKernelGGL(k_gen_hbox, dim3(grid_for((a.y1 - a.y0) * g.W * g.DO)), dim3(kGT), 0, s, g, a);
        hipLaunchKernelGGL((k_gen_t1c<T>), dim3(grid_for((a.y1 - a.y0) * g.W, kGT / 64)), dim3(kGT), 0, s, g, a,
                           proj);
        hipLaunchKernelGGL((k_gen_t1p<T>), dim3(grid_for((a.y1 - a.y0) * g.W)), dim3(kGT), 0, s, g, a, cam);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    prof_end(PROF_BWD, s);
    for (int side = 0; side < 2; ++side) {
        float* out = side == 0 ? dcam : dproj;
        if (!out) continue;
        hipLaunchKernelGGL(k_gen_hsum, dim3(grid_for(g.H * g.W)), dim3(kGT), 0, s, g, a, side);
        hipLaunchKernelGGL((k_gen_combine<T>), dim3(grid_for(g.H * g.W)), dim3(kGT), 0, s, g, a,
                           side == 0 ? cam : proj, side, out);
    }
    return hipGetLastError();
}

}  // namespace

size_t backward_generic_workspace_bytes(const Geo& g) {
    const GenPlan p = plan_gen(g);
    return al(p.A) + al(p.VA) + al(p.BA) + 4 * al(p.img) + 2 * al(p.t1) + 3 * al(p.img);
}

hipError_t launch_backward_generic(const float* grad, const float* vol, const void* cam, const void* proj,
                                   int dtype, const Geo& g, Stats sc, Stats sp, float* dcam, float* dproj,
                                   void* ws, hipStream_t s) {
    if (dtype == CUSTMA_F16)
        return run_gen(grad, vol, (const __half*)cam, (const __half*)proj, g, sc, sp, dcam, dproj, ws, s);
    return run_gen(grad, vol, (const float*)cam, (const float*)proj, g, sc, sp, dcam, dproj, ws, s);
}

}  // namespace custma
