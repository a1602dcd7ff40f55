// Backward for every kernel size the fused sweep (bwd_fused.hip) has no
// instantiation for: even k (taps at offsets -k/2 .. k-1-k/2, the reference's
// `kernel_size / 2` origin, custma/src/stereo_matching_kernel.cu:103-105, 172-173)
// and odd k > 15.  Same decomposition as the fused path, every sum in fp64 and
// every pass a plain streaming kernel over volume-shaped fp64 workspace:
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
// Deterministic: fixed per-thread loops and fixed-shape block reductions.
// Cost: O(k) per voxel for the two box passes (separable), O(k^2) per pixel
// for the final combination; workspace ~ 3 x 8 bytes per voxel.
#include "common.h"

namespace custma {

namespace {

constexpr int kGT = 256;  // threads per block

struct GenArgs {
    const float* grad;  // [HV][WO][DO]
    const float* vol;   // forward output for the same images
    Stats sc, sp;
    double* A;          // [HV][WO][DO]
    double* VA;         // [NYB][WO][DO]   vertical box of A
    double* BA;         // [NYB][W][DO]    horizontal box of VA (camera column x, not w)
    double* Am;         // [H][W] (the volume rows; zero elsewhere)
    double* Bc;         // [H][W]
    double* Ac;         // [H][W]
    double* Bp;         // [H][W]
    double* T1c;        // [NYB][W]
    double* T1p;        // [NYB][W]
    int64_t ylo, yhi;   // image rows whose gradient can be nonzero
    int o, a;           // tap offsets: rows/cols [h - o, h + a] (o = k/2, a = k-1-o)
};

__device__ __forceinline__ int64_t gdo(const Geo& g, int64_t w, int64_t s) {
    return g.layout == CUSTMA_LAYOUT_WINDOW ? w + s : s;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int off = kGT / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

// One block per volume row (h, w): A for every voxel of the row, Am and B.
__global__ __launch_bounds__(kGT) void k_gen_row(Geo g, GenArgs a) {
    __shared__ double red[kGT];
    const int64_t row = blockIdx.x;  // (h - h_lo) * WO + w
    const int64_t hv = row / g.WO, w = row % g.WO, h = g.h_lo + hv;
    const double rk2 = 1.0 / ((double)g.k * g.k);
    const double X = (double)a.sc.sqt[h * g.W + w];
    double am = 0.0, b = 0.0;
    for (int64_t s = threadIdx.x; s < g.DO; s += kGT) {
        const int64_t d = gdo(g, w, s);
        const int64_t e = row * g.DO + s;
        const double Y = (double)a.sp.sqt[h * g.W + d];
        const double S = sqrt(X * Y + (double)kEps);
        const double A = (double)a.grad[e] / S;
        const double V = A * (double)a.vol[e] / S;
        a.A[e] = A;
        am += A * (a.sp.box[h * g.W + d] * rk2);
        b += V * Y;
    }
    am = block_sum(am, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        a.Am[h * g.W + w] = am;
        a.Bc[h * g.W + w] = b;
    }
}

// One thread per (volume row h, projector column d): Ac and Bp (sums over the camera columns).
__global__ __launch_bounds__(kGT) void k_gen_col(Geo g, GenArgs a) {
    const int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x;
    if (t >= g.HV() * g.W) return;
    const int64_t hv = t / g.W, d = t % g.W, h = g.h_lo + hv;
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    const double rk2 = 1.0 / ((double)g.k * g.k);
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
        const double A = a.A[e];
        ac += A * (a.sc.box[h * g.W + w] * rk2);
        bp += A * (double)a.vol[e] / S * X;
    }
    a.Ac[h * g.W + d] = ac;
    a.Bp[h * g.W + d] = bp;
}

// VA(y, w, s) = sum of A(h, w, s) over the volume rows h in [y - a, y + o].
__global__ __launch_bounds__(kGT) void k_gen_vbox(Geo g, GenArgs a) {
    const int64_t slab = g.WO * g.DO, n = (a.yhi - a.ylo) * slab;
    for (int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x; t < n; t += (int64_t)gridDim.x * kGT) {
        const int64_t y = a.ylo + t / slab, e = t % slab;
        int64_t h0 = y - a.a, h1 = y + a.o;
        h0 = h0 > g.h_lo ? h0 : g.h_lo;
        h1 = h1 < g.h_hi - 1 ? h1 : g.h_hi - 1;
        double v = 0.0;
        for (int64_t h = h0; h <= h1; ++h) v += a.A[(h - g.h_lo) * slab + e];
        a.VA[t] = v;
    }
}

// BA(y, x, s) = sum of VA(y, w, s_w) over camera columns w in [x - a, x + o] on the same diagonal
// (window: s_w = s; full: projector column d_w = s + w - x).
__global__ __launch_bounds__(kGT) void k_gen_hbox(Geo g, GenArgs a) {
    const int64_t slab = g.W * g.DO, n = (a.yhi - a.ylo) * slab;
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

// One block per pixel (y, x): T1c = sum_s p(y, d(x, s)) BA(y, x, s).
template <typename T>
__global__ __launch_bounds__(kGT) void k_gen_t1c(Geo g, GenArgs a, const T* __restrict__ proj) {
    __shared__ double red[kGT];
    const int64_t p = blockIdx.x, yy = p / g.W, x = p % g.W, y = a.ylo + yy;
    const double* ba = a.BA + p * g.DO;
    double v = 0.0;
    for (int64_t s = threadIdx.x; s < g.DO; s += kGT) {
        const int64_t d = gdo(g, x, s);
        if (d < g.W) v += (double)to_f(proj[y * g.W + d]) * ba[s];
    }
    v = block_sum(v, red);
    if (threadIdx.x == 0) a.T1c[p] = v;
}

// One thread per pixel (y, o): T1p = sum_x c(y, x) BA(y, x, s) at projector column o.
template <typename T>
__global__ __launch_bounds__(kGT) void k_gen_t1p(Geo g, GenArgs a, const T* __restrict__ cam) {
    const int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x;
    if (t >= (a.yhi - a.ylo) * g.W) return;
    const int64_t yy = t / g.W, o = t % g.W, y = a.ylo + yy;
    const bool window = g.layout == CUSTMA_LAYOUT_WINDOW;
    int64_t x0 = 0, x1 = g.W;
    if (window) {
        x0 = o - g.D > 0 ? o - g.D : 0;
        x1 = o + 1;
    }
    double v = 0.0;
    for (int64_t x = x0; x < x1; ++x)
        v += (double)to_f(cam[y * g.W + x]) * a.BA[(yy * g.W + x) * g.DO + (window ? o - x : o)];
    a.T1p[t] = v;
}

// Per pixel: the box sums of the row / column terms, and the gradient (zero outside [ylo, yhi)).
template <typename T>
__global__ __launch_bounds__(kGT) void k_gen_combine(Geo g, GenArgs a, const T* __restrict__ cam,
                                                     const T* __restrict__ proj, float* __restrict__ dcam,
                                                     float* __restrict__ dproj) {
    const int64_t t = (int64_t)blockIdx.x * kGT + threadIdx.x;
    if (t >= g.H * g.W) return;
    const int64_t y = t / g.W, x = t % g.W;
    const double rk2 = 1.0 / ((double)g.k * g.k);
    if (y < a.ylo || y >= a.yhi) {
        if (dcam) dcam[t] = 0.f;
        if (dproj) dproj[t] = 0.f;
        return;
    }
    const int64_t h0 = y - a.a > 0 ? y - a.a : 0, h1 = y + a.o < g.H - 1 ? y + a.o : g.H - 1;
    const int64_t w0 = x - a.a > 0 ? x - a.a : 0, w1 = x + a.o < g.W - 1 ? x + a.o : g.W - 1;
    double sa = 0.0, sb = 0.0, sm = 0.0, pa = 0.0, pbb = 0.0, pm = 0.0;
    for (int64_t h = h0; h <= h1; ++h)
        for (int64_t w = w0; w <= w1; ++w) {
            const int64_t q = h * g.W + w;
            sa += a.Am[q];
            sb += a.Bc[q];
            sm += a.sc.box[q] * rk2 * a.Bc[q];
            pa += a.Ac[q];
            pbb += a.Bp[q];
            pm += a.sp.box[q] * rk2 * a.Bp[q];
        }
    const int64_t u = (y - a.ylo) * g.W + x;
    if (dcam) dcam[t] = (float)(a.T1c[u] - sa - (double)to_f(cam[t]) * sb + sm);
    if (dproj) dproj[t] = (float)(a.T1p[u] - pa - (double)to_f(proj[t]) * pbb + pm);
}

struct GenPlan {
    int64_t ylo, yhi;
    size_t A, VA, BA, img, t1;
};

GenPlan plan_gen(const Geo& g) {
    GenPlan p;
    const int o = g.k / 2, a = g.k - 1 - o;
    p.ylo = g.h_lo - o > 0 ? g.h_lo - o : 0;
    p.yhi = g.h_hi + a < g.H ? g.h_hi + a : g.H;
    const size_t ny = (size_t)(p.yhi - p.ylo);
    p.A = (size_t)g.HV() * g.WO * g.DO * 8;
    p.VA = ny * g.WO * g.DO * 8;
    p.BA = ny * g.W * g.DO * 8;
    p.img = (size_t)g.H * g.W * 8;
    p.t1 = ny * g.W * 8;
    return p;
}

inline size_t al(size_t n) { return (n + 255) & ~(size_t)255; }

unsigned grid_for(int64_t n) {
    const int64_t b = cdiv(n, kGT);
    return (unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536);
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
    a.T1p = (double*)w;
    // rows outside the volume band hold no row / column terms
    hipError_t e = hipMemsetAsync(imgs, 0, (size_t)((char*)a.T1c - (char*)imgs), s);
    if (e != hipSuccess) return e;
    prof_begin(PROF_BWD, s);
    hipLaunchKernelGGL(k_gen_row, dim3((unsigned)(g.HV() * g.WO)), dim3(kGT), 0, s, g, a);
    hipLaunchKernelGGL(k_gen_col, dim3((unsigned)cdiv(g.HV() * g.W, kGT)), dim3(kGT), 0, s, g, a);
    hipLaunchKernelGGL(k_gen_vbox, dim3(grid_for((p.yhi - p.ylo) * g.WO * g.DO)), dim3(kGT), 0, s, g, a);
    hipLaunchKernelGGL(k_gen_hbox, dim3(grid_for((p.yhi - p.ylo) * g.W * g.DO)), dim3(kGT), 0, s, g, a);
    hipLaunchKernelGGL((k_gen_t1c<T>), dim3((unsigned)((p.yhi - p.ylo) * g.W)), dim3(kGT), 0, s, g, a, proj);
    hipLaunchKernelGGL((k_gen_t1p<T>), dim3((unsigned)cdiv((p.yhi - p.ylo) * g.W, kGT)), dim3(kGT), 0, s, g, a,
                       cam);
    prof_end(PROF_BWD, s);
    hipLaunchKernelGGL((k_gen_combine<T>), dim3((unsigned)cdiv(g.H * g.W, kGT)), dim3(kGT), 0, s, g, a, cam, proj,
                       dcam, dproj);
    return hipGetLastError();
}

}  // namespace

size_t backward_generic_workspace_bytes(const Geo& g) {
    const GenPlan p = plan_gen(g);
    return al(p.A) + al(p.VA) + al(p.BA) + 4 * al(p.img) + 2 * al(p.t1);
}

hipError_t launch_backward_generic(const float* grad, const float* vol, const void* cam, const void* proj,
                                   int dtype, const Geo& g, Stats sc, Stats sp, float* dcam, float* dproj,
                                   void* ws, hipStream_t s) {
    if (dtype == CUSTMA_F16)
        return run_gen(grad, vol, (const __half*)cam, (const __half*)proj, g, sc, sp, dcam, dproj, ws, s);
    return run_gen(grad, vol, (const float*)cam, (const float*)proj, g, sc, sp, dcam, dproj, ws, s);
}

}  // namespace custma
