// Backward: deterministic, atomic-free gradients w.r.t. both images.
//
// The reference (custma/src/stereo_matching_kernel.cu:97-179) forms, per
// voxel and tap t, the patch gradient  g * (y_t / S - Y x_t (E+eps) / S^3)
// (S = sqrt(X Y + eps); the centring Jacobian vanishes because centred
// patches sum to zero) and scatters it with float atomics.  Summed over all
// voxels, with A = g/S and V = g (E+eps)/S^3 (zero outside valid voxels),
// the camera gradient at pixel (y, x) is exactly
//
//   dC(y,x) =  sum_delta p(y, x+delta) * BoxA(y, x, delta)       (T1)
//            - Box[ Am ](y,x)          Am(h,w) = sum_delta A * mean_p(h, w+delta)
//            - c(y,x) * Box[ B ](y,x)  B(h,w)  = sum_delta V * Y(h, w+delta)
//            + Box[ mean_c * B ](y,x)
//
// where BoxA(y,x,delta) and Box[F] are k x k box sums over patch centres
// (h, w) around (y, x).  BoxA slides exactly like the forward's product sums,
// so the backward is O(1) per voxel instead of the reference's O(k^2) plus
// k^2 atomics per voxel.  The projector gradient is the same pass with the
// roles of the images swapped (other = camera, delta -> -delta) over a
// transposed copy of the gradient so that its reads stay coalesced.
//
// One "role" pass: lanes own diagonals delta (as in the forward sweep), a
// workgroup owns TW own-image columns and walks a band of rows keeping two
// fp64 register arrays: colE (vertical sums of image products, for E) and
// colA (vertical sums of A, for BoxA).  A for the row leaving colA is
// recomputed from g (re-read, cache-resident) rather than stored.  Per-pixel
// sums over a workgroup's diagonals are reduced through LDS and written as
// fp64 partials per disparity chunk; k_bwd_reduce / k_bwd_combine finish.
#include "common.h"
#include "sweep.h"

namespace custma {

namespace {

struct Role {
    const void* own;
    const void* oth;
    Stats so, st;               // own / other image stats
    const float* g;             // gradient volume (own-major addressing below)
    int64_t gsH, gsU, gsD, gOff;
    int64_t ownMax, othMax;     // voxel exists iff u < ownMax and u+delta < othMax
    int64_t dWinLo, dWinHi;     // window layout delta range (full: unbounded)
    int window;
    double* Bp;                 // [nChunk][H][W]
    double* Amp;                // [nChunk][H][W]
    double* T1p;                // [nChunk][H][W]
};

template <int K, typename T>
__global__ __launch_bounds__(320) void k_sweep_bwd(Geo g, Role ro, SweepGrid sg) {
    constexpr int R = K / 2, NX = TW + 2 * R;
    const int NL = sg.NL, NO = NX + NL - 1, NS = TW + NL - 1;
    const T* __restrict__ own = (const T*)ro.own;
    const T* __restrict__ oth = (const T*)ro.oth;
    extern __shared__ __attribute__((aligned(16))) double ldsd[];
    double* red = ldsd;                      // [TW][NL] reduction tile
    double* mO = red + TW * NL;              // [NS]  other-image fp64 mean, row h
    double* bU = mO + NS;                    // [TW]  own-image fp64 box sum, row h
    float* ringU = (float*)(bU + TW);        // [K][NX] own image rows
    float* ringO = ringU + K * NX;           // [K][NO] other image rows
    float* qU = ringO + K * NO;              // [K][NX] own sqt rows (A ring)
    float* qO = qU + K * NX;                 // [K][NO] other sqt rows (A ring)

    int64_t bid = blockIdx.x;
    const int chunk = (int)(bid % sg.nChunk);
    bid /= sg.nChunk;
    const int wt = (int)(bid % sg.nTile);
    const int band = (int)(bid / sg.nTile);
    const int64_t u0 = (int64_t)wt * TW;
    const int64_t h0 = (int64_t)band * sg.TH, h1 = min(g.H, h0 + sg.TH);
    const int64_t dlo = ro.window ? ro.dWinLo : -(u0 + TW - 1);
    const int64_t d0 = dlo + (int64_t)chunk * NL;
    const int tid = threadIdx.x;
    const int64_t delta = d0 + tid;
    const double rk2 = 1.0 / (double)(K * K);
    const int64_t xbase = u0 - R;                // own column of x-slot 0
    const int64_t obase = u0 - R + d0;           // other column of ring slot 0

    auto slot_of = [](int64_t y) { return (int)(((y % K) + K) % K); };
    auto stage_img = [&](int64_t y) {
        const int s = slot_of(y);
        for (int x = tid; x < NX; x += NL) ringU[s * NX + x] = ldpad(own, g.H, g.W, y, xbase + x);
        for (int x = tid; x < NO; x += NL) ringO[s * NO + x] = ldpad(oth, g.H, g.W, y, obase + x);
    };
    auto stage_q = [&](int64_t y) {
        const int s = slot_of(y);
        const bool yok = y >= 0 && y < g.H;
        for (int x = tid; x < NX; x += NL) {
            const int64_t c = xbase + x;
            qU[s * NX + x] = (yok && c >= 0 && c < g.W) ? ro.so.sqt[y * g.W + c] : 0.f;
        }
        for (int x = tid; x < NO; x += NL) {
            const int64_t c = obase + x;
            qO[s * NO + x] = (yok && c >= 0 && c < g.W) ? ro.st.sqt[y * g.W + c] : 0.f;
        }
    };
    auto stage_rowstats = [&](int64_t h) {
        for (int n = tid; n < NS; n += NL) {
            const int64_t o = u0 + d0 + n;
            mO[n] = (o >= 0 && o < g.W) ? ro.st.box[h * g.W + o] * rk2 : 0.0;
        }
        if (tid < TW) {
            const int64_t u = u0 + tid;
            bU[tid] = u < g.W ? ro.so.box[h * g.W + u] : 0.0;
        }
    };
    auto voxel_ok = [&](int64_t y, int64_t u) {
        const int64_t o = u + delta;
        bool ok = y >= g.h_lo && y < g.h_hi && u >= 0 && u < ro.ownMax && o >= 0 && o < ro.othMax;
        if (ro.window) ok = ok && delta >= ro.dWinLo && delta <= ro.dWinHi;
        return ok;
    };
    // A(y, x-slot) = g / sqrt(X Y + eps) with fp64-accurate moments
    auto a_val = [&](int64_t y, int x) -> float {
        const int64_t u = xbase + x;
        if (!voxel_ok(y, u)) return 0.f;
        const int s = slot_of(y);
        const float gv = ro.g[(y - g.h_lo) * ro.gsH + u * ro.gsU + delta * ro.gsD + ro.gOff];
        const float s2 = __builtin_fmaf(qU[s * NX + x], qO[s * NO + x + tid], kEps);
        return gv * __builtin_amdgcn_rsqf(s2);
    };

    double colE[NX], colA[NX];
#pragma unroll
    for (int x = 0; x < NX; ++x) { colE[x] = 0.0; colA[x] = 0.0; }
    auto accE = [&](int64_t y, double sgn) {
        const int s = slot_of(y);
        const float* ru = ringU + s * NX;
        const float* rO = ringO + s * NO + tid;
#pragma unroll
        for (int x = 0; x < NX; ++x) colE[x] = fma(sgn * (double)ru[x], (double)rO[x], colE[x]);
    };

    // TPR threads per own column for the LDS reduction
    int TPR = 1;
    while (TPR * 2 * TW <= NL && TPR < 16) TPR *= 2;
    const int PER = (NL + TPR - 1) / TPR;
    const int rm = tid / TPR, rpart = tid % TPR;
    // Per-pixel sums over the workgroup's diagonals: every lane writes its TW
    // values into red[m][lane] (between red_begin and red_end), then TPR
    // threads per column add them in a fixed order (deterministic).
    auto red_begin = [&]() { __syncthreads(); };
    auto red_end = [&](double* dst, int64_t row) {
        __syncthreads();
        double acc = 0.0;
        if (rm < TW)
            for (int e = 0; e < PER; ++e) {
                const int l = rpart * PER + e;
                if (l < NL) acc += red[rm * NL + l];
            }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            if (off >= TPR) break;
            acc += __shfl_xor(acc, off);
        }
        const int64_t u = u0 + rm;
        if (rm < TW && rpart == 0 && u < g.W) dst[((int64_t)chunk * g.H + row) * g.W + u] = acc;
    };

    // warm-up of the image ring / colE: rows h0-R .. h0+R-1
    for (int64_t y = h0 - R; y < h0 + R; ++y) stage_img(y);
    __syncthreads();
    for (int64_t y = h0 - R; y < h0 + R; ++y) accE(y, 1.0);

    for (int64_t h = h0 - R; h < h1 + R; ++h) {
        const bool rowE = h >= h0 && h < h1;
        const bool rowT = h - R >= h0 && h - R < h1;
        __syncthreads();
        if (h >= h0) stage_img(h + R);
        stage_q(h);
        if (rowE) stage_rowstats(h);
        __syncthreads();

        // A entering colA (row h); keep owned columns' A for V / Am
        float aown[TW];
#pragma unroll
        for (int x = 0; x < NX; ++x) {
            const float a = a_val(h, x);
            colA[x] += (double)a;
            if (x >= R && x < R + TW) aown[x - R] = a;
        }
        if (rowE) {
            accE(h + R, 1.0);
            const int s = slot_of(h);
            double e = 0.0;
#pragma unroll
            for (int x = 0; x < 2 * R + 1; ++x) e += colE[x];
            red_begin();
#pragma unroll
            for (int m = 0; m < TW; ++m) {
                if (m > 0) e = (e + colE[m + 2 * R]) - colE[m - 1];
                const float a = aown[m];
                double bv = 0.0;
                if (a != 0.f) {
                    const double E = fma(-bU[m], mO[m + tid], e);
                    const float yq = qO[s * NO + m + R + tid];
                    const float s2 = __builtin_fmaf(qU[s * NX + m + R], yq, kEps);
                    const float V = a * (float)(E + (double)kEps) / s2;
                    bv = (double)V * (double)yq;
                }
                red[m * NL + tid] = bv;
            }
            red_end(ro.Bp, h);
            red_begin();
#pragma unroll
            for (int m = 0; m < TW; ++m) red[m * NL + tid] = (double)aown[m] * mO[m + tid];
            red_end(ro.Amp, h);
            accE(h - R, -1.0);
        }
        if (rowT) {
            // BoxA for y = h - R covers A rows [h-2R, h]
            const int64_t y = h - R;
            const int s = slot_of(y);
            double bx = 0.0;
#pragma unroll
            for (int x = 0; x < 2 * R + 1; ++x) bx += colA[x];
            red_begin();
#pragma unroll
            for (int m = 0; m < TW; ++m) {
                if (m > 0) bx = (bx + colA[m + 2 * R]) - colA[m - 1];
                red[m * NL + tid] = (double)ringO[s * NO + m + R + tid] * bx;
            }
            red_end(ro.T1p, y);
        }
        if (h >= h0 + R) {
            // A leaving colA: row h - 2R (its stats are still in the q ring)
#pragma unroll
            for (int x = 0; x < NX; ++x) colA[x] -= (double)a_val(h - 2 * R, x);
        }
    }
}

// Sum the per-chunk partials; also form mean_own * B.
__global__ __launch_bounds__(256) void k_bwd_reduce(Geo g, int nChunk, const double* __restrict__ Bp,
                                                    const double* __restrict__ Amp, const double* __restrict__ T1p,
                                                    const double* __restrict__ boxU, double* __restrict__ Bt,
                                                    double* __restrict__ Amt, double* __restrict__ T1t,
                                                    double* __restrict__ MBt) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = g.H * g.W;
    if (p >= n) return;
    double b = 0, a = 0, t = 0;
    for (int c = 0; c < nChunk; ++c) {
        b += Bp[c * n + p];
        a += Amp[c * n + p];
        t += T1p[c * n + p];
    }
    Bt[p] = b;
    Amt[p] = a;
    T1t[p] = t;
    MBt[p] = b * boxU[p] / (double)(g.k * g.k);
}

// grad(y,x) = T1 - Box[Am] - img(y,x) * Box[B] + Box[mean*B]
template <typename T>
__global__ __launch_bounds__(256) void k_bwd_combine(Geo g, const T* __restrict__ img,
                                                     const double* __restrict__ Bt, const double* __restrict__ Amt,
                                                     const double* __restrict__ T1t, const double* __restrict__ MBt,
                                                     float* __restrict__ out) {
    constexpr int TS = 16;
    extern __shared__ __attribute__((aligned(16))) double tl[];
    const int r = g.r, L = TS + 2 * r;
    double* tB = tl;
    double* tA = tB + L * L;
    double* tM = tA + L * L;
    const int64_t y0 = (int64_t)blockIdx.y * TS, x0 = (int64_t)blockIdx.x * TS;
    for (int e = threadIdx.x; e < L * L; e += 256) {
        const int64_t y = y0 + e / L - r, x = x0 + e % L - r;
        const bool ok = y >= 0 && y < g.H && x >= 0 && x < g.W;
        const int64_t q = y * g.W + x;
        tB[e] = ok ? Bt[q] : 0.0;
        tA[e] = ok ? Amt[q] : 0.0;
        tM[e] = ok ? MBt[q] : 0.0;
    }
    __syncthreads();
    const int ly = threadIdx.x / TS, lx = threadIdx.x % TS;
    const int64_t y = y0 + ly, x = x0 + lx;
    if (y >= g.H || x >= g.W) return;
    double sb = 0, sa = 0, sm = 0;
    for (int i = 0; i < g.k; ++i)
        for (int j = 0; j < g.k; ++j) {
            const int e = (ly + i) * L + lx + j;
            sb += tB[e];
            sa += tA[e];
            sm += tM[e];
        }
    const int64_t q = y * g.W + x;
    out[q] = (float)(T1t[q] - sa - (double)to_f(img[q]) * sb + sm);
}

// gT = gradient volume re-laid so the projector-role pass reads it coalesced:
//  full:   gT[h][d][w]        = g[h][w][d]
//  window: gT[h][d][s' = D-s] = g[h][w = d - s][s]   (zero where w is not a camera column)
__global__ __launch_bounds__(256) void k_transpose_full(Geo g, const float* __restrict__ src,
                                                        float* __restrict__ dst) {
    __shared__ float t[32][33];
    const int64_t h = blockIdx.z;  // volume row
    const int64_t bx = (int64_t)blockIdx.x * 32, by = (int64_t)blockIdx.y * 32;  // bx: d, by: w
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;                       // 32 x 8
    for (int i = ty; i < 32; i += 8) {
        const int64_t w = by + i, d = bx + tx;
        t[i][tx] = (w < g.W && d < g.W) ? src[(h * g.W + w) * g.W + d] : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 32; i += 8) {
        const int64_t d = bx + i, w = by + tx;
        if (d < g.W && w < g.W) dst[(h * g.W + d) * g.W + w] = t[tx][i];
    }
}

__global__ __launch_bounds__(256) void k_transpose_window(Geo g, const float* __restrict__ src,
                                                          float* __restrict__ dst) {
    extern __shared__ __attribute__((aligned(16))) float tw[];  // [32][DO]
    const int64_t h = blockIdx.y, d0 = (int64_t)blockIdx.x * 32;
    const int64_t DO = g.DO;
    for (int64_t e = threadIdx.x; e < 32 * DO; e += 256) tw[e] = 0.f;
    __syncthreads();
    // source rows w in [d0 - D, d0 + 31]; from row w take s with w + s in [d0, d0+32)
    const int64_t nrows = g.D + 32;
    for (int64_t e = threadIdx.x; e < nrows * 32; e += 256) {
        const int64_t w = d0 - g.D + e / 32;
        const int c = (int)(e % 32);
        const int64_t s = d0 + c - w;
        if (w >= 0 && w < g.WO && s >= 0 && s <= g.D) tw[c * DO + s] = src[(h * g.WO + w) * DO + s];
    }
    __syncthreads();
    for (int64_t e = threadIdx.x; e < 32 * DO; e += 256) {
        const int c = (int)(e / DO);
        const int64_t sp = e % DO, d = d0 + c;
        if (d < g.W) dst[(h * g.W + d) * DO + sp] = tw[c * DO + (g.D - sp)];
    }
}

template <int K, typename T>
hipError_t launch_role(const Geo& g, const Role& ro, const SweepGrid& sg, hipStream_t s) {
    constexpr int R = K / 2, NX = TW + 2 * R;
    const int NL = sg.NL, NO = NX + NL - 1, NS = TW + NL - 1;
    const size_t lds = sizeof(double) * (TW * NL + NS + TW) + sizeof(float) * (2 * K * NX + 2 * K * NO);
    hipLaunchKernelGGL((k_sweep_bwd<K, T>), dim3((unsigned)sweep_blocks(sg)), dim3(NL), lds, s, g, ro, sg);
    return hipGetLastError();
}

template <typename T>
hipError_t run_role(const Geo& g, const Role& ro, const SweepGrid& sg, hipStream_t s) {
    switch (g.k) {
#define CUSTMA_K(KK) \
    case KK: return launch_role<KK, T>(g, ro, sg, s);
        CUSTMA_SWEEP_KS(CUSTMA_K)
#undef CUSTMA_K
        default: return hipErrorInvalidValue;
    }
}

SweepGrid bwd_grid(const Geo& g) {
    SweepGrid sg = sweep_grid(g);
    sg.nTile = (int)cdiv(g.W, TW);  // every own-image column needs its gradient
    sg.TH = 64;
    while (sg.TH > 8 && (int64_t)sg.nTile * sg.nChunk * cdiv(g.H, sg.TH) < 2048) sg.TH /= 2;
    sg.nBand = (int)cdiv(g.H, sg.TH);
    return sg;
}

}  // namespace

size_t backward_partial_bytes(const Geo& g) {
    const SweepGrid sg = bwd_grid(g);
    const size_t n = (size_t)g.H * g.W;
    return n * 8 * (3 * (size_t)sg.nChunk + 4);
}

size_t backward_transpose_bytes(const Geo& g) {
    return (size_t)g.HV() * g.W * (size_t)g.DO * sizeof(float);
}

hipError_t launch_backward(const float* grad, const void* cam, const void* proj, int dtype, const Geo& g,
                           Stats sc, Stats sp, float* dcam, float* dproj, void* ws, hipStream_t s) {
    const SweepGrid sg = bwd_grid(g);
    const size_t n = (size_t)g.H * g.W;
    double* Bp = (double*)ws;
    double* Amp = Bp + (size_t)sg.nChunk * n;
    double* T1p = Amp + (size_t)sg.nChunk * n;
    double* Bt = T1p + (size_t)sg.nChunk * n;
    double* Amt = Bt + n;
    double* T1t = Amt + n;
    double* MBt = T1t + n;
    float* gT = (float*)(MBt + n);
    const bool win = g.layout == CUSTMA_LAYOUT_WINDOW;
    const size_t lds_c = sizeof(double) * 3 * (16 + 2 * g.r) * (16 + 2 * g.r);
    const dim3 cgrid((unsigned)cdiv(g.W, 16), (unsigned)cdiv(g.H, 16));
    const unsigned rgrid = (unsigned)cdiv((int64_t)n, 256);
    hipError_t e;

    for (int role = 0; role < 2; ++role) {
        float* out = role == 0 ? dcam : dproj;
        if (!out) continue;
        Role ro;
        ro.Bp = Bp; ro.Amp = Amp; ro.T1p = T1p;
        ro.window = win;
        if (role == 0) {  // camera: own = camera, other = projector, delta = d - w
            ro.own = cam; ro.oth = proj; ro.so = sc; ro.st = sp;
            ro.g = grad;
            if (win) { ro.gsH = g.WO * g.DO; ro.gsU = g.DO; ro.gsD = 1; ro.gOff = 0; }
            else { ro.gsH = g.W * g.W; ro.gsU = g.W + 1; ro.gsD = 1; ro.gOff = 0; }
            ro.ownMax = g.WO; ro.othMax = g.W;
            ro.dWinLo = 0; ro.dWinHi = g.D;
        } else {          // projector: own = projector, other = camera, delta' = w - d
            if (win) {
                const unsigned lds_t = (unsigned)(sizeof(float) * 32 * g.DO);
                hipLaunchKernelGGL(k_transpose_window, dim3((unsigned)cdiv(g.W, 32), (unsigned)g.HV()), dim3(256),
                                   lds_t, s, g, grad, gT);
            } else {
                hipLaunchKernelGGL(k_transpose_full, dim3((unsigned)cdiv(g.W, 32), (unsigned)cdiv(g.W, 32),
                                   (unsigned)g.HV()), dim3(256), 0, s, g, grad, gT);
            }
            if ((e = hipGetLastError()) != hipSuccess) return e;
            ro.own = proj; ro.oth = cam; ro.so = sp; ro.st = sc;
            ro.g = gT;
            if (win) { ro.gsH = g.W * g.DO; ro.gsU = g.DO; ro.gsD = 1; ro.gOff = g.D; }
            else { ro.gsH = g.W * g.W; ro.gsU = g.W + 1; ro.gsD = 1; ro.gOff = 0; }
            ro.ownMax = g.W; ro.othMax = g.WO;
            ro.dWinLo = -g.D; ro.dWinHi = 0;
        }
        SweepGrid rg = sg;
        if (win) rg.nChunk = (int)cdiv((int64_t)g.D + 1, sg.NL);
        e = dtype == CUSTMA_F16 ? run_role<__half>(g, ro, rg, s) : run_role<float>(g, ro, rg, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_bwd_reduce, dim3(rgrid), dim3(256), 0, s, g, rg.nChunk, Bp, Amp, T1p, ro.so.box, Bt,
                           Amt, T1t, MBt);
        if (dtype == CUSTMA_F16)
            hipLaunchKernelGGL(k_bwd_combine<__half>, cgrid, dim3(256), lds_c, s, g, (const __half*)ro.own, Bt, Amt,
                               T1t, MBt, out);
        else
            hipLaunchKernelGGL(k_bwd_combine<float>, cgrid, dim3(256), lds_c, s, g, (const float*)ro.own, Bt, Amt,
                               T1t, MBt, out);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace custma
