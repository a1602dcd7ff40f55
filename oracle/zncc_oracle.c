/*
 * zncc_oracle.c -- CPU restatement of the reference ZNCC stereo cost volume.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (custereomatching_amd) never links, loads or calls it.
 *
 * It restates, in plain C, the arithmetic of the reference CUDA kernels of
 * lzhnb/CuStereoMatching (reference @ v0):
 *
 *   query_ij            custma/src/stereo_matching_kernel.cu:6-12   (zero pad)
 *   EPSILON = 1e-8f     custma/src/stereo_matching_kernel.cu:4
 *   forward             custma/src/stereo_matching_kernel.cu:39-71
 *   backward (patch g)  custma/src/stereo_matching_kernel.cu:97-151
 *   patch -> image      custma/src/stereo_matching_kernel.cu:155-179
 *
 * Floating-point contract.  The reference is built by nvcc with its default
 * -fmad=true, -prec-div=true, -prec-sqrt=true (setup.py:28-40 passes no
 * flags).  So every `acc += a * b` in the kernel is one fmaf, `ex2 * ey2 +
 * EPSILON` is fmaf(ex2, ey2, EPSILON), and `/`, `sqrtf` are IEEE
 * round-to-nearest.  ORC_CONTRACT=1 reproduces that; ORC_CONTRACT=0 is the
 * other legal compilation (-fmad=false: separate multiply and add).  This
 * file must be compiled with -ffp-contract=off so that only the explicit
 * fmaf() calls fuse.
 *
 * Layouts.  layout 0 ("full") is what the reference returns: [H, W, W],
 * out[h][w][d] for every projector column d of the same row
 * (stereo_matching_kernel.cu:35-37, :200).  layout 1 ("window") is the
 * reference's commented-out intent [H, W-D, D+1] (:30-33, :192-198) with the
 * convention out[h][w][s] = full[h][w][w+s].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EPS 1e-8f /* stereo_matching_kernel.cu:4 */

/* stereo_matching_kernel.cu:6-12 */
static inline float q(const float* img, int64_t H, int64_t W, int64_t i, int64_t j) {
    return (i < 0 || i >= H || j < 0 || j >= W) ? 0.f : img[i * W + j];
}

static inline float mac(float acc, float a, float b, int contract) {
    return contract ? fmaf(a, b, acc) : acc + a * b;
}

static inline void vol_dims(int64_t H, int64_t W, int layout, int D, int64_t* WO, int64_t* DO) {
    if (layout == 0) { *WO = W; *DO = W; }
    else { *WO = W - D; *DO = (int64_t)D + 1; }
    (void)H;
}

static inline int64_t d_of(int layout, int64_t w, int64_t s) { return layout == 0 ? s : w + s; }

int orc_volume_dims(int64_t H, int64_t W, int layout, int D, int64_t* WO, int64_t* DO) {
    if (layout != 0 && layout != 1) return -1;
    if (layout == 1 && (D < 0 || D >= W)) return -2;
    vol_dims(H, W, layout, D, WO, DO);
    return 0;
}

/* Per-pixel patch statistics, in the reference's order: mean = (sum_{i,j}
 * q) / (k*k) with a sequential float sum (.cu:40-54), then sq = sum_{i,j}
 * (q - mean)^2 as an fma chain (.cu:56-69).  Every reference thread computes
 * exactly this sequence for its camera pixel (h,w) and projector pixel (h,d),
 * so hoisting it per pixel is bit-identical. */
int orc_stats(const float* img, int64_t H, int64_t W, int k, int contract, float* mean, float* sq) {
    if (k <= 0) return -3; /* even k: taps at offsets -k/2 .. k-1-k/2, as .cu:44,60 */
    const int64_t r = k / 2;
    for (int64_t h = 0; h < H; ++h)
        for (int64_t w = 0; w < W; ++w) {
            float m = 0.f;
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) m += q(img, H, W, h + i - r, w + j - r);
            m /= (float)(k * k);
            float s = 0.f;
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    const float v = q(img, H, W, h + i - r, w + j - r) - m;
                    s = mac(s, v, v, contract);
                }
            mean[h * W + w] = m;
            sq[h * W + w] = s;
        }
    return 0;
}

/* Literal restatement of forward_cost_volume_kernel (.cu:17-72): every voxel
 * recomputes its own means and moments.  Slow (O(k^2) per voxel, twice);
 * used to pin orc_forward on small inputs. */
int orc_forward_literal(const float* cam, const float* proj, int64_t H, int64_t W, int k,
                        int layout, int D, int contract, float* out) {
    int64_t WO, DO;
    int rc = orc_volume_dims(H, W, layout, D, &WO, &DO);
    if (rc) return rc;
    if (k <= 0) return -3; /* even k: taps at offsets -k/2 .. k-1-k/2, as .cu:44,60 */
    const int64_t r = k / 2;
    for (int64_t h = 0; h < H; ++h)
        for (int64_t w = 0; w < WO; ++w)
            for (int64_t s = 0; s < DO; ++s) {
                const int64_t d = d_of(layout, w, s);
                float cm = 0.f, pm = 0.f;
                for (int i = 0; i < k; ++i)
                    for (int j = 0; j < k; ++j) {
                        cm += q(cam, H, W, h + i - r, w + j - r);
                        pm += q(proj, H, W, h + i - r, d + j - r);
                    }
                cm /= (float)(k * k);
                pm /= (float)(k * k);
                float exy = 0.f, ex2 = 0.f, ey2 = 0.f;
                for (int i = 0; i < k; ++i)
                    for (int j = 0; j < k; ++j) {
                        const float c = q(cam, H, W, h + i - r, w + j - r) - cm;
                        const float p = q(proj, H, W, h + i - r, d + j - r) - pm;
                        exy = mac(exy, c, p, contract);
                        ex2 = mac(ex2, c, c, contract);
                        ey2 = mac(ey2, p, p, contract);
                    }
                const float den = sqrtf(contract ? fmaf(ex2, ey2, ORC_EPS) : ex2 * ey2 + ORC_EPS);
                out[(h * WO + w) * DO + s] = (exy + ORC_EPS) / den;
            }
    return 0;
}

/* Same arithmetic as orc_forward_literal with the per-pixel statistics
 * hoisted (bit-identical, see orc_stats) and the centred patches cached per
 * row.  This is the oracle the tests use at every size. */
int orc_forward(const float* cam, const float* proj, int64_t H, int64_t W, int k,
                int layout, int D, int contract, float* out) {
    int64_t WO, DO;
    int rc = orc_volume_dims(H, W, layout, D, &WO, &DO);
    if (rc) return rc;
    if (k <= 0) return -3; /* even k: taps at offsets -k/2 .. k-1-k/2, as .cu:44,60 */
    const int64_t r = k / 2, K = (int64_t)k * k;
    float* cm = (float*)malloc(sizeof(float) * H * W);
    float* cx = (float*)malloc(sizeof(float) * H * W);
    float* pm = (float*)malloc(sizeof(float) * H * W);
    float* py = (float*)malloc(sizeof(float) * H * W);
    float* xt = (float*)malloc(sizeof(float) * W * K); /* centred camera patches of row h */
    float* yt = (float*)malloc(sizeof(float) * W * K); /* centred projector patches */
    if (!cm || !cx || !pm || !py || !xt || !yt) { rc = -10; goto done; }
    orc_stats(cam, H, W, k, contract, cm, cx);
    orc_stats(proj, H, W, k, contract, pm, py);
    for (int64_t h = 0; h < H; ++h) {
        for (int64_t w = 0; w < W; ++w)
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    xt[w * K + i * k + j] = q(cam, H, W, h + i - r, w + j - r) - cm[h * W + w];
                    yt[w * K + i * k + j] = q(proj, H, W, h + i - r, w + j - r) - pm[h * W + w];
                }
        for (int64_t w = 0; w < WO; ++w) {
            const float* a = xt + w * K;
            const float ex2 = cx[h * W + w];
            for (int64_t s = 0; s < DO; ++s) {
                const int64_t d = d_of(layout, w, s);
                const float* b = yt + d * K;
                float exy = 0.f;
                for (int64_t t = 0; t < K; ++t) exy = mac(exy, a[t], b[t], contract);
                const float ey2 = py[h * W + d];
                const float den = sqrtf(contract ? fmaf(ex2, ey2, ORC_EPS) : ex2 * ey2 + ORC_EPS);
                out[(h * WO + w) * DO + s] = (exy + ORC_EPS) / den;
            }
        }
    }
done:
    free(cm); free(cx); free(pm); free(py); free(xt); free(yt);
    return rc;
}

/* fp64 "truth" of the same formula (no rounding to fp32 until the end). */
int orc_forward_f64(const float* cam, const float* proj, int64_t H, int64_t W, int k,
                    int layout, int D, double* out) {
    int64_t WO, DO;
    int rc = orc_volume_dims(H, W, layout, D, &WO, &DO);
    if (rc) return rc;
    if (k <= 0) return -3; /* even k: taps at offsets -k/2 .. k-1-k/2, as .cu:44,60 */
    const int64_t r = k / 2, K = (int64_t)k * k;
    double* xt = (double*)malloc(sizeof(double) * W * K);
    double* yt = (double*)malloc(sizeof(double) * W * K);
    double* sx = (double*)malloc(sizeof(double) * W);
    double* sy = (double*)malloc(sizeof(double) * W);
    if (!xt || !yt || !sx || !sy) { rc = -10; goto done; }
    for (int64_t h = 0; h < H; ++h) {
        for (int64_t w = 0; w < W; ++w) {
            double mc = 0, mp = 0;
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    mc += q(cam, H, W, h + i - r, w + j - r);
                    mp += q(proj, H, W, h + i - r, w + j - r);
                }
            mc /= (double)K; mp /= (double)K;
            double a = 0, b = 0;
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    const double x = q(cam, H, W, h + i - r, w + j - r) - mc;
                    const double y = q(proj, H, W, h + i - r, w + j - r) - mp;
                    xt[w * K + i * k + j] = x; yt[w * K + i * k + j] = y;
                    a += x * x; b += y * y;
                }
            sx[w] = a; sy[w] = b;
        }
        for (int64_t w = 0; w < WO; ++w)
            for (int64_t s = 0; s < DO; ++s) {
                const int64_t d = d_of(layout, w, s);
                double e = 0;
                for (int64_t t = 0; t < K; ++t) e += xt[w * K + t] * yt[d * K + t];
                out[(h * WO + w) * DO + s] = (e + (double)ORC_EPS) / sqrt(sx[w] * sy[d] + (double)ORC_EPS);
            }
    }
done:
    free(xt); free(yt); free(sx); free(sy);
    return rc;
}

/* Backward.  The reference (get_patches_grad_kernel, .cu:97-151) gives, for
 * each voxel and tap t, the patch gradient
 *     g * ( y_t / S  -  Y * x_t * (E + eps) / S^3 ),   S = sqrt(X*Y + eps)
 * (deno, deno3 at .cu:135; the centring Jacobian is omitted because both
 * centred patches sum to zero), summed over the voxels of a pixel with
 * float atomics, then scattered to the image skipping out-of-bounds taps
 * (.cu:155-179).  The atomics make the reference non-deterministic; this
 * oracle sums in double in a fixed order, so it is the reference's value
 * without the arrival-order noise.  The projector gradient is the symmetric
 * formula (the reference returns None for it, stereo_matching_wrapper.py:33). */
int orc_backward(const float* g, const float* cam, const float* proj, int64_t H, int64_t W, int k,
                 int layout, int D, float* dcam, float* dproj) {
    int64_t WO, DO;
    int rc = orc_volume_dims(H, W, layout, D, &WO, &DO);
    if (rc) return rc;
    if (k <= 0) return -3; /* even k: taps at offsets -k/2 .. k-1-k/2, as .cu:44,60 */
    const int64_t r = k / 2, K = (int64_t)k * k;
    float* cm = (float*)malloc(sizeof(float) * H * W);
    float* cx = (float*)malloc(sizeof(float) * H * W);
    float* pm = (float*)malloc(sizeof(float) * H * W);
    float* py = (float*)malloc(sizeof(float) * H * W);
    float* xt = (float*)malloc(sizeof(float) * W * K);
    float* yt = (float*)malloc(sizeof(float) * W * K);
    double* pgc = (double*)calloc((size_t)(W * K), sizeof(double)); /* camera patch grads, row h */
    double* pgp = (double*)calloc((size_t)(W * K), sizeof(double)); /* projector patch grads */
    double* acc_c = (double*)calloc((size_t)(H * W), sizeof(double));
    double* acc_p = (double*)calloc((size_t)(H * W), sizeof(double));
    if (!cm || !cx || !pm || !py || !xt || !yt || !pgc || !pgp || !acc_c || !acc_p) { rc = -10; goto done; }
    orc_stats(cam, H, W, k, 1, cm, cx);
    orc_stats(proj, H, W, k, 1, pm, py);
    for (int64_t h = 0; h < H; ++h) {
        for (int64_t w = 0; w < W; ++w)
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    xt[w * K + i * k + j] = q(cam, H, W, h + i - r, w + j - r) - cm[h * W + w];
                    yt[w * K + i * k + j] = q(proj, H, W, h + i - r, w + j - r) - pm[h * W + w];
                }
        memset(pgc, 0, sizeof(double) * W * K);
        memset(pgp, 0, sizeof(double) * W * K);
        for (int64_t w = 0; w < WO; ++w) {
            const float* a = xt + w * K;
            const double X = cx[h * W + w];
            for (int64_t s = 0; s < DO; ++s) {
                const int64_t d = d_of(layout, w, s);
                const double gv = g[(h * WO + w) * DO + s];
                if (gv == 0.0) continue;
                const float* b = yt + d * K;
                float exy = 0.f;
                for (int64_t t = 0; t < K; ++t) exy = fmaf(a[t], b[t], exy);
                const double Y = py[h * W + d];
                const double S = sqrt((double)fmaf((float)X, (float)Y, ORC_EPS));
                const double inv = 1.0 / S, inv3 = inv * inv * inv;
                const double E = (double)exy + (double)ORC_EPS;
                for (int64_t t = 0; t < K; ++t) {
                    pgc[w * K + t] += gv * (b[t] * inv - Y * a[t] * E * inv3);
                    pgp[d * K + t] += gv * (a[t] * inv - X * b[t] * E * inv3);
                }
            }
        }
        for (int64_t w = 0; w < W; ++w)
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    const int64_t y = h + i - r, x = w + j - r;
                    if (y < 0 || y >= H || x < 0 || x >= W) continue; /* .cu:177 */
                    acc_c[y * W + x] += pgc[w * K + i * k + j];
                    acc_p[y * W + x] += pgp[w * K + i * k + j];
                }
    }
    for (int64_t n = 0; n < H * W; ++n) {
        if (dcam) dcam[n] = (float)acc_c[n];
        if (dproj) dproj[n] = (float)acc_p[n];
    }
done:
    free(cm); free(cx); free(pm); free(py); free(xt); free(yt);
    free(pgc); free(pgp); free(acc_c); free(acc_p);
    return rc;
}

/* fp64 truth of the backward: the same formula with means, centred patches,
 * moments and E all in double.  (It equals torch fp64 autograd of
 * examples/verify.py:107-123 to ~1e-15, the centring Jacobian being exactly
 * zero in exact arithmetic.)  The fp32 reference arithmetic above deviates
 * from it by up to ~1.5e-5 * max|grad| on ill-conditioned (quantized, flat)
 * images -- the reference's own rounding, see DESIGN.md §6. */
int orc_backward_f64(const float* g, const float* cam, const float* proj, int64_t H, int64_t W, int k,
                     int layout, int D, double* dcam, double* dproj) {
    int64_t WO, DO;
    int rc = orc_volume_dims(H, W, layout, D, &WO, &DO);
    if (rc) return rc;
    if (k <= 0) return -3; /* even k: taps at offsets -k/2 .. k-1-k/2, as .cu:44,60 */
    const int64_t r = k / 2, K = (int64_t)k * k;
    double* xt = (double*)malloc(sizeof(double) * W * K);
    double* yt = (double*)malloc(sizeof(double) * W * K);
    double* sx = (double*)malloc(sizeof(double) * W);
    double* sy = (double*)malloc(sizeof(double) * W);
    double* pgc = (double*)malloc(sizeof(double) * W * K);
    double* pgp = (double*)malloc(sizeof(double) * W * K);
    if (!xt || !yt || !sx || !sy || !pgc || !pgp) { rc = -10; goto done; }
    for (int64_t n = 0; n < H * W; ++n) { dcam[n] = 0; dproj[n] = 0; }
    for (int64_t h = 0; h < H; ++h) {
        for (int64_t w = 0; w < W; ++w) {
            double mc = 0, mp = 0;
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    mc += q(cam, H, W, h + i - r, w + j - r);
                    mp += q(proj, H, W, h + i - r, w + j - r);
                }
            mc /= (double)K; mp /= (double)K;
            double a = 0, b = 0;
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    const double x = q(cam, H, W, h + i - r, w + j - r) - mc;
                    const double y = q(proj, H, W, h + i - r, w + j - r) - mp;
                    xt[w * K + i * k + j] = x; yt[w * K + i * k + j] = y;
                    a += x * x; b += y * y;
                }
            sx[w] = a; sy[w] = b;
        }
        memset(pgc, 0, sizeof(double) * W * K);
        memset(pgp, 0, sizeof(double) * W * K);
        for (int64_t w = 0; w < WO; ++w)
            for (int64_t s = 0; s < DO; ++s) {
                const int64_t d = d_of(layout, w, s);
                const double gv = g[(h * WO + w) * DO + s];
                if (gv == 0.0) continue;
                const double* a = xt + w * K;
                const double* b = yt + d * K;
                double e = 0;
                for (int64_t t = 0; t < K; ++t) e += a[t] * b[t];
                const double S = sqrt(sx[w] * sy[d] + (double)ORC_EPS);
                const double inv = 1.0 / S, inv3 = inv * inv * inv, E = e + (double)ORC_EPS;
                for (int64_t t = 0; t < K; ++t) {
                    pgc[w * K + t] += gv * (b[t] * inv - sy[d] * a[t] * E * inv3);
                    pgp[d * K + t] += gv * (a[t] * inv - sx[w] * b[t] * E * inv3);
                }
            }
        for (int64_t w = 0; w < W; ++w)
            for (int i = 0; i < k; ++i)
                for (int j = 0; j < k; ++j) {
                    const int64_t y = h + i - r, x = w + j - r;
                    if (y < 0 || y >= H || x < 0 || x >= W) continue;
                    dcam[y * W + x] += pgc[w * K + i * k + j];
                    dproj[y * W + x] += pgp[w * K + i * k + j];
                }
    }
done:
    free(xt); free(yt); free(sx); free(sy); free(pgc); free(pgp);
    return rc;
}

/* First-index argmax over the last axis (torch.argmax / torch.max
 * semantics, which the caller uses at examples/verify.py:72 and
 * examples/test.py:78-83). NaN is not expected (costs are finite). */
int orc_argmax(const float* vol, int64_t rows, int64_t n, int64_t* idx, float* best) {
    for (int64_t p = 0; p < rows; ++p) {
        const float* v = vol + p * n;
        int64_t bi = 0;
        float bv = v[0];
        for (int64_t s = 1; s < n; ++s)
            if (v[s] > bv) { bv = v[s]; bi = s; }
        idx[p] = bi;
        if (best) best[p] = bv;
    }
    return 0;
}
