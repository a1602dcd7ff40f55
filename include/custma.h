/*
 * custma.h -- C ABI of the MI355X (gfx950) ZNCC stereo cost-volume library
 * (libcustma_hip.so).  Plain pointers, sizes and a hipStream_t passed as
 * void*; no torch types.  Every entry point returns 0 on success or a
 * negative CUSTMA_E_* code; custma_last_error() returns the message of the
 * last failure on the calling thread.
 *
 * Each entry point replaces a piece of the reference extension
 * (lzhnb/CuStereoMatching @ v0), cited file:line below.  Device pointers
 * must be on the current HIP device; images are row-major [H, W],
 * contiguous, of element type `dtype`.  Outputs are written fully (no
 * pre-zeroing needed).  `workspace` is device memory of at least
 * custma_workspace_bytes(...) bytes, owned by the caller (the torch caching
 * allocator in the Python shim); no device memory is allocated inside a call
 * and nothing synchronises the host.  Every launch of a call goes to
 * `stream` (no side streams, no library-owned streams or events), so every
 * call is hipGraph-capturable
 * (tests/test_gpu_graph.py captures forward + backward into a
 * torch.cuda.CUDAGraph and replays it bit-identically).
 */
#ifndef CUSTMA_H
#define CUSTMA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element type of the images */
#define CUSTMA_F32 0
#define CUSTMA_F16 1

/* volume layout */
#define CUSTMA_LAYOUT_FULL 0   /* [H, W, W]: out[h][w][d], every projector column d (reference behaviour,
                                  custma/src/stereo_matching_kernel.cu:35-37, :200) */
#define CUSTMA_LAYOUT_WINDOW 1 /* [H, W-D, D+1]: out[h][w][s] = full[h][w][w+s] (the reference's
                                  commented-out intent, stereo_matching_kernel.cu:30-33, :192-198) */

/* forward arithmetic */
#define CUSTMA_EXACT 0 /* bit-identical to the reference arithmetic (nvcc -fmad=true): per voxel a k*k-long
                          fp32 fma chain, IEEE sqrt and divide (stereo_matching_kernel.cu:39-71) */
#define CUSTMA_FAST 1  /* fp64 sliding-window sums: |cost - exact| <= (k^2+6) 2^-24 */

/* ops for custma_workspace_bytes */
#define CUSTMA_OP_FORWARD 0
#define CUSTMA_OP_BACKWARD 1
#define CUSTMA_OP_DISPARITY 2
#define CUSTMA_OP_BACKWARD_RECOMPUTE 3 /* custma_backward with cost_volume == NULL */

/* error codes */
#define CUSTMA_OK 0
#define CUSTMA_E_ARG (-1)       /* bad scalar argument (shape, kernel size, layout, D, dtype) */
#define CUSTMA_E_NULL (-2)      /* null pointer where one is required */
#define CUSTMA_E_WORKSPACE (-3) /* workspace too small */
#define CUSTMA_E_LAUNCH (-4)    /* HIP launch / runtime error */
#define CUSTMA_E_UNSUPPORTED (-5)

/* kernel_size range.  Even k has its taps at offsets -k/2 .. k-1-k/2, exactly as the reference's
 * `kernel_size / 2` origin (stereo_matching_kernel.cu:44,60).  Every k <= 31 runs the sliding-window
 * kernels (fused backward, fused disparity; the fast volume up to k = 11, where it stays within 1e-5 of
 * the reference, the exact one above -- capi.hip kFastVolumeMaxK); the exact forward has compile-time instantiations up to k = 33;
 * other sizes up to CUSTMA_MAX_KERNEL run the runtime-k exact forward and the generic fp64 backward. */
#define CUSTMA_MAX_KERNEL 63

int custma_abi_version(void); /* 2 */
const char* custma_last_error(void);

/* Volume dims for a layout: *wo = W (full) or W-D (window); *dout = W or D+1. */
int custma_volume_dims(int64_t H, int64_t W, int32_t layout, int32_t D, int64_t* wo, int64_t* dout);

size_t custma_workspace_bytes(int64_t H, int64_t W, int32_t kernel_size, int32_t layout, int32_t D,
                              int32_t op);

/* Forward cost volume.
 * Replaces stereo::stereo_matching_forward (custma/src/stereo_matching.cpp:16-42) and
 * stereo::stereo_matching_forward_wrapper + forward_cost_volume_kernel
 * (custma/src/stereo_matching_kernel.cu:17-72, :182-216).
 * `D` is ignored for CUSTMA_LAYOUT_FULL, exactly like the reference. */
int custma_forward(const void* camera, const void* projector, int32_t dtype, int64_t H, int64_t W,
                   int32_t kernel_size, int32_t layout, int32_t D, int32_t precision, float* cost_volume,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Backward: gradients of sum(grad * cost_volume) w.r.t. both images.
 * Replaces stereo::stereo_matching_backward (custma/src/stereo_matching.cpp:45-73) and
 * stereo_matching_backward_wrapper + get_patches_grad_kernel + patches_grad_to_image_kernel
 * (custma/src/stereo_matching_kernel.cu:75-179, :218-261).  Deterministic (no atomics).
 * `cost_volume` is the forward's output for the same images (the autograd op keeps it); NULL makes
 * the call recompute it into the workspace exactly as custma_forward(precision FAST) returns it (the
 * sliding fp64 volume up to k = 11, the exact one above; size the workspace with
 * CUSTMA_OP_BACKWARD_RECOMPUTE).
 * Window layouts with D = 64 n recompute the last diagonal's cost from the images rather than read
 * it (one 128-byte line per voxel saved), as the reference recomputes every voxel's cost.
 * camera_grad / projector_grad may each be NULL (not computed); the reference computes the
 * camera gradient only (custma/stereo_matching_wrapper.py:33). */
int custma_backward(const float* grad, const float* cost_volume, const void* camera, const void* projector,
                    int32_t dtype, int64_t H, int64_t W, int32_t kernel_size, int32_t layout, int32_t D,
                    float* camera_grad, float* projector_grad, void* workspace, size_t workspace_bytes, void* stream);

/* Row-band variants (multi-GPU row sharding): the image buffers hold H rows -- a band plus
 * its halo -- and only volume rows [row_begin, row_end) are produced / consumed.  The volume (and grad)
 * has row_end - row_begin rows; patches of those rows read the halo rows, and zero padding applies only
 * at the buffer's edges (= the global image's edges when the band has no halo there).  The backward
 * writes gradients for all H buffer rows: the halo rows hold partial sums a neighbour must add. */
int custma_forward_band(const void* camera, const void* projector, int32_t dtype, int64_t H, int64_t W,
                        int32_t kernel_size, int32_t layout, int32_t D, int32_t precision, int64_t row_begin,
                        int64_t row_end, float* cost_volume, void* workspace, size_t workspace_bytes,
                        void* stream);
int custma_backward_band(const float* grad, const float* cost_volume, const void* camera, const void* projector,
                         int32_t dtype, int64_t H, int64_t W, int32_t kernel_size, int32_t layout, int32_t D,
                         int64_t row_begin, int64_t row_end, float* camera_grad, float* projector_grad,
                         void* workspace, size_t workspace_bytes, void* stream);
int custma_disparity_band(const void* camera, const void* projector, int32_t dtype, int64_t H, int64_t W,
                          int32_t kernel_size, int32_t layout, int32_t D, int64_t row_begin, int64_t row_end,
                          int64_t* index, float* best, int32_t* n_rechecked, void* workspace,
                          size_t workspace_bytes, void* stream);

/* Optional timing of the main kernel of each forward (which = 0: the fast sweep) / backward (which = 1: the
 * fused gradient sweep) launched on the calling thread while enabled: HIP events recorded on the op's stream
 * around that one launch (bench.py uses it for the roofline figure over its timed region).
 * custma_profile_enable(1) starts a new collection; custma_profile_mean_ms synchronises on the last end
 * event, returns the mean duration and the number of launches, and clears the collection. */
int custma_profile_enable(int32_t on);
int custma_profile_mean_ms(int32_t which, float* ms, int32_t* count);

/* Diagnostics (parity tests): the per-pixel patch statistics every op computes first, for image rows
 * [row_begin, row_end) of both images (plane 0 = camera, 1 = projector), in `mode`:
 *   FULL      mean, sq, box, sqt        BOX   box, sqt
 *   BWD_PREP  box + the fused backward's six prepared fp32 images into prep ([2][3][H][W]: X = centred
 *             moment, patch mean - shift[i], raw image), given shift[2]
 *   FWD       sq, box                   MSB   mean, sq, box
 * mean / sq: the reference's own fp32 patch mean and centred-square chain (stereo_matching_kernel.cu:40-69);
 * box: fp64 patch sum; sqt: fp64-accurate centred moment rounded to fp32.  Outputs: box [2][H][W] doubles,
 * mean / sq / sqt [2][H][W] floats (all four non-NULL; fields the mode does not write are left as they are).
 * No counterpart in the reference (its kernel recomputes them per voxel). */
#define CUSTMA_STATS_FULL 0
#define CUSTMA_STATS_BOX 1
#define CUSTMA_STATS_BWD_PREP 2
#define CUSTMA_STATS_FWD 3
#define CUSTMA_STATS_MSB 4
int custma_patch_stats(const void* camera, const void* projector, int32_t dtype, int64_t H, int64_t W,
                       int32_t kernel_size, int32_t mode, int64_t row_begin, int64_t row_end, double* box,
                       float* mean, float* sq, float* sqt, const float* shift, float* prep, void* stream);

/* Image preprocessing before the path (examples/verify.py:138-142, 148): an 8-bit image [H][W][channels]
 * (interleaved, as cv2.imread returns it; channels = 1 for grayscale) -> out[H][W] = image[.][.][channel] / 255,
 * computed as numpy does (float64 division, rounded once to float32; out_dtype CUSTMA_F16 rounds that float32
 * to float16).  Replaces the host-side `np.array(cv2.imread(...)) / 255` + `torch.tensor(..., float32).cuda()`
 * + `rgb[:, :, 0]` of the reference's driver with one HBM pass on the device. */
int custma_image_u8_to_unit(const uint8_t* image, int64_t H, int64_t W, int32_t channels, int32_t channel,
                            int32_t out_dtype, void* out, void* stream);

/* First-index argmax over the last axis of a [rows, n] fp32 array (torch.argmax semantics), as the
 * reference's callers do on the volume (examples/verify.py:72, examples/test.py:78-83).  n < 2^29
 * (CUSTMA_E_UNSUPPORTED otherwise: a row is read through one 32-bit buffer range). */
int custma_argmax(const float* volume, int64_t rows, int64_t n, int64_t* index, float* best, void* stream);

/* Fused disparity without materialising the volume: index[h][w] = argmax_s cost(h, w, s) (first index
 * on ties; s as in the layout), best[h][w] = that cost.  Computed by the fast path and certified: every
 * pixel whose fast top-2 gap is below the fast path's error margin is re-decided with the exact
 * reference arithmetic, so `index` is bit-identical to argmax of the CUSTMA_EXACT volume.
 * n_rechecked (device int32, may be NULL) receives the number of re-decided pixels. */
int custma_disparity(const void* camera, const void* projector, int32_t dtype, int64_t H, int64_t W,
                     int32_t kernel_size, int32_t layout, int32_t D, int64_t* index, float* best,
                     int32_t* n_rechecked, void* workspace, size_t workspace_bytes, void* stream);

/* Fused disparity with the rest of the reference caller's post-processing, still without the volume
 * (examples/test.py:78-86; examples/verify.py:31-39 soft_argmax, :72-74 max-cost mask), over volume rows
 * [row_begin, row_end) of a (haloed) band:
 *   index, best   as custma_disparity (index certified bit-identical to argmax of the exact volume)
 *   soft          (nullable) sum_s s softmax(beta * cost)_s over the layout's last axis s, from the fast
 *                 costs (the exact ones for re-decided pixels); beta > 0
 *   mask          (nullable) 1.0f where best > threshold, else 0.0f (the reference's torch.where)
 * Workspace: custma_workspace_bytes(..., CUSTMA_OP_DISPARITY). */
int custma_disparity_soft_band(const void* camera, const void* projector, int32_t dtype, int64_t H, int64_t W,
                               int32_t kernel_size, int32_t layout, int32_t D, int64_t row_begin, int64_t row_end,
                               float beta, float threshold, int64_t* index, float* best, float* soft, float* mask,
                               int32_t* n_rechecked, void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CUSTMA_H */
