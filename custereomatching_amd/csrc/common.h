// Shared device/host definitions for the gfx950 ZNCC kernels.
// Compiled with -ffp-contract=off: every fused multiply-add below is an
// explicit __builtin_fmaf / fma, so the reference's nvcc contraction
// (custma/src/stereo_matching_kernel.cu:66-71 under -fmad=true) is
// reproduced exactly where the exact path needs it and nowhere else.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/custma.h"

namespace custma {

constexpr float kEps = 1e-8f;  // stereo_matching_kernel.cu:4

// Problem geometry shared by every kernel.
struct Geo {
    int64_t H, W;   // image
    int32_t k, r;   // kernel size, radius
    int32_t layout; // CUSTMA_LAYOUT_*
    int32_t D;
    int64_t WO, DO; // volume [h_hi - h_lo, WO, DO]
    int64_t h_lo, h_hi;  // volume rows = image rows [h_lo, h_hi) (row bands: the rest is halo)
    int32_t seg_min = 0;  // fused backward: at least this many column segments per diagonal chunk (run_bwd's
                          // tail balancing; 0 = segments of up to kSeg columns)
    __host__ __device__ int64_t HV() const { return h_hi - h_lo; }
};

// Per-image statistics produced by the stats pass ([H*W] each).
//   mean, sq : the reference's own fp32 values (sequential sum / k^2, fma chain of
//              centred squares) -- bit-identical to what every reference thread computes.
//   box      : fp64 sum of the zero-padded k x k patch (exact for fp32 inputs up to
//              2^29 dynamic range).
//   sqt      : fp64-accurate centred second moment (box2 - box^2/k^2), rounded to fp32.
struct Stats {
    float* mean;
    float* sq;
    double* box;
    float* sqt;
};

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<__half>(__half v) { return __half2float(v); }

// zero-padded read (stereo_matching_kernel.cu:6-12), 64-bit indexing
template <typename T>
__device__ __forceinline__ float ldpad(const T* img, int64_t H, int64_t W, int64_t y, int64_t x) {
    return (y < 0 || y >= H || x < 0 || x >= W) ? 0.f : to_f(img[y * W + x]);
}

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// XCD-aware block order.  Workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md, "Workgroup dispatch"): hardware block b runs on XCD
// b % 8.  Map it to a logical block so that each XCD gets one contiguous range
// of logical blocks (bijective for any grid size); neighbouring logical blocks
// then share an L2.  Only speed depends on this, never correctness.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, rem = nb % 8, x = b % 8, i = b / 8;
    return x < rem ? x * (q + 1) + i : rem * (q + 1) + (x - rem) * q + i;
}

// Volume voxel validity and linear index for camera column w, projector column d.
__device__ __forceinline__ bool voxel_valid(const Geo& g, int64_t w, int64_t d) {
    if (w < 0 || w >= g.WO || d < 0 || d >= g.W) return false;
    if (g.layout == CUSTMA_LAYOUT_WINDOW) return d >= w && d - w <= g.D;
    return true;
}
__device__ __forceinline__ int64_t voxel_index(const Geo& g, int64_t h, int64_t w, int64_t d) {
    const int64_t s = (g.layout == CUSTMA_LAYOUT_WINDOW) ? d - w : d;
    return ((h - g.h_lo) * g.WO + w) * g.DO + s;
}

// Raw buffer access (MI355X: 128-bit descriptor in SGPRs, 32-bit per-lane byte
// offset, hardware range check).  An out-of-range offset (0x80000000) makes a
// load return 0 and a store a no-op -- branch-free zero padding / masking.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <typename T>
__device__ __forceinline__ float ld_buf(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <>
__device__ __forceinline__ float ld_buf<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
template <>
__device__ __forceinline__ float ld_buf<__half>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const unsigned short b = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
    return __half2float(__ushort_as_half(b));
}
// Raw bits of one image element (no conversion at the load, so a software pipeline that
// holds loads in flight across steps does not wait for them where they are issued).
template <typename T>
__device__ __forceinline__ uint32_t ld_raw(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <>
__device__ __forceinline__ uint32_t ld_raw<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
template <>
__device__ __forceinline__ uint32_t ld_raw<__half>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}
// Software-pipelined loads whose waits the caller places itself (the compiler's vmcnt
// tracking is conservative at loop headers and would wait for the newest loads).  The
// compiler does not see these as memory operations: the caller must run
// `s_waitcnt vmcnt(N)` (asm_vmcnt) before ANY use of the destination, and tie the
// destination registers to that wait (asm_tie) so no use is scheduled above it.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 make_rsrc_sgpr(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(a >> 32) & 0xffff);  // stride 0
    r.z = __builtin_amdgcn_readfirstlane((int32_t)bytes);
    r.w = 0x00020000;
    return r;
}
template <typename T>
__device__ __forceinline__ void asm_ld_raw(uint32_t& d, uint32_t off, i32x4 r);
template <>
__device__ __forceinline__ void asm_ld_raw<float>(uint32_t& d, uint32_t off, i32x4 r) {
    asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(d) : "v"(off), "s"(r));
}
template <>
__device__ __forceinline__ void asm_ld_raw<__half>(uint32_t& d, uint32_t off, i32x4 r) {
    asm volatile("buffer_load_ushort %0, %1, %2, 0 offen" : "=v"(d) : "v"(off), "s"(r));
}
// Grouped forms for code with SGPR pressure: a VALU write of an SGPR (e.g. the v_readlane
// that restores a spilled descriptor) needs 5 wait states before a VMEM reads that SGPR
// (gfx9 "VALU writes SGPR -> VMEM reads that SGPR"), and the compiler's hazard recognizer
// does not look inside inline asm -- so each group starts with `s_nop 4`.  Outputs are
// early-clobber: no destination may alias an address operand of a later load in the group.
__device__ __forceinline__ void asm_ld5s(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t& a4,
                                         uint32_t oA, uint32_t oB, uint32_t oC, i32x4 r0, i32x4 r1, i32x4 r2,
                                         i32x4 r3, i32x4 r4, uint32_t sA, uint32_t sB) {
    asm volatile(
        "s_nop 4\n\t"
        "buffer_load_dword %0, %5, %8, %13 offen\n\t"
        "buffer_load_dword %1, %5, %9, %13 offen\n\t"
        "buffer_load_dword %2, %6, %10, %14 offen\n\t"
        "buffer_load_dword %3, %6, %11, %14 offen\n\t"
        "buffer_load_dword %4, %7, %12, %14 offen"
        : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(a4)
        : "v"(oA), "v"(oB), "v"(oC), "s"(r0), "s"(r1), "s"(r2), "s"(r3), "s"(r4), "s"(sA), "s"(sB));
}
// NOP = false drops the `s_nop 4`: only for loads whose SGPR operands no VALU op writes
// within 5 wait states before them -- custereomatching_amd/hazard_check.py (rule R1) verifies that on
// the listing at build time for the translation units that use it.
#define CUSTMA_LD_ASM(NOP, BODY, ...)                       \
    do {                                                    \
        if constexpr (NOP)                                  \
            asm volatile("s_nop 4\n\t" BODY __VA_ARGS__);  \
        else                                                \
            asm volatile(BODY __VA_ARGS__);                 \
    } while (0)
template <bool NOP = true>
__device__ __forceinline__ void asm_ld2s(uint32_t& a0, uint32_t& a1, uint32_t oA, uint32_t oB, i32x4 r0, i32x4 r1,
                                         uint32_t sA, uint32_t sB) {
    CUSTMA_LD_ASM(NOP,
                  "buffer_load_dword %0, %2, %4, %6 offen\n\t"
                  "buffer_load_dword %1, %3, %5, %7 offen",
                  : "=&v"(a0), "=&v"(a1)
                  : "v"(oA), "v"(oB), "s"(r0), "s"(r1), "s"(sA), "s"(sB));
}
template <bool NOP = true>
__device__ __forceinline__ void asm_ld1s(uint32_t& a0, uint32_t oA, i32x4 r0, uint32_t sA) {
    CUSTMA_LD_ASM(NOP, "buffer_load_dword %0, %1, %2, %3 offen", : "=&v"(a0) : "v"(oA), "s"(r0), "s"(sA));
}
template <bool NOP = true>
__device__ __forceinline__ void asm_ld4(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t oA,
                                        uint32_t oB, uint32_t oC, uint32_t oD, i32x4 r0, i32x4 r1, i32x4 r2) {
    CUSTMA_LD_ASM(NOP,
                  "buffer_load_dword %0, %4, %8, 0 offen\n\t"
                  "buffer_load_dword %1, %5, %8, 0 offen\n\t"
                  "buffer_load_dword %2, %6, %9, 0 offen\n\t"
                  "buffer_load_dword %3, %7, %10, 0 offen",
                  : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3)
                  : "v"(oA), "v"(oB), "v"(oC), "v"(oD), "s"(r0), "s"(r1), "s"(r2));
}
// Four loads through one descriptor, the first three at soffset sA, the fourth at sB.
template <bool NOP = true>
__device__ __forceinline__ void asm_ld4s(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t oA,
                                         uint32_t oB, uint32_t oC, uint32_t oD, i32x4 r, uint32_t sA, uint32_t sB) {
    CUSTMA_LD_ASM(NOP,
                  "buffer_load_dword %0, %4, %8, %9 offen\n\t"
                  "buffer_load_dword %1, %5, %8, %9 offen\n\t"
                  "buffer_load_dword %2, %6, %8, %9 offen\n\t"
                  "buffer_load_dword %3, %7, %8, %10 offen",
                  : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3)
                  : "v"(oA), "v"(oB), "v"(oC), "v"(oD), "s"(r), "s"(sA), "s"(sB));
}
// Image-row groups for the forward sweep: 8 image loads (projector enter/leave x 2 halves,
// camera enter/leave x 2 halves) / 6 statistics loads, rows selected by SGPR soffsets.
// `s_nop 4` first: the soffsets may have been written by a VALU op (hazard note above).
// Third camera register of the sweeps for 32 < 16 + k - 1 <= 48 columns (k = 19 .. 33): the entering and
// leaving rows' columns 32 + (lane & 15) of the tile.
template <typename T>
__device__ __forceinline__ void asm_ld_img2(uint32_t& ce2, uint32_t& cl2, uint32_t vC2, i32x4 dC, uint32_t sE,
                                            uint32_t sL) {
    if constexpr (sizeof(T) == 4)
        asm volatile("s_nop 4\n\tbuffer_load_dword %0, %2, %3, %4 offen\n\tbuffer_load_dword %1, %2, %3, %5 offen"
                     : "=&v"(ce2), "=&v"(cl2) : "v"(vC2), "s"(dC), "s"(sE), "s"(sL));
    else
        asm volatile("s_nop 4\n\tbuffer_load_ushort %0, %2, %3, %4 offen\n\tbuffer_load_ushort %1, %2, %3, %5 offen"
                     : "=&v"(ce2), "=&v"(cl2) : "v"(vC2), "s"(dC), "s"(sE), "s"(sL));
}
template <typename T>
__device__ __forceinline__ void asm_ld_img8(uint32_t& pe0, uint32_t& pe1, uint32_t& pl0, uint32_t& pl1,
                                            uint32_t& ce0, uint32_t& ce1, uint32_t& cl0, uint32_t& cl1,
                                            uint32_t vP0, uint32_t vP1, uint32_t vC0, uint32_t vC1, i32x4 dP,
                                            i32x4 dC, uint32_t sE, uint32_t sL) {
    if constexpr (sizeof(T) == 4) {
        asm volatile(
            "s_nop 4\n\t"
            "buffer_load_dword %0, %8, %12, %14 offen\n\t"
            "buffer_load_dword %1, %9, %12, %14 offen\n\t"
            "buffer_load_dword %2, %8, %12, %15 offen\n\t"
            "buffer_load_dword %3, %9, %12, %15 offen\n\t"
            "buffer_load_dword %4, %10, %13, %14 offen\n\t"
            "buffer_load_dword %5, %11, %13, %14 offen\n\t"
            "buffer_load_dword %6, %10, %13, %15 offen\n\t"
            "buffer_load_dword %7, %11, %13, %15 offen"
            : "=&v"(pe0), "=&v"(pe1), "=&v"(pl0), "=&v"(pl1), "=&v"(ce0), "=&v"(ce1), "=&v"(cl0), "=&v"(cl1)
            : "v"(vP0), "v"(vP1), "v"(vC0), "v"(vC1), "s"(dP), "s"(dC), "s"(sE), "s"(sL));
    } else {
        asm volatile(
            "s_nop 4\n\t"
            "buffer_load_ushort %0, %8, %12, %14 offen\n\t"
            "buffer_load_ushort %1, %9, %12, %14 offen\n\t"
            "buffer_load_ushort %2, %8, %12, %15 offen\n\t"
            "buffer_load_ushort %3, %9, %12, %15 offen\n\t"
            "buffer_load_ushort %4, %10, %13, %14 offen\n\t"
            "buffer_load_ushort %5, %11, %13, %14 offen\n\t"
            "buffer_load_ushort %6, %10, %13, %15 offen\n\t"
            "buffer_load_ushort %7, %11, %13, %15 offen"
            : "=&v"(pe0), "=&v"(pe1), "=&v"(pl0), "=&v"(pl1), "=&v"(ce0), "=&v"(ce1), "=&v"(cl0), "=&v"(cl1)
            : "v"(vP0), "v"(vP1), "v"(vC0), "v"(vC1), "s"(dP), "s"(dC), "s"(sE), "s"(sL));
    }
}
// The projector half of asm_ld_img8 (the tile kernel's camera rows come from LDS: CPL).
template <typename T>
__device__ __forceinline__ void asm_ld_img4(uint32_t& pe0, uint32_t& pe1, uint32_t& pl0, uint32_t& pl1,
                                            uint32_t vP0, uint32_t vP1, i32x4 dP, uint32_t sE, uint32_t sL) {
    if constexpr (sizeof(T) == 4) {
        asm volatile(
            "s_nop 4\n\t"
            "buffer_load_dword %0, %4, %6, %7 offen\n\t"
            "buffer_load_dword %1, %5, %6, %7 offen\n\t"
            "buffer_load_dword %2, %4, %6, %8 offen\n\t"
            "buffer_load_dword %3, %5, %6, %8 offen"
            : "=&v"(pe0), "=&v"(pe1), "=&v"(pl0), "=&v"(pl1)
            : "v"(vP0), "v"(vP1), "s"(dP), "s"(sE), "s"(sL));
    } else {
        asm volatile(
            "s_nop 4\n\t"
            "buffer_load_ushort %0, %4, %6, %7 offen\n\t"
            "buffer_load_ushort %1, %5, %6, %7 offen\n\t"
            "buffer_load_ushort %2, %4, %6, %8 offen\n\t"
            "buffer_load_ushort %3, %5, %6, %8 offen"
            : "=&v"(pe0), "=&v"(pe1), "=&v"(pl0), "=&v"(pl1)
            : "v"(vP0), "v"(vP1), "s"(dP), "s"(sE), "s"(sL));
    }
}
__device__ __forceinline__ void asm_ld_stat6(double& m0, double& m1, uint32_t& q0, uint32_t& q1, double& ub,
                                             uint32_t& uq, uint32_t vM0, uint32_t vM1, uint32_t vQ0, uint32_t vQ1,
                                             uint32_t vUB, uint32_t vUQ, i32x4 dPB, i32x4 dPS, i32x4 dCB, i32x4 dCS,
                                             uint32_t s8, uint32_t s4) {
    asm volatile("s_nop 4\n\t"
                 "buffer_load_dwordx2 %0, %6, %12, %16 offen\n\t"
                 "buffer_load_dwordx2 %1, %7, %12, %16 offen\n\t"
                 "buffer_load_dword %2, %8, %13, %17 offen\n\t"
                 "buffer_load_dword %3, %9, %13, %17 offen\n\t"
                 "buffer_load_dwordx2 %4, %10, %14, %16 offen\n\t"
                 "buffer_load_dword %5, %11, %15, %17 offen"
                 : "=&v"(m0), "=&v"(m1), "=&v"(q0), "=&v"(q1), "=&v"(ub), "=&v"(uq)
                 : "v"(vM0), "v"(vM1), "v"(vQ0), "v"(vQ1), "v"(vUB), "v"(vUQ), "s"(dPB), "s"(dPS), "s"(dCB), "s"(dCS),
                   "s"(s8), "s"(s4));
}
__device__ __forceinline__ void asm_ld_f64(double& d, uint32_t off, i32x4 r) {
    asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(d) : "v"(off), "s"(r));
}
template <int N>
__device__ __forceinline__ void asm_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt field");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// N vector-memory stores that write nothing (offset past the descriptor's range): they stand in for a
// step's N real stores where a hand-counted `s_waitcnt vmcnt` expects them in flight (inline asm, so
// the compiler neither merges nor drops them; each with its own `s_nop 4` for a VALU-written SGPR of r,
// as the compiler may restore r from VGPR lanes between them -- a few cycles, once per row band)
template <int N>
__device__ __forceinline__ void asm_null_stores(i32x4 r) {
    const uint32_t oob = 0x80000000u, z = 0u;
#pragma unroll
    for (int i = 0; i < N; ++i)
        asm volatile("s_nop 4\n\tbuffer_store_dword %0, %1, %2, 0 offen" ::"v"(z), "v"(oob), "s"(r) : "memory");
}
template <typename V>
__device__ __forceinline__ void asm_tie(V& v) {
    asm volatile("" : "+v"(v));
}
template <typename T>
__device__ __forceinline__ double raw_to_f64(uint32_t b);
template <>
__device__ __forceinline__ double raw_to_f64<float>(uint32_t b) { return (double)__builtin_bit_cast(float, b); }
template <>
__device__ __forceinline__ double raw_to_f64<__half>(uint32_t b) {
    return (double)__half2float(__ushort_as_half((unsigned short)b));
}
__device__ __forceinline__ double ld_buf_f64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
// Same with a wave-uniform byte offset `so` (SGPR soffset) added to the address.  Callers keep
// so + (any in-range voffset) below the descriptor's num_records, so an out-of-range voffset
// (0x80000000) reads 0 whether or not the hardware range check includes soffset.
template <typename T>
__device__ __forceinline__ float ld_bufs(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t so);
template <>
__device__ __forceinline__ float ld_bufs<float>(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, so, 0));
}
template <>
__device__ __forceinline__ float ld_bufs<__half>(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t so) {
    const unsigned short b = __builtin_amdgcn_raw_buffer_load_b16(r, off, so, 0);
    return __half2float(__ushort_as_half(b));
}
__device__ __forceinline__ double ld_bufs_f64(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t so) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, so, 0));
}
// Zero-padded 2-D tile of an image into LDS (as float): image rows y0 .. y0 + ny - 1, columns
// x0 .. x0 + nx - 1, at LDS row pitch `pitch`.  Raw buffer loads over the image rows from max(0, y0) on:
// an element outside the image takes an out-of-range offset and reads 0 (the reference's zero padding,
// stereo_matching_kernel.cu:6-12), so every load is unconditional and B of them per thread are in flight
// together (a bounds-tested load per element -- ldpad -- was waited for one at a time).
template <typename T, int B = 4>
__device__ __forceinline__ void tile_to_lds(const T* img, int64_t H, int64_t W, int64_t y0, int64_t x0, int ny,
                                            int nx, float* dst, int pitch, int tid, int nthreads) {
    const int64_t yb = y0 > 0 ? y0 : 0;
    const uint64_t nb = (uint64_t)(H > yb ? H - yb : 0) * (uint64_t)W * sizeof(T);
    const auto r = make_rsrc(img + yb * W, nb < 0x7FFFFFF0u ? (uint32_t)nb : 0x7FFFFFF0u);
    const int total = ny * nx;
    for (int e0 = 0; e0 < total; e0 += B * nthreads) {
        float v[B];
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const int e = e0 + tid + i * nthreads, ee = e < total ? e : 0;
            const int ty = ee / nx, tx = ee - ty * nx;
            const int64_t y = y0 + ty, x = x0 + tx;
            const bool in = e < total && y >= 0 && y < H && x >= 0 && x < W;
            v[i] = ld_bufs<T>(r, in ? (uint32_t)(((y - yb) * W + x) * (int64_t)sizeof(T)) : 0x80000000u, 0u);
        }
#pragma unroll
        for (int i = 0; i < B; ++i) {
            const int e = e0 + tid + i * nthreads;
            if (e < total) dst[(e / nx) * pitch + e % nx] = v[i];
        }
    }
}
// Cache-policy bits of the volume stores (gfx950: 1 sc0, 2 nt, 16 sc1).  nt (streaming): the
// volume is written once and far exceeds L2 / MALL, and keeping it out of L2 leaves the
// sweep's image-statistics rows there (C3 window tile kernel 1.26 -> 1.10 ms on MI355X).
constexpr int kStoreAux = 2;  // nt (sc1 alone and plain measured 2 % slower)
__device__ __forceinline__ void st_buf(float v, __amdgpu_buffer_rsrc_t r, uint32_t off) {  // plain policy
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, off, 0, 0);
}
__device__ __forceinline__ void st_vol(float v, __amdgpu_buffer_rsrc_t r, uint32_t off) {  // volume stores
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, off, 0, kStoreAux);
}

}  // namespace custma

// Dynamic LDS above 64 KiB (up to the CU's 160 KiB) must be opted into per kernel.
template <typename F>
inline hipError_t allow_lds(F* kernel, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

// ---- internal launchers (one translation unit each), called from capi.hip ----
namespace custma {
hipError_t launch_u8_to_unit(const uint8_t* src, int64_t npix, int C, int ch, int out_dtype, void* out,
                             hipStream_t s);
// Which statistics launch_stats writes (stats.hip k_stats): FULL = mean, sq, box, sqt; BOX = box, sqt (the
// generic backward); BWD_PREP = box + the fused backward's prepared images (`prep`, needs `shift`); FWD = sq,
// box (what the fast forward sweeps read).  BAND: only the volume rows [h_lo, h_hi) (a forward or disparity
// reads the statistics of its volume rows only: voxel (h, w, d) the camera's at (h, w), the projector's at
// (h, d)); otherwise every image row (the backward reads its gradient rows and their halo).
enum StatsMode {
    STATS_FULL = CUSTMA_STATS_FULL,
    STATS_BOX = CUSTMA_STATS_BOX,
    STATS_BWD_PREP = CUSTMA_STATS_BWD_PREP,
    STATS_FWD = CUSTMA_STATS_FWD,
    STATS_MSB = CUSTMA_STATS_MSB
};
enum StatsRows { STATS_ALL_ROWS = 0, STATS_BAND_ROWS = 1 };
hipError_t launch_stats(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, hipStream_t s,
                        int mode = STATS_FULL, float* prep = nullptr, const float* shift = nullptr,
                        int rows = STATS_ALL_ROWS);
hipError_t launch_fwd_exact(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            float* out, hipStream_t s);
hipError_t launch_fwd_fast(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                           float* out, hipStream_t s);
hipError_t launch_argmax(const float* vol, int64_t rows, int64_t n, int64_t* idx, float* best, hipStream_t s);
size_t disparity_partial_bytes(const Geo& g);
// soft (nullable): soft-argmax with beta; mask (nullable): best > threshold as 1 / 0
hipError_t launch_disparity(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp,
                            int64_t* idx, float* best, int32_t* n_rechecked, void* ws, hipStream_t s, float* soft,
                            float beta, float* mask, float threshold);
size_t backward_workspace_bytes(const Geo& g);
bool backward_supported(const Geo& g);
// generic backward (any k; bwd_generic.hip)
size_t backward_generic_workspace_bytes(const Geo& g);
hipError_t launch_backward_generic(const float* grad, const float* vol, const void* cam, const void* proj, int dtype,
                                   const Geo& g, Stats sc, Stats sp, float* dcam, float* dproj, void* ws,
                                   hipStream_t s);
hipError_t launch_backward(const float* grad, const float* vol, const void* cam, const void* proj, int dtype,
                           const Geo& g, Stats sc, Stats sp, float* dcam, float* dproj, void* ws, hipStream_t s);
bool fast_supported(int k);

// Optional HIP-event timing of the main kernel of an op (custma_profile_*): no-ops unless enabled.
enum ProfSlot { PROF_FWD = 0, PROF_BWD = 1, PROF_NSLOT = 2 };
void prof_begin(int slot, hipStream_t s);
void prof_end(int slot, hipStream_t s);
}  // namespace custma
