// Cross-lane helpers for 64-lane waves (gfx950 DPP / permlane), shared by the
// backward sweep and its unit test (scripts/micro/xlane_test.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace custma {

template <int L>
__device__ __forceinline__ float bcast(float a) {  // lane L of each 16-lane row, to the whole row
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x150 + L, 0xf, 0xf,
                                                                 false));
}
// The same broadcast with bound_ctrl set (row_newbcast has no out-of-range source lane, so
// the value is identical): the form the compiler folds into the consuming VOP2 op
// (v_mul_f32_dpp / v_add_f32_dpp), with its own hazard tracking.
template <int L>
__device__ __forceinline__ float rbc(float a) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x150 + L, 0xf, 0xf,
                                                                 true));
}
// Sliding column registers (backward sweep): each v moves down one lane (lane l <- v[l + 1],
// wave_shl:1) and its lane 63 takes lane 63 of its block register b, which first rotates
// down one lane (wave_rol:1: lane l <- b[(l + 1) & 63]).  After its i-th rotation since it
// was loaded, b's lane 63 holds the block's element i - 1, so a block loaded once feeds 64
// steps at two VALU ops per register and step.  The 12 own-row registers and the HP halo
// registers go through one asm block (VCC, the lane-63 select, set once by SALU).  No
// `s_nop`: the DPP sources were last written a step earlier; custereomatching_amd/hazard_check.py checks
// that on the listing at build time (rule R2: VALU write -> DPP read, 2 wait states).
template <int HP>
__device__ __forceinline__ void slide_rows(uint32_t (&v)[12], uint32_t (&b)[12], uint32_t (&hv)[HP],
                                           uint32_t (&hb)[HP], uint64_t lane63);
template <>
__device__ __forceinline__ void slide_rows<1>(uint32_t (&v)[12], uint32_t (&b)[12], uint32_t (&hv)[1], uint32_t (&hb)[1],
                                                uint64_t lane63) {
    asm volatile(
        "s_mov_b64 vcc, %26\n\t"
        "v_mov_b32_dpp %13, %13 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %14, %14 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %15, %15 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %16, %16 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %17, %17 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %18, %18 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %19, %19 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %20, %20 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %21, %21 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %22, %22 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %23, %23 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %24, %24 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %25, %25 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %0, %0, %13, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %1, %1, %14, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %2, %2, %15, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %3, %3, %16, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %4, %4, %17, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %5, %5, %18, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %6, %6, %19, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %7, %7, %20, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %8, %8, %21, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %9, %9, %22, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %10, %10, %23, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %11, %11, %24, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %12, %12, %25, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(hv[0]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
          "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]), "+v"(b[8]), "+v"(b[9]), "+v"(b[10]),
          "+v"(b[11]), "+v"(hb[0])
        : "s"(lane63)
        : "vcc");
}
template <>
__device__ __forceinline__ void slide_rows<2>(uint32_t (&v)[12], uint32_t (&b)[12], uint32_t (&hv)[2], uint32_t (&hb)[2],
                                                uint64_t lane63) {
    asm volatile(
        "s_mov_b64 vcc, %28\n\t"
        "v_mov_b32_dpp %14, %14 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %15, %15 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %16, %16 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %17, %17 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %18, %18 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %19, %19 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %20, %20 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %21, %21 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %22, %22 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %23, %23 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %24, %24 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %25, %25 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %26, %26 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %27, %27 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %0, %0, %14, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %1, %1, %15, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %2, %2, %16, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %3, %3, %17, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %4, %4, %18, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %5, %5, %19, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %6, %6, %20, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %7, %7, %21, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %8, %8, %22, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %9, %9, %23, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %10, %10, %24, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %11, %11, %25, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %12, %12, %26, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %13, %13, %27, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(hv[0]), "+v"(hv[1]), "+v"(b[0]), "+v"(b[1]),
          "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]), "+v"(b[8]), "+v"(b[9]),
          "+v"(b[10]), "+v"(b[11]), "+v"(hb[0]), "+v"(hb[1])
        : "s"(lane63)
        : "vcc");
}
template <>
__device__ __forceinline__ void slide_rows<3>(uint32_t (&v)[12], uint32_t (&b)[12], uint32_t (&hv)[3], uint32_t (&hb)[3],
                                                uint64_t lane63) {
    asm volatile(
        "s_mov_b64 vcc, %30\n\t"
        "v_mov_b32_dpp %15, %15 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %16, %16 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %17, %17 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %18, %18 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %19, %19 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %20, %20 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %21, %21 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %22, %22 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %23, %23 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %24, %24 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %25, %25 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %26, %26 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %27, %27 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %28, %28 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %29, %29 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %0, %0, %15, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %1, %1, %16, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %2, %2, %17, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %3, %3, %18, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %4, %4, %19, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %5, %5, %20, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %6, %6, %21, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %7, %7, %22, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %8, %8, %23, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %9, %9, %24, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %10, %10, %25, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %11, %11, %26, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %12, %12, %27, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %13, %13, %28, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %14, %14, %29, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(hv[0]), "+v"(hv[1]), "+v"(hv[2]), "+v"(b[0]),
          "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]), "+v"(b[8]),
          "+v"(b[9]), "+v"(b[10]), "+v"(b[11]), "+v"(hb[0]), "+v"(hb[1]), "+v"(hb[2])
        : "s"(lane63)
        : "vcc");
}
template <>
__device__ __forceinline__ void slide_rows<4>(uint32_t (&v)[12], uint32_t (&b)[12], uint32_t (&hv)[4], uint32_t (&hb)[4],
                                                uint64_t lane63) {
    asm volatile(
        "s_mov_b64 vcc, %32\n\t"
        "v_mov_b32_dpp %16, %16 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %17, %17 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %18, %18 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %19, %19 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %20, %20 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %21, %21 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %22, %22 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %23, %23 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %24, %24 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %25, %25 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %26, %26 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %27, %27 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %28, %28 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %29, %29 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %30, %30 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %31, %31 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %0, %0, %16, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %1, %1, %17, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %2, %2, %18, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %3, %3, %19, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %4, %4, %20, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %5, %5, %21, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %6, %6, %22, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %7, %7, %23, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %8, %8, %24, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %9, %9, %25, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %10, %10, %26, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %11, %11, %27, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %12, %12, %28, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %13, %13, %29, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %14, %14, %30, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %15, %15, %31, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(hv[0]), "+v"(hv[1]), "+v"(hv[2]), "+v"(hv[3]),
          "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]),
          "+v"(b[8]), "+v"(b[9]), "+v"(b[10]), "+v"(b[11]), "+v"(hb[0]), "+v"(hb[1]), "+v"(hb[2]), "+v"(hb[3])
        : "s"(lane63)
        : "vcc");
}
// More than 4 halo rows per wave (k >= 19): the first 4 as above, each further one by its own pair
// (rotate the block register, lane 63 of the column from it).  hazard_check.py checks the listing.
template <int HP>
__device__ __forceinline__ void slide_rows(uint32_t (&v)[12], uint32_t (&b)[12], uint32_t (&hv)[HP], uint32_t (&hb)[HP],
                                           uint64_t lane63) {
    static_assert(HP > 4 && HP <= 8, "slide_rows: 1 .. 8 halo rows");
    uint32_t v4[4] = {hv[0], hv[1], hv[2], hv[3]}, b4[4] = {hb[0], hb[1], hb[2], hb[3]};
    slide_rows<4>(v, b, v4, b4, lane63);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        hv[i] = v4[i];
        hb[i] = b4[i];
    }
#pragma unroll
    for (int i = 4; i < HP; ++i)
        asm volatile(
            "s_mov_b64 vcc, %2\n\t"
            "v_mov_b32_dpp %1, %1 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
            "v_cndmask_b32_dpp %0, %0, %1, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
            : "+v"(hv[i]), "+v"(hb[i])
            : "s"(lane63)
            : "vcc");
}
__device__ __forceinline__ float shl1_add(float acc, float v) {  // lane l <- acc[l+1] + v[l]; lane 63 <- v
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, acc), 0x130, 0xf, 0xf,
                                                                 true)) + v;
}
template <int CTRL>
__device__ __forceinline__ float dpp(float a) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), CTRL, 0xf, 0xf, false));
}
// v_permlane32_swap: lanes 32-63 of a <-> lanes 0-31 of b; v_permlane16_swap: the odd 16-lane
// rows of a <-> the even rows of b.  Inline asm: the builtin's second result is lost by
// hipcc (ROCm 7.2) when both results feed one add (it emitted v_add x, x, x); the two
// v_nop are the gfx950 "VALU write -> v_permlane read" wait states (cdna_hip_programming T21).
__device__ __forceinline__ void swap32(float& a, float& b) {
    asm volatile("v_nop\n\tv_nop\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap16(float& a, float& b) {
    asm volatile("v_nop\n\tv_nop\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
// DPP controls: row_mirror, row_half_mirror, quad_perm [3,2,1,0], quad_perm [1,0,3,2]
constexpr int kMirror16 = 0x140, kMirror8 = 0x141, kQuad3210 = 0x1B, kQuad1032 = 0xB1;
template <int CTRL, int BIT>
__device__ __forceinline__ float pair_level(float a, float b, int lane) {
    const float sa = a + dpp<CTRL>(a), sb = b + dpp<CTRL>(b);
    return (lane & BIT) ? sb : sa;
}
// Sum each of v[0..47] over the 64 lanes; afterwards lane bitrev6(q) holds sum q
// (q < 48).  Tree order is fixed, so the result is deterministic.
__device__ __forceinline__ float reduce48(float (&v)[48], int lane) {
    float u[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) {
        float a = v[2 * i], b = v[2 * i + 1];
        swap32(a, b);
        u[i] = a + b;
    }
    float w[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        float a = u[2 * i], b = u[2 * i + 1];
        swap16(a, b);
        w[i] = a + b;
    }
    float x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = pair_level<kMirror16, 8>(w[2 * i], w[2 * i + 1], lane);
    float y[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = pair_level<kMirror8, 4>(x[2 * i], x[2 * i + 1], lane);
    const float z0 = pair_level<kQuad3210, 2>(y[0], y[1], lane);
    const float z1 = y[2] + dpp<kQuad3210>(y[2]);
    return pair_level<kQuad1032, 1>(z0, z1, lane);
}
// A reduction level's swaps in one asm: one `s_nop 1` (the inputs may be fresh VALU results)
// instead of two v_nop per swap.
__device__ __forceinline__ void swap32x6(float& a0, float& b0, float& a1, float& b1, float& a2, float& b2, float& a3,
                                         float& b3, float& a4, float& b4, float& a5, float& b5) {
    asm volatile(
        "s_nop 1\n\t"
        "v_permlane32_swap_b32 %0, %1\n\t"
        "v_permlane32_swap_b32 %2, %3\n\t"
        "v_permlane32_swap_b32 %4, %5\n\t"
        "v_permlane32_swap_b32 %6, %7\n\t"
        "v_permlane32_swap_b32 %8, %9\n\t"
        "v_permlane32_swap_b32 %10, %11"
        : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3), "+v"(a4), "+v"(b4),
          "+v"(a5), "+v"(b5));
}
__device__ __forceinline__ void swap16x3(float& a0, float& b0, float& a1, float& b1, float& a2, float& b2) {
    asm volatile(
        "s_nop 1\n\t"
        "v_permlane16_swap_b32 %0, %1\n\t"
        "v_permlane16_swap_b32 %2, %3\n\t"
        "v_permlane16_swap_b32 %4, %5"
        : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2));
}
// Pair reductions for values produced one at a time: (a, b) -> one register holding
// a's pair sums in the low half (or even rows) and b's in the other.
__device__ __forceinline__ float red32(float a, float b) {
    swap32(a, b);
    return a + b;
}
__device__ __forceinline__ float red16(float a, float b) {
    swap16(a, b);
    return a + b;
}
// Finish 12 registers (each already summed over the 4 lanes {l, l+16, l+32, l+48}):
// afterwards every lane holds the full 64-lane sum of one of the 48 values.
__device__ __forceinline__ float reduce_tail12(const float (&w)[12], int lane) {
    float x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = pair_level<kMirror16, 8>(w[2 * i], w[2 * i + 1], lane);
    float y[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = pair_level<kMirror8, 4>(x[2 * i], x[2 * i + 1], lane);
    const float z0 = pair_level<kQuad3210, 2>(y[0], y[1], lane);
    const float z1 = y[2] + dpp<kQuad3210>(y[2]);
    return pair_level<kQuad1032, 1>(z0, z1, lane);
}

__host__ __device__ inline int bitrev6(int x) { return (int)(__builtin_bitreverse32((unsigned)x) >> 26); }

}  // namespace custma
