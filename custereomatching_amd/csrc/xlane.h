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
// Sliding column registers (backward sweep): v moves down one lane (lane l <- v[l + 1],
// wave_shl:1) and its lane 63 takes lane 63 of the block register b, which first rotates
// down one lane (wave_rol:1: lane l <- b[(l + 1) & 63]).  After its i-th rotation since it
// was loaded, b's lane 63 holds the block's element i - 1, so a block loaded once feeds 64
// steps at two VALU ops per register and step.  `s_nop 1`: a DPP source written by the
// previous VALU op needs 2 wait states; VCC (the lane-63 select) is written by SALU.
__device__ __forceinline__ void slide3(uint32_t& v0, uint32_t& v1, uint32_t& v2, uint32_t& b0, uint32_t& b1,
                                       uint32_t& b2, uint64_t lane63) {
    asm volatile(
        "s_mov_b64 vcc, %6\n\t"
        "s_nop 1\n\t"
        "v_mov_b32_dpp %3, %3 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %4, %4 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %5, %5 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %0, %0, %3, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %1, %1, %4, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "v_cndmask_b32_dpp %2, %2, %5, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(b0), "+v"(b1), "+v"(b2)
        : "s"(lane63)
        : "vcc");
}
__device__ __forceinline__ void slide1(uint32_t& v, uint32_t& b, uint64_t lane63) {
    asm volatile(
        "s_mov_b64 vcc, %2\n\t"
        "s_nop 1\n\t"
        "v_mov_b32_dpp %1, %1 wave_rol:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %0, %0, %1, vcc wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:0"
        : "+v"(v), "+v"(b)
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
