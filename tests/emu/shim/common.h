// CPU emulation shim for custereomatching_amd/csrc/stats.hip (tests/test_stats_emulated.py).
// Stands in for csrc/common.h: the HIP keywords become host C++, a launch runs every workgroup in
// turn with its threads as std::threads meeting at a std::barrier for __syncthreads(), and the
// dynamic LDS is a per-workgroup buffer.  The structs / enums the kernel reads are taken from the
// real csrc/common.h by the test (the placeholder line below), so a layout change there cannot drift here.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <barrier>
#include <thread>
#include <vector>

#include "custma.h"

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__

struct dim3 {
    unsigned x, y, z;
    dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};
inline thread_local dim3 threadIdx;
inline dim3 blockIdx, gridDim, blockDim;
inline std::barrier<>* g_bar = nullptr;
inline double* g_lds = nullptr;
inline void __syncthreads() { g_bar->arrive_and_wait(); }

typedef void* hipStream_t;
typedef int hipError_t;
constexpr hipError_t hipSuccess = 0;
inline hipError_t hipGetLastError() { return hipSuccess; }

struct __half {
    uint16_t bits;
};
inline float __half2float(__half h) {
    const uint32_t s = (h.bits >> 15) & 1, e = (h.bits >> 10) & 31, m = h.bits & 1023;
    float v = e == 0 ? ldexpf((float)m, -24) : e == 31 ? (m ? NAN : INFINITY) : ldexpf((float)(m | 1024), (int)e - 25);
    return s ? -v : v;
}

template <typename K, typename... A>
void emu_launch(K kernel, dim3 grid, dim3 block, size_t lds, A... args) {
    const unsigned nt = block.x * block.y * block.z;
    std::vector<double> mem(lds / 8 + 16, 0.0);
    gridDim = grid;
    blockDim = block;
    for (unsigned z = 0; z < grid.z; ++z)
        for (unsigned y = 0; y < grid.y; ++y)
            for (unsigned x = 0; x < grid.x; ++x) {
                blockIdx = dim3(x, y, z);
                // LDS is not cleared between workgroups on the GPU either: poison it
                memset(mem.data(), 0xA5, mem.size() * sizeof(double));
                g_lds = mem.data();
                std::barrier<> bar(nt);
                g_bar = &bar;
                std::vector<std::thread> th;
                for (unsigned t = 0; t < nt; ++t)
                    th.emplace_back([&, t] {
                        threadIdx = dim3(t, 0, 0);
                        kernel(args...);
                    });
                for (auto& h : th) h.join();
            }
}
#define hipLaunchKernelGGL(K, G, B, L, S, ...) emu_launch(K, G, B, L, __VA_ARGS__)

namespace custma {
@EMU_DECLS@
template <typename F>
inline hipError_t allow_lds(F*, size_t) { return hipSuccess; }
template <typename T>
inline float to_f(T v);
template <>
inline float to_f<float>(float v) { return v; }
template <>
inline float to_f<__half>(__half v) { return __half2float(v); }
template <typename T>
inline float ldpad(const T* img, int64_t H, int64_t W, int64_t y, int64_t x) {
    return (y < 0 || y >= H || x < 0 || x >= W) ? 0.f : to_f(img[y * W + x]);
}
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
// raw buffer loads: an access past num_records reads 0 (the gfx950 range check)
struct EmuRsrc {
    const char* base;
    uint32_t n;
};
inline EmuRsrc make_rsrc(const void* base, uint32_t bytes) { return EmuRsrc{(const char*)base, bytes}; }
template <typename T>
inline float ld_bufs(EmuRsrc r, uint32_t off, uint32_t so) {
    const uint64_t o = (uint64_t)off + so;
    if (o + sizeof(T) > r.n) return 0.f;
    T v;
    memcpy(&v, r.base + o, sizeof(T));
    return to_f(v);
}
hipError_t launch_stats(const void* cam, const void* proj, int dtype, const Geo& g, Stats sc, Stats sp, hipStream_t s,
                        int mode, float* prep, const float* shift, int rows);
}  // namespace custma
