// Unit test of the cross-lane helpers (xlane.h) on the GPU: prints, for each lane,
// the reduce48 result and the value index it should hold, plus a shl1_add check.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/micro/xlane_test.hip -o scripts/micro/xlane_test
#include <cstdio>
#include <vector>
#include "../../custereomatching_amd/csrc/xlane.h"

using namespace custma;

__global__ void k(float* out, float* out2) {
    const int lane = threadIdx.x;
    float v[48];
#pragma unroll
    for (int q = 0; q < 48; ++q) v[q] = (float)(q * 1000 + lane);  // sum over lanes = 64000 q + 2016
    out[lane] = reduce48(v, lane);
    float acc = (float)(lane * 10);
    out2[lane] = shl1_add(acc, 1.0f);  // expect lane l: 10 (l+1) + 1, lane 63: 1
}

int main() {
    float *d, *d2;
    hipMalloc(&d, 256); hipMalloc(&d2, 256);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, d2);
    std::vector<float> h(64), h2(64);
    hipMemcpy(h.data(), d, 256, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), d2, 256, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        const int q = bitrev6(l);
        const double want = 64000.0 * q + 2016.0;
        const double qgot = (h[l] - 2016.0) / 64000.0;
        if (q < 48 && h[l] != want) ++bad;
        printf("lane %2d q %2d got %10.1f (q=%.3f)  shl1 %6.1f\n", l, q, h[l], qgot, h2[l]);
    }
    printf("reduce48 bad lanes: %d\n", bad);
    return 0;
}
