// Does the raw-buffer range check include soffset?  Loads one dword per lane with
// voffset = 4*lane and a uniform soffset, from a 256-byte descriptor over a 1 KiB buffer.
// If soffset counts, soffset = 256 returns zeros; if not, it returns buf[64 + lane].
#include <cstdio>
#include <vector>
#include "../../custereomatching_amd/csrc/common.h"

__global__ void k(const float* buf, float* out, unsigned so) {
    const auto r = custma::make_rsrc(buf, 256u);
    out[threadIdx.x] = custma::ld_bufs<float>(r, threadIdx.x * 4u, so);
}

int main() {
    std::vector<float> h(256);
    for (int i = 0; i < 256; ++i) h[i] = (float)(i + 1);
    float *d, *o;
    (void)hipMalloc(&d, 1024);
    (void)hipMalloc(&o, 256);
    (void)hipMemcpy(d, h.data(), 1024, hipMemcpyHostToDevice);
    for (unsigned so : {0u, 128u, 256u}) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, so);
        std::vector<float> r(64);
        (void)hipMemcpy(r.data(), o, 256, hipMemcpyDeviceToHost);
        printf("soffset %3u: lane0 %5.0f lane31 %5.0f lane32 %5.0f lane63 %5.0f\n", so, r[0], r[31], r[32], r[63]);
    }
    return 0;
}
