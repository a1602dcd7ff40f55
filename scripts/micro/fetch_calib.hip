// FETCH_SIZE / WRITE_SIZE calibration for this repo's access shapes: stream N bytes with
// (a) one dword per lane (256 B per wave-instruction, the sweep kernels' loads) and
// (b) 16 B per lane; write N bytes with one dword per lane.  Run under rocprofv3 --pmc.
#include <cstdio>
#include <hip/hip_runtime.h>

__global__ void rd1(const float* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 1234.5f) out[0] = s;
}
__global__ void rd4(const float4* __restrict__ a, size_t n4, float* out) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void wr1(float* __restrict__ a, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.f;
}

int main() {
    const size_t bytes = (size_t)1 << 30, n = bytes / 4;
    float *a, *o;
    (void)hipMalloc(&a, bytes);
    (void)hipMalloc(&o, 64);
    (void)hipMemset(a, 0, bytes);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(rd1, dim3(8192), dim3(256), 0, 0, a, n, o);
        hipLaunchKernelGGL(rd4, dim3(8192), dim3(256), 0, 0, (const float4*)a, n / 4, o);
        hipLaunchKernelGGL(wr1, dim3(8192), dim3(256), 0, 0, a, n);
    }
    (void)hipDeviceSynchronize();
    printf("streamed %zu bytes per kernel\n", bytes);
    return 0;
}
