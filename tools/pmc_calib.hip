// pmc_calib.hip — known-byte kernels to calibrate rocprofv3 FETCH_SIZE /
// WRITE_SIZE on gfx950 for the access widths the magnifier's kernels use
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a 16-B/lane stream;
// other widths are uncalibrated).  Each kernel streams 512 MiB once.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T>
__global__ void rd(const T *__restrict__ a, size_t n, float *sink)
{
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        acc += reinterpret_cast<const float *>(&v)[0];
    }
    if (acc == 12345.678f) sink[0] = acc;
}

template <typename T>
__global__ void wr(T *__restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        memset(&v, 0, sizeof(T));
        a[i] = v;
    }
}

int main()
{
    const size_t bytes = 512ull << 20;
    char *buf;
    float *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const dim3 g(4096), b(256);
    hipLaunchKernelGGL(rd<float>, g, b, 0, 0, (const float *)buf, bytes / 4, sink);
    hipLaunchKernelGGL(rd<float2>, g, b, 0, 0, (const float2 *)buf, bytes / 8, sink);
    hipLaunchKernelGGL(rd<float4>, g, b, 0, 0, (const float4 *)buf, bytes / 16, sink);
    hipLaunchKernelGGL(wr<float>, g, b, 0, 0, (float *)buf, bytes / 4);
    hipLaunchKernelGGL(wr<float2>, g, b, 0, 0, (float2 *)buf, bytes / 8);
    hipLaunchKernelGGL(wr<float4>, g, b, 0, 0, (float4 *)buf, bytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("pmc_calib: 6 kernels x %zu bytes\n", bytes);
    (void)hipFree(buf);
    (void)hipFree(sink);
    return 0;
}
