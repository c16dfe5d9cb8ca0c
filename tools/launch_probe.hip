// Fixed per-launch cost of a kernel shape: back-to-back launches of an empty
// kernel (512 workgroups x 512 threads, like k_cols at N = 2048) with 0, 40 or
// 78 KB of dynamic LDS, and of a kernel that writes B bytes (whole lines,
// plain or non-temporal stores) -- HIP-event time per launch over 200 launches.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/launch_probe tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(512) void k_empty(int *flag)
{
    extern __shared__ int l[];
    if (flag[0] == 12345) { l[threadIdx.x] = 1; flag[1] = l[threadIdx.x ^ 1]; }   // never true
}

template <bool NT>
__global__ __launch_bounds__(512) void k_write(float4 *out, size_t n4)
{
    for (size_t i = (size_t)blockIdx.x * 512 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 512) {
        const float4 v = make_float4(1.0f, 2.0f, 3.0f, (float)i);
        if (NT) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4 *>(out + i));
        } else {
            out[i] = v;
        }
    }
}

int main()
{
    int *flag;
    float4 *buf;
    const size_t bytes = 8864000;   // one frame's Q at 1080p
    CHK(hipMalloc(&flag, 64));
    CHK(hipMemset(flag, 0, 64));
    CHK(hipMalloc(&buf, bytes));
    CHK(hipFuncSetAttribute((const void *)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int R = 200;
    for (int v = 0; v < 6; ++v) {
        for (int pass = 0; pass < 2; ++pass) {
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0, 0));
            for (int r = 0; r < R; ++r) {
                if (v < 3) {
                    const size_t lds = v == 0 ? 0 : v == 1 ? 40 * 1024 : 78 * 1024;
                    hipLaunchKernelGGL(k_empty, dim3(512), dim3(512), lds, 0, flag);
                } else if (v == 3) {
                    hipLaunchKernelGGL(k_write<false>, dim3(1024), dim3(512), 0, 0, buf, bytes / 16);
                } else if (v == 4) {
                    hipLaunchKernelGGL(k_write<true>, dim3(1024), dim3(512), 0, 0, buf, bytes / 16);
                } else {
                    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, flag);
                }
            }
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const char *nm[] = {"empty 512x512, LDS 0", "empty 512x512, LDS 40 KB", "empty 512x512, LDS 78 KB",
                                "write 8.86 MB (plain)", "write 8.86 MB (nt)", "empty 1x64"};
            if (pass) printf("{\"kernel\": \"%s\", \"us_per_launch\": %.2f}\n", nm[v], ms * 1e3 / R);
        }
    }
    // the same 200 empty 512x512 launches captured once into a hipGraph and
    // replayed: per-node cost of graph dispatch against stream launches
    {
        hipStream_t cs;
        CHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        hipGraph_t gr;
        hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
        for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_empty, dim3(512), dim3(512), 0, cs, flag);
        CHK(hipStreamEndCapture(cs, &gr));
        CHK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        for (int pass = 0; pass < 2; ++pass) {
            CHK(hipStreamSynchronize(cs));
            CHK(hipEventRecord(e0, cs));
            CHK(hipGraphLaunch(ge, cs));
            CHK(hipEventRecord(e1, cs));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (pass) printf("{\"kernel\": \"graph of 200 empty 512x512\", \"us_per_launch\": %.2f}\n", ms * 1e3 / R);
        }
    }
    return 0;
}
