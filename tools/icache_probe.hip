// Instruction-fetch probe: does a cold, straight-line kernel pay for its code
// size?  One workgroup (one wave) runs REPS independent VALU instructions
//   (a) straight-line (REPS * 8 bytes of code) and
//   (b) as a loop over a 64-instruction body,
// each launched alone many times; per launch the in-kernel s_memtime span and
// the HIP-event time are printed.  Equal instruction counts, so any excess of
// (a) over (b) is instruction fetch (the acquire fence at each launch leaves
// the instruction cache cold).  Also a 2-launch form to see whether a second
// launch of the same code object is warm.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/icache_probe tools/icache_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#define I1(r) asm volatile("v_add_f32_e64 %0, %0, 1.0" : "+v"(r));
#define I8 I1(a0) I1(a1) I1(a2) I1(a3) I1(a4) I1(a5) I1(a6) I1(a7)
#define I64 I8 I8 I8 I8 I8 I8 I8 I8
#define I512 I64 I64 I64 I64 I64 I64 I64 I64
#define I4096 I512 I512 I512 I512 I512 I512 I512 I512

__global__ void k_straight(float *out, unsigned long long *t)
{
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    I4096
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

__global__ void k_loop(float *out, unsigned long long *t, int iters)
{
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        I64
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) t[0] = t1 - t0;
}

int main()
{
    float *out;
    unsigned long long *t, th;
    CHK(hipMalloc(&out, 4096));
    CHK(hipMalloc(&t, 64));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int R = 40;
    for (int variant = 0; variant < 3; ++variant) {
        std::vector<double> cyc, us;
        for (int r = 0; r < R; ++r) {
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0, 0));
            if (variant == 0) hipLaunchKernelGGL(k_straight, dim3(1), dim3(64), 0, 0, out, t);
            else if (variant == 1) hipLaunchKernelGGL(k_loop, dim3(1), dim3(64), 0, 0, out, t, 64);
            else {   // straight-line twice back to back: is the second launch warm?
                hipLaunchKernelGGL(k_straight, dim3(1), dim3(64), 0, 0, out, t);
                hipLaunchKernelGGL(k_straight, dim3(1), dim3(64), 0, 0, out, t);
            }
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(&th, t, 8, hipMemcpyDeviceToHost));
            if (r >= 4) { cyc.push_back((double)th); us.push_back(ms * 1e3); }
        }
        std::sort(cyc.begin(), cyc.end());
        std::sort(us.begin(), us.end());
        const char *nm[] = {"straight 4096 (32 KB code)", "loop 64x64 (0.5 KB body)", "straight x2 launches (last span)"};
        printf("{\"variant\": \"%s\", \"span_cycles_p50\": %.0f, \"span_cycles_min\": %.0f, \"event_us_p50\": %.2f, \"event_us_min\": %.2f}\n",
               nm[variant], cyc[cyc.size() / 2], cyc[0], us[us.size() / 2], us[0]);
    }
    return 0;
}
