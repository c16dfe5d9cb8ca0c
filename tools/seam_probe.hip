// seam_probe.hip — what a persistent one-frame kernel would pay per seam
// (DESIGN.md §6 "The one-frame call").
//
// The one-frame call is K1 -> K2 -> K3 -> K4: four launches whose hand-offs
// are all-to-all (every K2 column reads every K1 row, every K3 row every K2
// column), so a persistent kernel would separate its phases by grid-wide
// barriers.  This probe measures, at K2's geometry (512 workgroups of 512
// threads, two per CU, the only shape K2's 128 VGPRs and 69.6 KB of LDS allow
// co-resident), four phases that each read 16 KB written by another
// workgroup in the previous phase and write 16 KB of their own (8.4 MB per
// phase, the size of one frame's G or Q hand-off):
//   launches : four dependent launches on one stream (today's form)
//   barrier  : one launch, the phases separated by three grid barriers
//              (monotonic counter: workgroup barrier, agent release fence,
//              vmcnt drain, one relaxed agent-scope atomic add, a relaxed
//              agent-scope poll with s_sleep, agent acquire fence)
//   + the same two forms with empty phases (pure launch / barrier cost).
// Every spin is bounded: a barrier that does not complete within ~0.5 s sets
// an error flag and lets the waves run out (no hang); the grid is checked
// against the occupancy query before any launch.
//
//   seam_probe [iters]   -> one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

constexpr int kThreads = 512;
constexpr int kFloat4PerWg = 1024;   // 16 KB per workgroup and phase

// One phase: read the 16 KB workgroup (b + 37) % nb wrote in the previous
// phase, add, write this workgroup's 16 KB.
__device__ __forceinline__ void phase_body(const float4 *src, float4 *dst, int nb, int phase, float *sink)
{
    const int b = blockIdx.x;
    const int from = (b + 37) % nb;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 *s = src + (size_t)from * kFloat4PerWg;
    float4 *d = dst + (size_t)b * kFloat4PerWg;
#pragma unroll
    for (int k = 0; k < kFloat4PerWg / kThreads; ++k) {
        const float4 v = s[threadIdx.x + k * kThreads];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
#pragma unroll
    for (int k = 0; k < kFloat4PerWg / kThreads; ++k) {
        float4 o = acc;
        o.x += (float)(phase + k);
        d[threadIdx.x + k * kThreads] = o;
    }
    if (acc.x == -1.0f) *sink = acc.y;   // keeps the loads
}

__global__ __launch_bounds__(kThreads) void k_phase(const float4 *src, float4 *dst, int nb, int phase, int work,
                                                    float *sink)
{
    if (work) phase_body(src, dst, nb, phase, sink);
}

__device__ __forceinline__ void grid_barrier(unsigned *ctr, unsigned target, int *err)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 21)) {   // ~0.5 s: give up, flag it
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// Four phases in one launch; ctr counts arrivals monotonically across
// launches (base = arrivals before this launch).
__global__ __launch_bounds__(kThreads) void k_persistent(float4 *buf0, float4 *buf1, int nb, int work,
                                                         unsigned *ctr, unsigned base, int *err, float *sink)
{
    for (int p = 0; p < 4; ++p) {
        if (p > 0) grid_barrier(ctr, base + (unsigned)(p * nb), err);
        if (work) phase_body(p & 1 ? buf1 : buf0, p & 1 ? buf0 : buf1, nb, p, sink);
    }
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(&k_persistent),
                                                     kThreads, 0));
    const int cus = prop.multiProcessorCount;
    const int nb = 2 * cus;   // K2's residency: two 512-thread workgroups per CU
    if (occ < 2) {
        fprintf(stderr, "occupancy %d < 2 per CU: the grid would not be co-resident\n", occ);
        return 1;
    }
    float4 *b0, *b1;
    unsigned *ctr;
    int *err;
    float *sink;
    const size_t bytes = sizeof(float4) * kFloat4PerWg * (size_t)nb;
    CHK(hipMalloc(&b0, bytes));
    CHK(hipMalloc(&b1, bytes));
    CHK(hipMalloc(&ctr, sizeof(unsigned)));
    CHK(hipMalloc(&err, sizeof(int)));
    CHK(hipMalloc(&sink, sizeof(float)));
    CHK(hipMemset(b0, 0, bytes));
    CHK(hipMemset(b1, 0, bytes));
    CHK(hipMemset(ctr, 0, sizeof(unsigned)));
    CHK(hipMemset(err, 0, sizeof(int)));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    unsigned arrivals = 0;
    double us[2][2];   // [work][form: 0 launches, 1 barrier]
    for (int work = 0; work < 2; ++work) {
        for (int form = 0; form < 2; ++form) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CHK(hipEventRecord(e0, s));
                for (int it = 0; it < iters; ++it) {
                    if (form == 0) {
                        for (int p = 0; p < 4; ++p)
                            hipLaunchKernelGGL(k_phase, dim3(nb), dim3(kThreads), 0, s, p & 1 ? b1 : b0,
                                               p & 1 ? b0 : b1, nb, p, work, sink);
                    } else {
                        hipLaunchKernelGGL(k_persistent, dim3(nb), dim3(kThreads), 0, s, b0, b1, nb, work, ctr,
                                           arrivals, err, sink);
                        arrivals += 3u * (unsigned)nb;
                    }
                }
                CHK(hipGetLastError());
                CHK(hipEventRecord(e1, s));
                CHK(hipEventSynchronize(e1));
                float ms = 0.f;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            us[work][form] = 1e3 * best / iters;
        }
    }
    int herr = 0;
    CHK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
    printf("{\"probe\": \"seam_probe\", \"workgroups\": %d, \"threads\": %d, \"cus\": %d, "
           "\"phase_bytes\": %zu, \"iters\": %d, \"barrier_timeouts\": %d, "
           "\"us_per_call\": {\"launches_empty\": %.2f, \"barrier_empty\": %.2f, "
           "\"launches_16KB\": %.2f, \"barrier_16KB\": %.2f}, "
           "\"us_per_seam\": {\"launch_empty\": %.2f, \"barrier_empty\": %.2f, "
           "\"launch_16KB_minus_barrier_16KB\": %.2f}}\n",
           nb, kThreads, cus, bytes, iters, herr, us[0][0], us[0][1], us[1][0], us[1][1], us[0][0] / 4.0,
           (us[0][1] - us[0][0] / 4.0) / 3.0, (us[1][0] - us[1][1]) / 3.0);
    return herr ? 2 : 0;
}
