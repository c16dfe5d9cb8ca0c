// Per-call cost of a 4-kernel chain: stream launches vs one hipGraph whose
// kernel nodes get new pointer arguments every call (hipGraphExecKernelNodeSetParams)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
__global__ __launch_bounds__(256) void k_touch(const float *in, float *out, int n, int salt)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i] * 1.0001f + (float)salt;
}
int main()
{
    const int n = 1 << 20, K = 4, C = 400;
    float *buf[8];
    for (int i = 0; i < 8; ++i) { CHK(hipMalloc(&buf[i], n * 4)); CHK(hipMemset(buf[i], 0, n * 4)); }
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const dim3 g(n / 256), b(256);
    for (int pass = 0; pass < 2; ++pass) {
        CHK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        CHK(hipEventRecord(e0, s));
        for (int c = 0; c < C; ++c)
            for (int k = 0; k < K; ++k)
                hipLaunchKernelGGL(k_touch, g, b, 0, s, buf[(c + k) & 7], buf[(c + k + 1) & 7], n, c);
        auto t1 = std::chrono::steady_clock::now();
        CHK(hipEventRecord(e1, s));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        if (pass) printf("{\"mode\": \"stream\", \"gpu_us_per_call\": %.2f, \"host_us_per_call\": %.2f}\n", ms * 1e3 / C,
                         std::chrono::duration<double, std::micro>(t1 - t0).count() / C);
    }
    hipGraph_t gr; CHK(hipGraphCreate(&gr, 0));
    hipGraphNode_t nodes[K];
    const float *ain[K]; float *aout[K]; int an = n, asalt = 0;
    void *args[K][4];
    hipKernelNodeParams p[K];
    for (int k = 0; k < K; ++k) {
        ain[k] = buf[k]; aout[k] = buf[k + 1];
        args[k][0] = &ain[k]; args[k][1] = &aout[k]; args[k][2] = &an; args[k][3] = &asalt;
        p[k] = {};
        p[k].func = (void *)k_touch; p[k].gridDim = g; p[k].blockDim = b; p[k].sharedMemBytes = 0;
        p[k].kernelParams = args[k]; p[k].extra = nullptr;
        CHK(hipGraphAddKernelNode(&nodes[k], gr, k ? &nodes[k - 1] : nullptr, k ? 1 : 0, &p[k]));
    }
    hipGraphExec_t ge; CHK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    for (int pass = 0; pass < 2; ++pass) {
        CHK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        CHK(hipEventRecord(e0, s));
        for (int c = 0; c < C; ++c) {
            asalt = c;
            for (int k = 0; k < K; ++k) {
                ain[k] = buf[(c + k) & 7]; aout[k] = buf[(c + k + 1) & 7];
                CHK(hipGraphExecKernelNodeSetParams(ge, nodes[k], &p[k]));
            }
            CHK(hipGraphLaunch(ge, s));
        }
        auto t1 = std::chrono::steady_clock::now();
        CHK(hipEventRecord(e1, s));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        if (pass) printf("{\"mode\": \"graph+setparams\", \"gpu_us_per_call\": %.2f, \"host_us_per_call\": %.2f}\n", ms * 1e3 / C,
                         std::chrono::duration<double, std::micro>(t1 - t0).count() / C);
    }
    // correctness: last call's output equals a stream recomputation
    float h1, h2;
    CHK(hipStreamSynchronize(s));
    const int c = C - 1;
    CHK(hipMemcpy(&h1, buf[(c + K) & 7] + 5, 4, hipMemcpyDeviceToHost));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_touch, g, b, 0, s, buf[(c + k) & 7], buf[(c + k + 1) & 7], n, c);
    CHK(hipStreamSynchronize(s));
    CHK(hipMemcpy(&h2, buf[(c + K) & 7] + 5, 4, hipMemcpyDeviceToHost));
    printf("{\"check\": %s}\n", h1 == h2 ? "true" : "false");
    return 0;
}
