// valu_calib.hip — issue cost of one wave64 VALU instruction on gfx950, by
// waves per SIMD, for the instruction kinds the magnifier's kernels issue.
//
// Each kernel runs ITERS iterations of an unrolled block of independent
// instructions (8 chains per lane, no memory traffic inside the loop).  The
// in-kernel shader clock comes from s_memtime / s_memrealtime (100 MHz) of
// lane 0 of every workgroup; cycles per wave-instruction per SIMD =
// (kernel cycles x SIMDs) / (wave-instructions issued).  tools/valu_summary.py
// uses the measured figure (profiles/*_valu_calib.json) instead of a guess.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr int ITERS = 4096;
constexpr int CHAINS = 8;

struct Stamp { unsigned long long t0, t1, r0, r1; };

template <int KIND>
__global__ void valu(float *out, Stamp *st, float a, float b)
{
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    float x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = (float)(threadIdx.x + c) * 1e-3f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 xp[CHAINS];
    const f2 ap = {a, a}, bp = {b, b};
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) xp[c] = f2{x[c], x[c] + 1.0f};
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if constexpr (KIND == 0) {          // v_fma_f32
                x[c] = __builtin_fmaf(x[c], a, b);
            } else if constexpr (KIND == 1) {   // v_add_f32
                x[c] = x[c] + a;
            } else if constexpr (KIND == 2) {   // v_sin_f32 (transcendental)
                x[c] = __builtin_amdgcn_sinf(x[c]);
            } else if constexpr (KIND == 3) {   // v_pk_fma_f32 (two floats per lane)
                xp[c] = __builtin_elementwise_fma(xp[c], ap, bp);
            } else if constexpr (KIND == 4) {   // v_pk_add_f32
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(xp[c]) : "v"(bp));
            } else if constexpr (KIND == 5) {   // v_pk_mul_f32
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(xp[c]) : "v"(ap));
            } else if constexpr (KIND == 6) {   // v_pk_fma_f32 with op_sel/neg swizzles (complex multiply half)
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
                             : "+v"(xp[c]) : "v"(ap), "v"(bp));
            } else if constexpr (KIND == 7) {   // v_pk_add_f32 with op_sel swizzle (+-i rotation)
                asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
                             : "+v"(xp[c]) : "v"(bp));
            } else {                            // v_mul_f32 + v_add_f32 pair (scalar reference for 6/7)
                x[c] = x[c] * a + b;
            }
        }
        asm volatile("" ::: "memory");
    }
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c] + xp[c].x + xp[c].y;
    if (s == 1234.5f) out[0] = s;
    if (threadIdx.x == 0) {
        st[blockIdx.x].t0 = t0;
        st[blockIdx.x].r0 = r0;
        st[blockIdx.x].t1 = __builtin_amdgcn_s_memtime();
        st[blockIdx.x].r1 = __builtin_amdgcn_s_memrealtime();
    }
}

template <int KIND>
static double run(int waves_per_simd, double *clk_ghz, float *ms_out)
{
    const int cus = 256, threads = 256;             // 4 waves per workgroup = 1 per SIMD
    const int blocks = cus * waves_per_simd;
    float *out;
    Stamp *st;
    if (hipMalloc(&out, 4) != hipSuccess || hipMalloc(&st, sizeof(Stamp) * blocks) != hipSuccess) return -1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(valu<KIND>, dim3(blocks), dim3(threads), 0, 0, out, st, 1.0001f, 0.5f);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(valu<KIND>, dim3(blocks), dim3(threads), 0, 0, out, st, 1.0001f, 0.5f);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return -1;
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<Stamp> h(blocks);
    (void)hipMemcpy(h.data(), st, sizeof(Stamp) * blocks, hipMemcpyDeviceToHost);
    double c = 0.0;
    int n = 0;
    for (auto &s : h)
        if (s.r1 > s.r0) { c += (double)(s.t1 - s.t0) / (double)(s.r1 - s.r0) * 0.1; ++n; }
    *clk_ghz = n ? c / n : 0.0;
    *ms_out = ms;
    // wave-instructions in the loop: ITERS * CHAINS per wave (build with
    // -fno-slp-vectorize so kinds 0-2 stay single-float instructions)
    const double waves = (double)blocks * threads / 64;
    const double insts = waves * ITERS * CHAINS;
    (void)hipFree(out);
    (void)hipFree(st);
    return (ms * 1e-3) * (*clk_ghz * 1e9) * (cus * 4) / insts;   // cycles per wave-instruction per SIMD
}

int main()
{
    const char *names[8] = {"v_fma_f32", "v_add_f32", "v_sin_f32", "v_pk_fma_f32", "v_pk_add_f32",
                            "v_pk_mul_f32", "v_pk_fma_f32 op_sel", "v_pk_add_f32 op_sel"};
    printf("{\"iters\": %d, \"chains\": %d, \"rows\": [\n", ITERS, CHAINS);
    bool first = true;
    for (int kind = 0; kind < 8; ++kind)
        for (int w : {1, 2, 4, 8}) {
            double clk = 0;
            float ms = 0;
            double cyc = kind == 0 ? run<0>(w, &clk, &ms) : kind == 1 ? run<1>(w, &clk, &ms)
                       : kind == 2 ? run<2>(w, &clk, &ms) : kind == 3 ? run<3>(w, &clk, &ms)
                       : kind == 4 ? run<4>(w, &clk, &ms) : kind == 5 ? run<5>(w, &clk, &ms)
                       : kind == 6 ? run<6>(w, &clk, &ms) : run<7>(w, &clk, &ms);
            printf("%s {\"inst\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_GHz\": %.3f, "
                   "\"cycles_per_wave_inst\": %.3f}",
                   first ? "" : ",\n", names[kind], w, ms, clk, cyc);
            first = false;
        }
    printf("\n]}\n");
    return 0;
}
