// cvtpk_probe.hip — rounding and range of v_cvt_pk_u8_f32 on gfx950
// (DESIGN.md §6 "RGBA8 pack"): one wave converts a list of floats into byte 1
// of 0xff000000 and the host prints input -> byte.
//   cvtpk_probe -> one JSON line
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

__global__ void k_probe(const float *in, unsigned *out, int n)
{
    const int i = threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_cvt_pk_u8_f32(in[i], 1u, 0xff000000u);
}

int main()
{
    const float h[] = {-1.0f, -0.6f, -0.5f, -0.4f, 0.0f, 0.4f, 0.5f, 0.6f, 1.5f, 2.5f, 3.5f,
                       127.5f, 128.5f, 254.4f, 254.5f, 254.6f, 255.0f, 255.4f, 255.6f, 256.0f,
                       300.0f, 1e9f, -1e9f, INFINITY, -INFINITY, NAN};
    const int n = sizeof(h) / sizeof(h[0]);
    float *din;
    unsigned *dout;
    unsigned out[64];
    if (hipMalloc(&din, sizeof(h)) != hipSuccess || hipMalloc(&dout, 64 * sizeof(unsigned)) != hipSuccess) return 1;
    if (hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, din, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpy(out, dout, n * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("{\"probe\": \"cvt_pk_u8_f32\", \"byte1_of\": {");
    for (int i = 0; i < n; ++i)
        printf("%s\"%g\": [%u, \"0x%08x\"]", i ? ", " : "", h[i], (out[i] >> 8) & 255u, out[i]);
    printf("}}\n");
    return 0;
}
