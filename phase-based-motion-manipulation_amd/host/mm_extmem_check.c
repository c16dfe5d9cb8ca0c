/*
 * mm_extmem_check.c — zero-copy frames through mm_import_frames (include/mm.h).
 *
 * Plays the engine: it allocates the input and output frame memory as HIP
 * virtual-memory allocations exportable as POSIX fds (what a Vulkan render
 * target exported with VK_KHR_external_memory_fd hands over), writes a
 * synthetic RGBA8 stream into the input through its own mapping, exports both
 * allocations, and lets the magnifier import them and work in place.  The
 * output read back through the exporter's mapping must be bitwise the output
 * of the same stream processed from ordinary device buffers.
 *
 *   mm_extmem_check [-w W] [-h H] [-n frames] [-f format]
 *                                                 -> prints "extmem ok ..." / exits 1
 * format: the mm.h code (0 RGBA8, 1 RGBA32F, 2 RGBA16F: the engine's HDR
 * target, with values up to 1.5; 3 RGBA8_SRGB): the synthetic RGBA8 stream
 * converted on the host.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mm.h"

#define HCHECK(x)                                                                       \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                                   \
        }                                                                               \
    } while (0)
#define MCHECK(x)                                                                       \
    do {                                                                                \
        int rc_ = (x);                                                                  \
        if (rc_ != MM_OK) {                                                             \
            fprintf(stderr, "%s failed: %s (%d)\n", #x, mm_strerror(rc_), rc_);         \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

typedef struct {
    hipMemGenericAllocationHandle_t h;
    void *va;
    size_t size;
    int fd;
} exported;

/* An exportable allocation mapped for the exporter, and its fd. */
static int export_alloc(size_t bytes, exported *x)
{
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof prop);
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    size_t gran = 0;
    HCHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    x->size = (bytes + gran - 1) / gran * gran;
    HCHECK(hipMemCreate(&x->h, x->size, &prop, 0));
    HCHECK(hipMemAddressReserve(&x->va, x->size, 0, NULL, 0));
    HCHECK(hipMemMap(x->va, x->size, 0, x->h, 0));
    hipMemAccessDesc acc;
    memset(&acc, 0, sizeof acc);
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    HCHECK(hipMemSetAccess(x->va, x->size, &acc, 1));
    HCHECK(hipMemExportToShareableHandle(&x->fd, x->h, hipMemHandleTypePosixFileDescriptor, 0));
    return 0;
}

/* binary16 bits of a float in [0, 65504) (round to nearest even; no
 * subnormals arise from the synthetic stream's values) */
static unsigned short half_bits(float f)
{
    unsigned x;
    memcpy(&x, &f, 4);
    if (f == 0.0f) return 0;
    unsigned h = ((((x >> 23) & 0xffu) - 127 + 15) << 10) | ((x & 0x7fffffu) >> 13);
    const unsigned rem = x & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return (unsigned short)h;
}

/* the synthetic RGBA8 stream as frames of `format` (host memory) */
static void *host_frames(int W, int H, int n, int format, size_t bytes)
{
    const size_t px = (size_t)W * H * 4 * n;
    unsigned char *u8 = (unsigned char *)malloc(px);
    void *d = NULL;
    if (!u8 || hipMalloc(&d, px) != hipSuccess) return NULL;
    if (mm_synth_frames(d, W, H, 0, n, 0x5EED0000ull, 0, NULL) != MM_OK ||
        hipMemcpy(u8, d, px, hipMemcpyDeviceToHost) != hipSuccess)
        return NULL;
    hipFree(d);
    if (format == MM_RGBA8 || format == MM_RGBA8_SRGB) return u8;
    void *out = malloc(bytes);
    if (!out) return NULL;
    for (size_t i = 0; i < px; ++i) {
        const float v = (float)u8[i] / 255.0f;
        if (format == MM_RGBA32F) ((float *)out)[i] = v;
        else ((unsigned short *)out)[i] = half_bits((i & 3) == 3 ? 1.0f : 1.5f * v);
    }
    free(u8);
    return out;
}

int main(int argc, char **argv)
{
    int W = 256, H = 144, n = 8, format = MM_RGBA8;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "-w")) W = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-h")) H = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-n")) n = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-f")) format = atoi(argv[i + 1]);
    }
    size_t fb = 0;
    MCHECK(mm_frame_bytes(W, H, format, &fb));
    const size_t bytes = fb * (size_t)n;
    HCHECK(hipSetDevice(0));
    void *src = host_frames(W, H, n, format, bytes);
    if (!src) {
        fprintf(stderr, "host frames failed\n");
        return 1;
    }
    exported xin, xout;
    if (export_alloc(bytes, &xin) || export_alloc(bytes, &xout)) return 1;
    HCHECK(hipMemcpy(xin.va, src, bytes, hipMemcpyHostToDevice));   /* the engine renders */
    HCHECK(hipMemset(xout.va, 0, xout.size));
    HCHECK(hipDeviceSynchronize());

    mm_params p;
    mm_params_default(&p);
    p.phase_scale = 25.0f;
    /* zero-copy: import both allocations, process in place */
    mm_handle *ha = NULL;
    MCHECK(mm_create(W, H, &p, 0, &ha));
    mm_ext_frames *in = NULL, *out = NULL;
    MCHECK(mm_import_frames(ha, xin.fd, xin.size, 0, &in));
    MCHECK(mm_import_frames(ha, xout.fd, xout.size, 0, &out));
    if (mm_ext_frames_ptr(in) == xin.va) {
        fprintf(stderr, "import returned the exporter's own mapping\n");
        return 1;
    }
    for (int k = 0; k < n; ++k)   /* the reference's pattern: one call per frame */
        MCHECK(mm_process(ha, (const char *)mm_ext_frames_ptr(in) + fb * k,
                          (char *)mm_ext_frames_ptr(out) + fb * k, format, MM_FRAMES_ON_DEVICE, NULL));
    HCHECK(hipDeviceSynchronize());

    /* the same stream from ordinary device buffers */
    mm_handle *hb = NULL;
    MCHECK(mm_create(W, H, &p, 0, &hb));
    void *din = NULL, *dout = NULL;
    HCHECK(hipMalloc(&din, bytes));
    HCHECK(hipMalloc(&dout, bytes));
    HCHECK(hipMemcpy(din, src, bytes, hipMemcpyHostToDevice));
    MCHECK(mm_process_stream(hb, din, dout, n, format, NULL));
    HCHECK(hipDeviceSynchronize());

    unsigned char *a = (unsigned char *)malloc(bytes), *b = (unsigned char *)malloc(bytes);
    if (!a || !b) return 1;
    HCHECK(hipMemcpy(a, xout.va, bytes, hipMemcpyDeviceToHost));   /* the exporter's view */
    HCHECK(hipMemcpy(b, dout, bytes, hipMemcpyDeviceToHost));
    size_t diff = 0;
    unsigned long long sum = 0;
    for (size_t i = 0; i < bytes; ++i) {
        diff += a[i] != b[i];
        sum += a[i];
    }
    MCHECK(mm_release_frames(in));
    MCHECK(mm_release_frames(out));
    mm_destroy(ha);
    mm_destroy(hb);
    hipFree(din);
    hipFree(dout);
    free(a);
    free(b);
    if (diff) {
        fprintf(stderr, "extmem: %zu of %zu bytes differ\n", diff, bytes);
        return 1;
    }
    free(src);
    printf("extmem ok: %dx%d x %d frames, format %d, zero-copy output == device-buffer output "
           "(byte sum %llu)\n", W, H, n, format, sum);
    return 0;
}
