/*
 * mm_cli.c — C host driver over the C-ABI (include/mm.h).
 *
 * Plays the role of the Unity camera that calls OnRenderImage once per frame
 * (Assets/Scripts/MotionMagnificationProcessor.cs:101): it generates a
 * synthetic RGBA8 stream on the device, or reads a clip, runs
 * the magnifier over it and reports throughput.
 *
 *   mm_cli [-w W] [-h H] [-n frames] [-l levels] [-s phase_scale]
 *          [-b frames_per_call] [-i in.{rgba,y4m}] [-o out.{rgba,y4m}] [-d device]
 *          [--full-range] [--srgb] [--standard] [--show-magnitude] [--show-phase]
 *          [--orientations O] [--iir] [--halo K]
 *          [--checksum] [--ring-world G --ring-rank R --ring-id FILE]
 *          [--ring-local G [--compare]]
 *
 * --orientations O (4/6/8): MM_MODE_STEERABLE extension,
 * DIFF temporal filter, or IIR with --iir.  A sharded IIR stream warms each
 * rank's filter on the halo of frames before its chunk (mm_ring_step_halo;
 * --halo K overrides mm_ring_halo_frames()).  --compare (with --ring-local):
 * the single-handle stream afterwards, frame by frame against the ring's
 * outputs ("cmp t maxabs ndiff" lines and a summary).
 *
 * --ring-*: frame-sharded synthetic stream over an RCCL ring (include/mm_ring.h,
 * SURVEY.md §8e), one process per GPU: rank R of G processes chunks of -b
 * frames, the ring carries the chunk-boundary state; rank 0 writes the ring id
 * to FILE, the others read it.  --checksum prints "frame <t> <byte sum>" per
 * output frame (global frame index t), so a sharded run can be compared with
 * the single-process stream.
 *
 * --ring-local G: the same frame-sharded stream at world G inside ONE process
 * on one device, one thread (and one mm_handle) per rank, through the ring's
 * test-only local transport (host/mm_ring_local.h): the product's mm_ring_step
 * logic at world > 1 on a one-GPU box.  Checksums are printed in global frame
 * order after every rank has finished.
 *
 * .y4m input: 8-bit 4:2:0 / 4:4:4 / mono YUV4MPEG2, geometry from its header
 * (host/y4m.h, BT.601 limited range unless --full-range); .y4m output is 4:4:4
 * at the input's frame rate.  Any other extension is raw RGBA8 (-w/-h).
 * --srgb: the 8-bit frames are sRGB-encoded (video and display-referred
 * clips are), processed in linear light as Unity's Linear colour space does
 * (MM_RGBA8_SRGB: decoded on read, encoded on write); default UNORM.
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mm.h"
#include "mm_ring.h"
#include "mm_ring_local.h"
#include "y4m.h"

#include <pthread.h>
#include <stdint.h>

#include <time.h>
#include <unistd.h>

/* frame format of every 8-bit frame this driver moves (--srgb) */
static int g_fmt = MM_RGBA8;

#define CHECK(x)                                                                      \
    do {                                                                              \
        int rc_ = (x);                                                                \
        if (rc_ != MM_OK) {                                                           \
            fprintf(stderr, "%s failed: %s (%d)\n", #x, mm_strerror(rc_), rc_);       \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

static int ends_with(const char *s, const char *suf)
{
    const size_t n = strlen(s), m = strlen(suf);
    return n >= m && strcmp(s + n - m, suf) == 0;
}

/* 64-bit FNV-1a over the frame's 8-byte words (any changed byte, and any
 * moved word, changes it; a byte sum would miss permutations) */
static uint64_t frame_hash(const unsigned char *p, size_t fb)
{
    uint64_t h = 0xcbf29ce484222325ull;
    size_t i = 0;
    for (; i + 8 <= fb; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
    }
    for (; i < fb; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

/* hashes of n device frames, one frame copied to the host at a time */
static int hash_frames(const unsigned char *dev, size_t fb, int n, uint64_t *out)
{
    unsigned char *h = (unsigned char *)malloc(fb);
    if (!h) return 1;
    for (int k = 0; k < n; ++k) {
        if (hipMemcpy(h, dev + fb * (size_t)k, fb, hipMemcpyDeviceToHost) != hipSuccess) {
            free(h);
            return 1;
        }
        out[k] = frame_hash(h, fb);
    }
    free(h);
    return 0;
}

static void print_checksums(const unsigned char *dev, size_t fb, int n, int t0)
{
    uint64_t *hs = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
    if (hs && !hash_frames(dev, fb, n, hs))
        for (int k = 0; k < n; ++k) printf("frame %d %llu\n", t0 + k, (unsigned long long)hs[k]);
    free(hs);
}

/* Ring id out of band: rank 0 writes FILE (atomically), the others wait for it. */
static int ring_id(int rank, const char *path, unsigned char id[MM_RING_ID_BYTES])
{
    if (rank == 0) {
        if (mm_ring_get_id(id)) return 1;
        char tmp[4096];
        snprintf(tmp, sizeof tmp, "%s.tmp", path);
        FILE *f = fopen(tmp, "wb");
        if (!f || fwrite(id, 1, MM_RING_ID_BYTES, f) != MM_RING_ID_BYTES) return 1;
        fclose(f);
        return rename(tmp, path) != 0;
    }
    for (int tries = 0; tries < 1200; ++tries) {   /* 60 s */
        FILE *f = fopen(path, "rb");
        if (f) {
            const size_t got = fread(id, 1, MM_RING_ID_BYTES, f);
            fclose(f);
            if (got == MM_RING_ID_BYTES) return 0;
        }
        struct timespec ts = {0, 50 * 1000 * 1000};
        nanosleep(&ts, NULL);
    }
    return 1;
}

/* Frame-sharded synthetic stream: rank R of G owns frames
 * [s*G*B + R*B, s*G*B + (R+1)*B) of step s. */
static int run_ring(mm_handle *h, int W, int H, int F, int B, int dev, int world, int rank,
                    const char *id_path, int checksum, int halo)
{
    unsigned char id[MM_RING_ID_BYTES];
    if (ring_id(rank, id_path, id)) {
        fprintf(stderr, "ring id exchange through %s failed\n", id_path);
        return 1;
    }
    mm_ring *r = NULL;
    int rc = mm_ring_create(world, rank, id, dev, h, W, H, B, g_fmt, &r);
    if (rc) {
        fprintf(stderr, "mm_ring_create: %s (%s)\n", mm_strerror(rc), mm_ring_last_error());
        return 1;
    }
    const size_t fb = (size_t)W * H * 4;
    void *d_in = NULL, *d_out = NULL, *d_next = NULL, *d_halo = NULL;
    int K = 0;
    if (mm_ring_halo_frames(r, &K)) return 1;
    if (halo >= 0 && K > 0) K = halo;
    if (hipMalloc(&d_in, fb * B) != hipSuccess || hipMalloc(&d_out, fb * B) != hipSuccess ||
        hipMalloc(&d_next, fb) != hipSuccess || (K > 0 && hipMalloc(&d_halo, fb * K) != hipSuccess)) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    hipStream_t s = (hipStream_t)mm_stream(h);
    const int steps = F / (world * B);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    double t_proc = 0.0;
    for (int st = 0; st < steps; ++st) {
        const int t0 = st * world * B + rank * B;
        CHECK(mm_synth_frames(d_in, W, H, t0, B, 0x5EED0000ull, 0, s));
        const int last = st + 1 < steps;
        if (last) CHECK(mm_synth_frames(d_next, W, H, t0 + world * B + B - 1, 1, 0x5EED0000ull, 0, s));
        const int hk = t0 < K ? t0 : K;   /* IIR: the warm-up halo before the chunk */
        if (hk) CHECK(mm_synth_frames(d_halo, W, H, t0 - hk, hk, 0x5EED0000ull, 0, s));
        hipEventRecord(e0, s);
        rc = K > 0 ? mm_ring_step_halo(r, st, d_halo, hk, d_in, d_out, s)
                   : mm_ring_step(r, st, d_in, d_out, last ? d_next : NULL, s);
        if (rc) {
            fprintf(stderr, "mm_ring_step: %s (%s)\n", mm_strerror(rc), mm_ring_last_error());
            return 1;
        }
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        if (st > 0) t_proc += ms * 1e-3;
        if (checksum) print_checksums((const unsigned char *)d_out, fb, B, t0);
    }
    if (steps > 1 && t_proc > 0)
        printf("rank %d/%d  steps %d  frames/s per rank %.1f\n", rank, world, steps,
               (steps - 1) * B / t_proc);
    mm_ring_destroy(r);
    hipFree(d_in);
    hipFree(d_out);
    hipFree(d_next);
    hipFree(d_halo);
    return 0;
}

/* --ring-local: rank threads of one process on one device (test-only transport) */
typedef struct {
    mm_ring_hub *hub;
    const mm_params *p;
    int W, H, F, B, dev, world, rank, checksum, halo;
    uint64_t *hashes;   /* [F], global frame index */
    unsigned char *d_all;   /* --compare: every output frame, global index (device) */
    int rc;
    char err[256];
} local_rank;

static void *local_rank_main(void *arg)
{
    local_rank *a = (local_rank *)arg;
    mm_handle *h = NULL;
    mm_ring *r = NULL;
    void *d_in = NULL, *d_out = NULL, *d_next = NULL;
    const size_t fb = (size_t)a->W * a->H * 4;
    const int steps = a->F / (a->world * a->B);
    int rc;
    a->rc = 1;
    if (hipSetDevice(a->dev) != hipSuccess) { snprintf(a->err, sizeof a->err, "hipSetDevice"); return NULL; }
    if ((rc = mm_create(a->W, a->H, a->p, a->dev, &h)) || (rc = mm_set_batch(h, a->B)) ||
        (rc = mm_ring_create_local(a->hub, a->rank, a->dev, h, a->W, a->H, a->B, g_fmt, &r))) {
        snprintf(a->err, sizeof a->err, "setup: %s (%s)", mm_strerror(rc), mm_ring_last_error());
        /* a rank that cannot join would leave the others at the hub's
         * barrier: report and stop the process */
        fprintf(stderr, "rank %d: %s\n", a->rank, a->err);
        exit(1);
    }
    int K = 0;
    void *d_halo = NULL;
    if (mm_ring_halo_frames(r, &K)) exit(1);
    if (a->halo >= 0 && K > 0) K = a->halo;
    if (hipMalloc(&d_in, fb * a->B) != hipSuccess || hipMalloc(&d_out, fb * a->B) != hipSuccess ||
        hipMalloc(&d_next, fb) != hipSuccess || (K > 0 && hipMalloc(&d_halo, fb * K) != hipSuccess)) {
        fprintf(stderr, "rank %d: hipMalloc failed\n", a->rank);
        exit(1);
    }
    hipStream_t s = (hipStream_t)mm_stream(h);
    for (int st = 0; st < steps; ++st) {
        const int t0 = st * a->world * a->B + a->rank * a->B;
        const int more = st + 1 < steps;
        if ((rc = mm_synth_frames(d_in, a->W, a->H, t0, a->B, 0x5EED0000ull, 0, s)) ||
            (more && (rc = mm_synth_frames(d_next, a->W, a->H, t0 + a->world * a->B + a->B - 1, 1,
                                           0x5EED0000ull, 0, s)))) {
            fprintf(stderr, "rank %d: mm_synth_frames: %s\n", a->rank, mm_strerror(rc));
            exit(1);
        }
        const int hk = t0 < K ? t0 : K;   /* IIR: the warm-up halo before the chunk */
        if (hk && (rc = mm_synth_frames(d_halo, a->W, a->H, t0 - hk, hk, 0x5EED0000ull, 0, s))) exit(1);
        if ((rc = K > 0 ? mm_ring_step_halo(r, st, d_halo, hk, d_in, d_out, s)
                        : mm_ring_step(r, st, d_in, d_out, more ? d_next : NULL, s))) {
            fprintf(stderr, "rank %d: mm_ring_step: %s (%s)\n", a->rank, mm_strerror(rc), mm_ring_last_error());
            exit(1);
        }
        if (a->d_all && hipMemcpyAsync(a->d_all + fb * (size_t)t0, d_out, fb * a->B, hipMemcpyDeviceToDevice, s) !=
                            hipSuccess) {
            fprintf(stderr, "rank %d: keep outputs\n", a->rank);
            exit(1);
        }
        if (a->checksum) {
            if (hipStreamSynchronize(s) != hipSuccess ||
                hash_frames((const unsigned char *)d_out, fb, a->B, a->hashes + t0)) {
                fprintf(stderr, "rank %d: readback failed\n", a->rank);
                exit(1);
            }
        }
    }
    if (hipStreamSynchronize(s) != hipSuccess) { fprintf(stderr, "rank %d: stream\n", a->rank); exit(1); }
    mm_ring_destroy(r);
    mm_destroy(h);
    hipFree(d_in);
    hipFree(d_out);
    hipFree(d_next);
    hipFree(d_halo);
    a->rc = 0;
    return NULL;
}

/* --compare: the same stream through one handle in calls of B frames, frame
 * by frame against the ring's outputs: "cmp t maxabs ndiff" per frame and a
 * summary line (the IIR halo's tolerance, tests/test_ring_c.py) */
static int compare_single(const mm_params *p, int W, int H, int F, int B, int dev, const unsigned char *d_all)
{
    const size_t fb = (size_t)W * H * 4;
    mm_handle *h = NULL;
    void *d_in = NULL, *d_out = NULL;
    unsigned char *a = (unsigned char *)malloc(fb), *b = (unsigned char *)malloc(fb);
    if (!a || !b) return 1;
    CHECK(mm_create(W, H, p, dev, &h));
    CHECK(mm_set_batch(h, B));
    if (hipMalloc(&d_in, fb * B) != hipSuccess || hipMalloc(&d_out, fb * B) != hipSuccess) return 1;
    hipStream_t s = (hipStream_t)mm_stream(h);
    long long ndiff_all = 0;
    int max_all = 0;
    for (int f0 = 0; f0 < F; f0 += B) {
        CHECK(mm_synth_frames(d_in, W, H, f0, B, 0x5EED0000ull, 0, s));
        CHECK(mm_process_stream(h, d_in, d_out, B, g_fmt, s));
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        for (int k = 0; k < B; ++k) {
            if (hipMemcpy(a, (unsigned char *)d_out + fb * k, fb, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(b, d_all + fb * (size_t)(f0 + k), fb, hipMemcpyDeviceToHost) != hipSuccess)
                return 1;
            int mx = 0;
            long long nd = 0;
            for (size_t i = 0; i < fb; ++i) {
                const int d = a[i] > b[i] ? a[i] - b[i] : b[i] - a[i];
                if (d) {
                    ++nd;
                    if (d > mx) mx = d;
                }
            }
            printf("cmp %d %d %lld\n", f0 + k, mx, nd);
            ndiff_all += nd;
            if (mx > max_all) max_all = mx;
        }
    }
    printf("compare frames %d maxabs %d ndiff %lld values %lld\n", F, max_all, ndiff_all, (long long)fb * F);
    mm_destroy(h);
    hipFree(d_in);
    hipFree(d_out);
    free(a);
    free(b);
    return 0;
}

static int run_ring_local(const mm_params *p, int W, int H, int F, int B, int dev, int world, int checksum,
                          int halo, int compare)
{
    if (world < 1 || world > 64 || F % (world * B) != 0) {
        fprintf(stderr, "--ring-local: need 1 <= G <= 64 and frames a multiple of G * batch\n");
        return 2;
    }
    mm_ring_hub *hub = NULL;
    if (mm_ring_hub_create(world, &hub)) return 1;
    uint64_t *hashes = (uint64_t *)calloc((size_t)F, sizeof(uint64_t));
    local_rank *ranks = (local_rank *)calloc((size_t)world, sizeof(local_rank));
    pthread_t *th = (pthread_t *)calloc((size_t)world, sizeof(pthread_t));
    if (!hashes || !ranks || !th) return 1;
    unsigned char *d_all = NULL;
    if (compare) {
        if (hipSetDevice(dev) != hipSuccess || hipMalloc((void **)&d_all, (size_t)W * H * 4 * (size_t)F) != hipSuccess) {
            fprintf(stderr, "--compare: hipMalloc of %d frames failed\n", F);
            return 1;
        }
    }
    for (int g = 0; g < world; ++g) {
        local_rank *a = &ranks[g];
        a->hub = hub;
        a->p = p;
        a->W = W; a->H = H; a->F = F; a->B = B; a->dev = dev;
        a->world = world; a->rank = g; a->checksum = checksum;
        a->hashes = hashes;
        a->halo = halo;
        a->d_all = d_all;
        if (pthread_create(&th[g], NULL, local_rank_main, a) != 0) {
            fprintf(stderr, "pthread_create failed\n");
            exit(1);
        }
    }
    int rc = 0;
    for (int g = 0; g < world; ++g) {
        pthread_join(th[g], NULL);
        rc |= ranks[g].rc;
    }
    if (!rc && checksum)
        for (int t = 0; t < F; ++t) printf("frame %d %llu\n", t, (unsigned long long)hashes[t]);
    printf("ring-local world %d  steps %d  chunk %d\n", world, F / (world * B), B);
    if (!rc && compare) rc = compare_single(p, W, H, F, B, dev, d_all);
    if (d_all) hipFree(d_all);
    mm_ring_hub_destroy(hub);
    free(hashes);
    free(ranks);
    free(th);
    return rc;
}

int main(int argc, char **argv)
{
    int W = 1920, H = 1080, F = 300, L = 5, B = 30, dev = 0;
    int full_range = 0, standard = 0, show_mag = 0, show_phase = 0, checksum = 0;
    int ring_world = 0, ring_rank = 0, ring_local = 0, orientations = 1, iir = 0, halo = -1, compare = 0;
    float S = 25.0f;
    const char *in_path = NULL, *out_path = NULL, *ring_id_path = NULL;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        if (!strcmp(a, "--full-range")) { full_range = 1; continue; }
        if (!strcmp(a, "--srgb")) { g_fmt = MM_RGBA8_SRGB; continue; }
        if (!strcmp(a, "--standard")) { standard = 1; continue; }
        if (!strcmp(a, "--show-magnitude")) { show_mag = 1; continue; }
        if (!strcmp(a, "--show-phase")) { show_phase = 1; continue; }
        if (!strcmp(a, "--checksum")) { checksum = 1; continue; }
        if (!strcmp(a, "--iir")) { iir = 1; continue; }
        if (!strcmp(a, "--compare")) { compare = 1; continue; }
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!v) { fprintf(stderr, "missing value for %s\n", a); return 2; }
        if (!strcmp(a, "-w")) W = atoi(v);
        else if (!strcmp(a, "-h")) H = atoi(v);
        else if (!strcmp(a, "-n")) F = atoi(v);
        else if (!strcmp(a, "-l")) L = atoi(v);
        else if (!strcmp(a, "-s")) S = (float)atof(v);
        else if (!strcmp(a, "-b")) B = atoi(v);
        else if (!strcmp(a, "-d")) dev = atoi(v);
        else if (!strcmp(a, "-i")) in_path = v;
        else if (!strcmp(a, "-o")) out_path = v;
        else if (!strcmp(a, "--ring-world")) ring_world = atoi(v);
        else if (!strcmp(a, "--ring-rank")) ring_rank = atoi(v);
        else if (!strcmp(a, "--ring-id")) ring_id_path = v;
        else if (!strcmp(a, "--ring-local")) ring_local = atoi(v);
        else if (!strcmp(a, "--orientations")) orientations = atoi(v);
        else if (!strcmp(a, "--halo")) halo = atoi(v);
        else { fprintf(stderr, "unknown option %s\n", a); return 2; }
        ++i;
    }
    if (B < 1) B = 1;
    FILE *fi = in_path ? fopen(in_path, "rb") : NULL;
    FILE *fo = out_path ? fopen(out_path, "wb") : NULL;
    if ((in_path && !fi) || (out_path && !fo)) { fprintf(stderr, "cannot open file\n"); return 1; }
    const int y4m_in = in_path && ends_with(in_path, ".y4m");
    const int y4m_out = out_path && ends_with(out_path, ".y4m");
    y4m_info yi = {0};
    yi.fps_num = 25;
    yi.fps_den = 1;
    if (y4m_in) {
        if (y4m_read_header(fi, &yi)) { fprintf(stderr, "%s: unsupported Y4M\n", in_path); return 1; }
        W = yi.width;
        H = yi.height;
    }
    mm_params p;
    mm_params_default(&p);
    p.levels = L;
    p.phase_scale = S;
    p.mode = standard ? MM_MODE_STANDARD : orientations > 1 ? MM_MODE_STEERABLE : MM_MODE_PYRAMID;
    p.orientations = orientations;
    p.temporal_filter = iir ? MM_FILTER_IIR : MM_FILTER_DIFF;
    p.show_magnitude = show_mag;
    p.show_phase = show_phase;
    if (ring_local > 0) {
        if (fi || fo) {
            fprintf(stderr, "--ring-local needs a synthetic stream\n");
            return 2;
        }
        return run_ring_local(&p, W, H, F, B, dev, ring_local, checksum, halo, compare);
    }
    /* mm_create runs on `dev` and gives the caller's current device back:
     * this program's own buffers, events and default stream must be on `dev`
     * too (before its first HIP allocation) */
    if (hipSetDevice(dev) != hipSuccess) {
        fprintf(stderr, "hipSetDevice(%d) failed\n", dev);
        return 1;
    }
    mm_handle *h = NULL;
    CHECK(mm_create(W, H, &p, dev, &h));
    int N = 0;
    mm_padded_size(h, &N);
    printf("Original: %dx%d, Padded: %dx%d\n", W, H, N, N);   /* .cs:304 */
    if (ring_world > 0) {
        if (!ring_id_path || fi || fo) {
            fprintf(stderr, "--ring-world needs --ring-id and a synthetic stream\n");
            return 2;
        }
        CHECK(mm_set_batch(h, B));
        const int rc = run_ring(h, W, H, F, B, dev, ring_world, ring_rank, ring_id_path, checksum, halo);
        mm_destroy(h);
        return rc;
    }

    const size_t fb = (size_t)W * H * 4;
    void *d_in = NULL, *d_out = NULL;
    if (hipMalloc(&d_in, fb * B) != hipSuccess || hipMalloc(&d_out, fb * B) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    hipStream_t s = (hipStream_t)mm_stream(h);
    unsigned char *host = (fi || fo) ? (unsigned char *)malloc(fb * B) : NULL;
    unsigned char *planes = (y4m_in || y4m_out)
        ? (unsigned char *)malloc(y4m_in ? (y4m_frame_bytes(&yi) > 3 * (size_t)W * H
                                               ? y4m_frame_bytes(&yi) : 3 * (size_t)W * H)
                                         : 3 * (size_t)W * H)
        : NULL;
    if (y4m_out && y4m_write_header(fo, W, H, yi.fps_num, yi.fps_den)) {
        fprintf(stderr, "write failed\n");
        return 1;
    }

    double t_proc = 0.0;
    int done = 0;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    while (done < F) {
        int n = F - done < B ? F - done : B;
        if (fi && y4m_in) {
            int got = 0;
            for (; got < n; ++got) {
                const int r = y4m_read_frame(fi, &yi, planes);
                if (r < 0) { fprintf(stderr, "%s: malformed frame\n", in_path); return 1; }
                if (r == 0) break;
                y4m_to_rgba(&yi, planes, host + fb * got, full_range);
            }
            if (got == 0) break;
            n = got;
            hipMemcpyAsync(d_in, host, fb * n, hipMemcpyHostToDevice, s);
        } else if (fi) {
            size_t got = fread(host, fb, (size_t)n, fi);
            if (got == 0) break;
            n = (int)got;
            hipMemcpyAsync(d_in, host, fb * n, hipMemcpyHostToDevice, s);
        } else {
            CHECK(mm_synth_frames(d_in, W, H, done, n, 0x5EED0000ull, 0, s));
        }
        hipEventRecord(e0, s);
        CHECK(mm_process_stream(h, d_in, d_out, n, g_fmt, s));
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        if (done > 0) t_proc += ms * 1e-3;      /* first call holds the passthrough frame */
        if (checksum) print_checksums((const unsigned char *)d_out, fb, n, done);
        if (fo) {
            hipMemcpy(host, d_out, fb * n, hipMemcpyDeviceToHost);
            if (y4m_out) {
                for (int k = 0; k < n; ++k) {
                    y4m_from_rgba(W, H, host + fb * k, planes, full_range);
                    if (y4m_write_frame(fo, W, H, planes)) { fprintf(stderr, "write failed\n"); return 1; }
                }
            } else {
                fwrite(host, fb, (size_t)n, fo);
            }
        }
        done += n;
    }
    int timed = done - (done > B ? B : done);
    if (timed > 0 && t_proc > 0)
        printf("frames %d  magnified fps %.1f  (%.3f ms/frame, %d frames per call)\n", done,
               timed / t_proc, 1e3 * t_proc / timed, B);
    else
        printf("frames %d\n", done);
    if (fi) fclose(fi);
    if (fo) fclose(fo);
    free(host);
    free(planes);
    hipFree(d_in);
    hipFree(d_out);
    mm_destroy(h);
    return 0;
}
