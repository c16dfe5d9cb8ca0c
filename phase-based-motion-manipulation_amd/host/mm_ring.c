/*
 * mm_ring.c — frame-sharded streaming over an RCCL ring (include/mm_ring.h).
 *
 * The C counterpart of mm355/stream.py's ShardedStream: one
 * ncclSend/ncclRecv pair per step carries the chunk-boundary temporal state
 * (mm_compute_state of the sender's last input frame) to the next rank.  The
 * shift of step s+1 is posted on the ring's own stream before step s's frames
 * are processed, so the transfer runs under step s's kernels.
 */
#define _GNU_SOURCE   /* dladdr */
#include "mm_ring.h"
#include "mm_ring_local.h"

#include <dlfcn.h>
#include <math.h>
#include <pthread.h>

#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Transport seam: how one ring shift moves the state.  The product ring uses
 * RCCL (ncclSend/ncclRecv on the ring's stream); the test-only local
 * transport (mm_ring_local.h) moves it between threads of one process that
 * share one GPU, with device copies and events, so that the multi-rank step
 * logic below runs at world > 1 on a one-GPU box (RCCL refuses two ranks on
 * one device).  shift(): enqueue on r->cs the send of st_out[k] to rank+1
 * and the receive of st_in[k] from rank-1; when r->cs passes the shift, the
 * receive has landed and the peer is done reading st_out[k]. */
typedef struct {
    int (*shift)(mm_ring *r, int k);
    void (*close)(mm_ring *r);
} ring_ops;

struct mm_ring {
    int world, rank, device, chunk, format;
    size_t frame_bytes, state_bytes;
    mm_handle *h;
    const ring_ops *ops;
    ncclComm_t comm;              /* RCCL transport */
    mm_ring_hub *hub;             /* local transport */
    hipStream_t cs;               /* the ring's stream */
    void *st_out[2], *st_in[2];   /* per posted step, slot = step & 1 */
    void *carry;                  /* rank 0: st_in of the previous step */
    int posted[2];                /* step posted in the slot, -1: none */
    int halo_mode;                /* MM_FILTER_IIR steerable: mm_ring_step_halo only */
    hipEvent_t ready[2];          /* st_out written (caller's stream) */
    hipEvent_t done[2];           /* shift finished (ring stream) */
};

static char g_err[256];

const char *mm_ring_last_error(void) { return g_err; }

static int fail_nccl(const char *what, ncclResult_t r)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, ncclGetErrorString(r));
    return MM_ERR_HIP;
}

static int fail_hip(const char *what, hipError_t e)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return MM_ERR_HIP;
}

#define NCCL_TRY(x)                                  \
    do {                                             \
        ncclResult_t r_ = (x);                       \
        if (r_ != ncclSuccess) return fail_nccl(#x, r_); \
    } while (0)
#define HIP_TRY(x)                                   \
    do {                                             \
        hipError_t e_ = (x);                         \
        if (e_ != hipSuccess) return fail_hip(#x, e_); \
    } while (0)

int mm_ring_get_id(unsigned char id[MM_RING_ID_BYTES])
{
    if (!id) return MM_ERR_INVALID;
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    memcpy(id, u.internal, MM_RING_ID_BYTES);
    return MM_OK;
}

static void release(mm_ring *r)
{
    if (!r) return;
    if (r->cs) (void)hipStreamSynchronize(r->cs);
    if (r->ops) r->ops->close(r);
    for (int k = 0; k < 2; ++k) {
        (void)hipFree(r->st_out[k]);
        (void)hipFree(r->st_in[k]);
        if (r->ready[k]) (void)hipEventDestroy(r->ready[k]);
        if (r->done[k]) (void)hipEventDestroy(r->done[k]);
    }
    (void)hipFree(r->carry);
    if (r->cs) (void)hipStreamDestroy(r->cs);
    free(r);
}

/* RCCL transport */
static int nccl_shift(mm_ring *r, int k)
{
    const int nxt = (r->rank + 1) % r->world, prv = (r->rank + r->world - 1) % r->world;
    NCCL_TRY(ncclGroupStart());
    NCCL_TRY(ncclSend(r->st_out[k], r->state_bytes, ncclUint8, nxt, r->comm, r->cs));
    NCCL_TRY(ncclRecv(r->st_in[k], r->state_bytes, ncclUint8, prv, r->comm, r->cs));
    NCCL_TRY(ncclGroupEnd());
    return MM_OK;
}

static void nccl_close(mm_ring *r)
{
    if (r->comm) (void)ncclCommDestroy(r->comm);
    r->comm = NULL;
}

static const ring_ops k_nccl_ops = {nccl_shift, nccl_close};

/* Everything but the transport: validates, allocates the state slots, the
 * ring stream and its events. */
static int ring_alloc(int world, int rank, int hip_device, mm_handle *h, int width, int height,
                      int chunk, int format, mm_ring **out)
{
    if (!out) return MM_ERR_INVALID;
    *out = NULL;
    size_t fbytes = 0;
    if (!h || world < 1 || rank < 0 || rank >= world || chunk < 1 || width < 1 || height < 1 ||
        mm_frame_bytes(width, height, format, &fbytes) != MM_OK)
        return MM_ERR_INVALID;
    mm_params p;
    int rc = mm_get_params(h, &p);
    if (rc) return rc;
    mm_ring *r = (mm_ring *)calloc(1, sizeof *r);
    if (!r) return MM_ERR_OOM;
    r->world = world;
    r->rank = rank;
    r->device = hip_device;
    r->chunk = chunk;
    r->format = format;
    r->h = h;
    r->posted[0] = r->posted[1] = -1;
    r->frame_bytes = fbytes;
    /* the IIR state is a history of frames, not one frame's function: nothing
     * is shifted, each rank warms its filter on a halo (mm_ring_step_halo) */
    r->halo_mode = p.mode == MM_MODE_STEERABLE && p.temporal_filter == MM_FILTER_IIR;
    if ((rc = mm_state_size(h, &r->state_bytes))) {
        release(r);
        return rc;
    }
    hipError_t e;
    if ((e = hipSetDevice(hip_device)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&r->cs, hipStreamNonBlocking)) != hipSuccess) {
        release(r);
        return fail_hip("ring stream", e);
    }
    for (int k = 0; k < 2 && !r->halo_mode; ++k) {
        if ((e = hipMalloc(&r->st_out[k], r->state_bytes)) != hipSuccess ||
            (e = hipMalloc(&r->st_in[k], r->state_bytes)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->ready[k], hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->done[k], hipEventDisableTiming)) != hipSuccess) {
            release(r);
            return MM_ERR_OOM;
        }
    }
    if (!r->halo_mode && (e = hipMalloc(&r->carry, r->state_bytes)) != hipSuccess) {
        release(r);
        return MM_ERR_OOM;
    }
    *out = r;
    return MM_OK;
}

int mm_ring_create(int world, int rank, const unsigned char id[MM_RING_ID_BYTES], int hip_device,
                   mm_handle *h, int width, int height, int chunk, int format, mm_ring **out)
{
    if (!out) return MM_ERR_INVALID;
    *out = NULL;
    if (!id) return MM_ERR_INVALID;
    mm_ring *r = NULL;
    int rc = ring_alloc(world, rank, hip_device, h, width, height, chunk, format, &r);
    if (rc) return rc;
    ncclUniqueId u;
    memcpy(u.internal, id, MM_RING_ID_BYTES);
    ncclResult_t nr = ncclCommInitRank(&r->comm, world, u, rank);
    if (nr != ncclSuccess) {
        r->comm = NULL;
        release(r);
        return fail_nccl("ncclCommInitRank", nr);
    }
    r->ops = &k_nccl_ops;
    *out = r;
    return MM_OK;
}

/* ---- local transport (test only: mm_ring_local.h) -------------------------
 * World ranks are threads of one process on one device.  Per shift, every
 * rank publishes st_out[k] and an event recorded on its ring stream behind
 * it; after a host barrier each rank's ring stream waits for its previous
 * rank's event and copies that rank's st_out[k] into its own st_in[k], then
 * records `copied`; after a second barrier each ring stream also waits for
 * its NEXT rank's `copied` (the receiver has read my st_out[k]: what a
 * completed ncclSend means for the sender's buffer).  The two barriers order
 * the host-side publication and every event record against the waits on it;
 * all ranks call shift() in the same order (mm_ring_step's step order), as
 * RCCL's send/receive pairs require too. */
#define MM_RING_LOCAL_MAX 64
struct mm_ring_hub {
    int world;
    pthread_barrier_t bar;
    const void *src[MM_RING_LOCAL_MAX];
    hipEvent_t posted[MM_RING_LOCAL_MAX], copied[MM_RING_LOCAL_MAX];
};

int mm_ring_hub_create(int world, mm_ring_hub **out)
{
    if (!out) return MM_ERR_INVALID;
    *out = NULL;
    if (world < 1 || world > MM_RING_LOCAL_MAX) return MM_ERR_INVALID;
    mm_ring_hub *hb = (mm_ring_hub *)calloc(1, sizeof *hb);
    if (!hb) return MM_ERR_OOM;
    hb->world = world;
    if (pthread_barrier_init(&hb->bar, NULL, (unsigned)world) != 0) {
        free(hb);
        return MM_ERR_OOM;
    }
    *out = hb;
    return MM_OK;
}

void mm_ring_hub_destroy(mm_ring_hub *hb)
{
    if (!hb) return;
    pthread_barrier_destroy(&hb->bar);
    free(hb);
}

static int local_shift(mm_ring *r, int k)
{
    mm_ring_hub *hb = r->hub;
    const int me = r->rank, nxt = (me + 1) % r->world, prv = (me + r->world - 1) % r->world;
    hb->src[me] = r->st_out[k];
    HIP_TRY(hipEventRecord(hb->posted[me], r->cs));   /* behind the wait on ready[k] */
    pthread_barrier_wait(&hb->bar);
    HIP_TRY(hipStreamWaitEvent(r->cs, hb->posted[prv], 0));
    HIP_TRY(hipMemcpyAsync(r->st_in[k], hb->src[prv], r->state_bytes, hipMemcpyDeviceToDevice, r->cs));
    HIP_TRY(hipEventRecord(hb->copied[me], r->cs));
    pthread_barrier_wait(&hb->bar);
    HIP_TRY(hipStreamWaitEvent(r->cs, hb->copied[nxt], 0));
    return MM_OK;
}

static void local_close(mm_ring *r)
{
    if (!r->hub) return;
    (void)hipEventDestroy(r->hub->posted[r->rank]);
    (void)hipEventDestroy(r->hub->copied[r->rank]);
    r->hub->posted[r->rank] = r->hub->copied[r->rank] = NULL;
    r->hub = NULL;
}

static const ring_ops k_local_ops = {local_shift, local_close};

int mm_ring_create_local(mm_ring_hub *hub, int rank, int hip_device, mm_handle *h, int width, int height,
                         int chunk, int format, mm_ring **out)
{
    if (!out) return MM_ERR_INVALID;
    *out = NULL;
    if (!hub || rank < 0 || rank >= hub->world) return MM_ERR_INVALID;
    mm_ring *r = NULL;
    int rc = ring_alloc(hub->world, rank, hip_device, h, width, height, chunk, format, &r);
    if (rc) return rc;
    hipError_t e;
    if ((e = hipEventCreateWithFlags(&hub->posted[rank], hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&hub->copied[rank], hipEventDisableTiming)) != hipSuccess) {
        /* release() closes the transport only once r->ops is set: the events
         * created so far are destroyed here */
        if (hub->posted[rank]) (void)hipEventDestroy(hub->posted[rank]);
        if (hub->copied[rank]) (void)hipEventDestroy(hub->copied[rank]);
        hub->posted[rank] = hub->copied[rank] = NULL;
        release(r);
        return fail_hip("local ring events", e);
    }
    r->hub = hub;
    r->ops = &k_local_ops;
    *out = r;
    return MM_OK;
}

/* Steps 1-2 for `step`: my last frame's state -> next rank, previous rank's -> me. */
static int exchange_begin(mm_ring *r, int step, const void *last, hipStream_t s)
{
    const int k = step & 1;
    if (r->posted[k] == step) return MM_OK;
    int rc = mm_compute_state(r->h, last, r->format, r->st_out[k], r->state_bytes, s);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(r->ready[k], s));
    HIP_TRY(hipStreamWaitEvent(r->cs, r->ready[k], 0));
    if ((rc = r->ops->shift(r, k))) return rc;
    HIP_TRY(hipEventRecord(r->done[k], r->cs));
    r->posted[k] = step;
    return MM_OK;
}

/* Step 3: wait for the shift of `step` and set the handle's state. */
static int exchange_end(mm_ring *r, int step, const void *in, hipStream_t s)
{
    const int k = step & 1;
    int rc;
    if (r->posted[k] != step) {   /* not posted ahead: post it now */
        const unsigned char *last = (const unsigned char *)in + r->frame_bytes * (size_t)(r->chunk - 1);
        if ((rc = exchange_begin(r, step, last, s))) return rc;
    }
    HIP_TRY(hipStreamWaitEvent(s, r->done[k], 0));
    if (r->rank == 0) {
        if (step == 0) rc = mm_reset(r->h);
        else rc = mm_set_state(r->h, r->carry, r->state_bytes, s);
        if (rc) return rc;
        /* the state received now is the one before my chunk of step+1; the
         * buffer handed back is only rewritten by a receive posted after this
         * stream's mm_set_state (ready[] orders it) */
        void *t = r->carry;
        r->carry = r->st_in[k];
        r->st_in[k] = t;
    } else if ((rc = mm_set_state(r->h, r->st_in[k], r->state_bytes, s))) {
        return rc;
    }
    r->posted[k] = -1;
    return MM_OK;
}

int mm_ring_step(mm_ring *r, int step, const void *in, void *out, const void *next_last,
                 void *hip_stream)
{
    if (!r || !in || !out || step < 0) return MM_ERR_INVALID;
    if (r->halo_mode) {
        snprintf(g_err, sizeof g_err, "IIR steerable handle: use mm_ring_step_halo");
        return MM_ERR_UNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)hip_stream;
    HIP_TRY(hipSetDevice(r->device));
    int rc;
    if ((rc = exchange_end(r, step, in, s))) return rc;
    if (next_last && (rc = exchange_begin(r, step + 1, next_last, s))) return rc;
    return mm_process_stream(r->h, in, out, r->chunk, r->format, s);
}

void mm_ring_destroy(mm_ring *r) { release(r); }

int mm_ring_step_halo(mm_ring *r, int step, const void *halo, int halo_frames, const void *in, void *out,
                      void *hip_stream)
{
    if (!r || !in || !out || step < 0 || halo_frames < 0 || (halo_frames > 0 && !halo))
        return MM_ERR_INVALID;
    if (!r->halo_mode) {
        snprintf(g_err, sizeof g_err, "mm_ring_step_halo is for IIR steerable handles");
        return MM_ERR_UNSUPPORTED;
    }
    hipStream_t s = (hipStream_t)hip_stream;
    HIP_TRY(hipSetDevice(r->device));
    /* a filter started from rest at the halo's first frame (which passes
     * through and seeds the local phases, as the stream's frame 0 does) */
    int rc = mm_reset(r->h);
    if (rc) return rc;
    /* the halo's outputs are discarded: `out` holds them until the chunk
     * overwrites it (at most `chunk` frames per call) */
    const unsigned char *hp = (const unsigned char *)halo;
    for (int f0 = 0; f0 < halo_frames; f0 += r->chunk) {
        const int n = halo_frames - f0 < r->chunk ? halo_frames - f0 : r->chunk;
        if ((rc = mm_process_stream(r->h, hp + r->frame_bytes * (size_t)f0, out, n, r->format, s))) return rc;
    }
    return mm_process_stream(r->h, in, out, r->chunk, r->format, s);
}

int mm_ring_halo_frames(const mm_ring *r, int *frames)
{
    if (!r || !frames) return MM_ERR_INVALID;
    if (!r->halo_mode) {
        *frames = 0;
        return MM_OK;
    }
    mm_params p;
    int rc = mm_get_params(r->h, &p);
    if (rc) return rc;
    /* the slower pole (1 - iir_low) decays below 1e-6 of its start value:
     * ceil(ln 1e-6 / ln(1 - iir_low)); 270 frames at the default 0.05 */
    const double k = ceil(log(1e-6) / log1p(-(double)p.iir_low));
    if (!(k <= MM_RING_HALO_MAX)) return MM_ERR_UNSUPPORTED;   /* iir_low below ~0.0067 */
    *frames = k < 1.0 ? 1 : (int)k;
    return MM_OK;
}

/* The libmm355 this library's mm_* calls resolve to (dladdr of the bound
 * mm_process_stream): a caller that loaded another build of the operator
 * (an A/B variant) checks that both libraries are the same one. */
const char *mm_ring_core_library(void)
{
    Dl_info info;
    if (dladdr((void *)&mm_process_stream, &info) && info.dli_fname) return info.dli_fname;
    return NULL;
}
