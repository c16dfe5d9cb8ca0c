/*
 * mm_ring.c — frame-sharded streaming over an RCCL ring (include/mm_ring.h).
 *
 * The C counterpart of mm355/stream.py's ShardedStream: one
 * ncclSend/ncclRecv pair per step carries the chunk-boundary temporal state
 * (mm_compute_state of the sender's last input frame) to the next rank.  The
 * shift of step s+1 is posted on the ring's own stream before step s's frames
 * are processed, so the transfer runs under step s's kernels.
 */
#include "mm_ring.h"

#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct mm_ring {
    int world, rank, device, chunk, format;
    size_t frame_bytes, state_bytes;
    mm_handle *h;
    ncclComm_t comm;
    hipStream_t cs;               /* the ring's stream */
    void *st_out[2], *st_in[2];   /* per posted step, slot = step & 1 */
    void *carry;                  /* rank 0: st_in of the previous step */
    int posted[2];                /* step posted in the slot, -1: none */
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
    if (r->comm) (void)ncclCommDestroy(r->comm);
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

int mm_ring_create(int world, int rank, const unsigned char id[MM_RING_ID_BYTES], int hip_device,
                   mm_handle *h, int width, int height, int chunk, int format, mm_ring **out)
{
    if (!out) return MM_ERR_INVALID;
    *out = NULL;
    if (!id || !h || world < 1 || rank < 0 || rank >= world || chunk < 1 || width < 1 || height < 1 ||
        (format != MM_RGBA8 && format != MM_RGBA32F))
        return MM_ERR_INVALID;
    mm_params p;
    int rc = mm_get_params(h, &p);
    if (rc) return rc;
    if (p.mode == MM_MODE_STEERABLE && p.temporal_filter == MM_FILTER_IIR)
        return MM_ERR_UNSUPPORTED;   /* the IIR state is a history, not one frame's */
    mm_ring *r = (mm_ring *)calloc(1, sizeof *r);
    if (!r) return MM_ERR_OOM;
    r->world = world;
    r->rank = rank;
    r->device = hip_device;
    r->chunk = chunk;
    r->format = format;
    r->h = h;
    r->posted[0] = r->posted[1] = -1;
    r->frame_bytes = (size_t)width * height * (format == MM_RGBA8 ? 4 : 16);
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
    for (int k = 0; k < 2; ++k) {
        if ((e = hipMalloc(&r->st_out[k], r->state_bytes)) != hipSuccess ||
            (e = hipMalloc(&r->st_in[k], r->state_bytes)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->ready[k], hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&r->done[k], hipEventDisableTiming)) != hipSuccess) {
            release(r);
            return MM_ERR_OOM;
        }
    }
    if ((e = hipMalloc(&r->carry, r->state_bytes)) != hipSuccess) {
        release(r);
        return MM_ERR_OOM;
    }
    ncclUniqueId u;
    memcpy(u.internal, id, MM_RING_ID_BYTES);
    ncclResult_t nr = ncclCommInitRank(&r->comm, world, u, rank);
    if (nr != ncclSuccess) {
        r->comm = NULL;
        release(r);
        return fail_nccl("ncclCommInitRank", nr);
    }
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
    const int nxt = (r->rank + 1) % r->world, prv = (r->rank + r->world - 1) % r->world;
    NCCL_TRY(ncclGroupStart());
    NCCL_TRY(ncclSend(r->st_out[k], r->state_bytes, ncclUint8, nxt, r->comm, r->cs));
    NCCL_TRY(ncclRecv(r->st_in[k], r->state_bytes, ncclUint8, prv, r->comm, r->cs));
    NCCL_TRY(ncclGroupEnd());
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
    hipStream_t s = (hipStream_t)hip_stream;
    HIP_TRY(hipSetDevice(r->device));
    int rc;
    if ((rc = exchange_end(r, step, in, s))) return rc;
    if (next_last && (rc = exchange_begin(r, step + 1, next_last, s))) return rc;
    return mm_process_stream(r->h, in, out, r->chunk, r->format, s);
}

void mm_ring_destroy(mm_ring *r) { release(r); }
