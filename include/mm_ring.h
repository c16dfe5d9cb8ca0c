/*
 * mm_ring.h — frame-sharded streaming over an RCCL ring, in C.
 *
 * One process per GPU.  Output frame t of the reference operator depends only
 * on input frames t-1 and t (MotionMagnificationProcessor.cs:142 keeps the
 * previous input as the only state), and that state is a pure function of
 * input t-1 (mm_compute_state).  So a stream shards into contiguous per-rank
 * chunks and the only exchange is ONE ring shift per step:
 *
 *   step s, world G, chunk C: rank g owns frames [s*G*C + g*C, s*G*C + (g+1)*C)
 *   1. st_out = state of my last frame of step s (from my own input)
 *   2. ncclSend(st_out -> g+1), ncclRecv(st_in <- g-1)   (one group call)
 *   3. rank g > 0: state := st_in of step s;  rank 0: state := st_in of step
 *      s-1 (rank G-1's last frame of the previous step); at s = 0: reset
 *      (the stream's first frame passes through, .cs:111-117)
 *   4. mm_process_stream over my C frames
 *
 * Steps 1-2 of step s+1 are posted before step s's frames are processed (the
 * shift runs on the ring's own HIP stream under step s's kernels; one chunk
 * of input lookahead), as mm355.stream.ShardedStream(prefetch=True) does in
 * Python.  The state buffers are device memory (mm_state_size bytes).
 *
 * This module links RCCL (librccl); the frame operator itself (libmm355) does
 * not.  Return codes are the MM_* codes of mm.h; an RCCL failure is MM_ERR_HIP
 * (mm_ring_last_error() gives RCCL's message).
 */
#ifndef MM_RING_H
#define MM_RING_H

#include <stddef.h>

#include "mm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MM_RING_ID_BYTES 128   /* == NCCL_UNIQUE_ID_BYTES */

typedef struct mm_ring mm_ring;

/* Rank 0 generates the ring id and hands it to every rank out of band (a
 * file, a launcher, MPI ...).  Replaces torch.distributed's rendezvous. */
int mm_ring_get_id(unsigned char id[MM_RING_ID_BYTES]);

/* Joins the ring as `rank` of `world` on HIP device `hip_device`, for the
 * width x height stream processed by handle `h` (same device, same geometry)
 * in chunks of `chunk` frames of `format` (MM_RGBA8 / MM_RGBA32F).  world may
 * be 1 (the shift is then a send to and a receive from itself). */
int mm_ring_create(int world, int rank, const unsigned char id[MM_RING_ID_BYTES], int hip_device,
                   mm_handle *h, int width, int height, int chunk, int format, mm_ring **out);

/* Runs step `step` (steps in order from 0): `in` = this rank's C input frames
 * of the step, `out` = their C output frames, `next_last` = the LAST input
 * frame of this rank's chunk of step+1 (posts that step's shift ahead), or
 * NULL for the final step.  All device pointers; work is ordered on
 * `hip_stream` (NULL: the default stream).  Asynchronous like mm_process_stream. */
int mm_ring_step(mm_ring *r, int step, const void *in, void *out, const void *next_last,
                 void *hip_stream);

/* MM_MODE_STEERABLE with MM_FILTER_IIR ("a recursive IIR
 * extension ... would need a warm-up halo").  The IIR state after frame t is a
 * history of every frame before it, so no single frame's state can be handed
 * to the next rank without serialising the ring.  Instead each rank restarts
 * its filter from rest `halo_frames` frames before its chunk: `halo` = the
 * input frames [c - halo_frames, c) immediately preceding the chunk's first
 * frame c (device memory, caller-owned: the caller reads them from its source
 * as it reads the chunk), processed with their outputs discarded, then the
 * chunk into `out`.  halo_frames = min(c, mm_ring_halo_frames()) (the halo of
 * a chunk near the stream's start begins at frame 0, which is then exact;
 * rank 0 of step 0 passes 0).  The filter's two poles decay by (1 - iir_high)
 * and (1 - iir_low) per frame, so the difference from the single-rank stream
 * falls as (1 - iir_low)^halo_frames: mm_ring_halo_frames() picks the halo at
 * which that factor is 1e-6 (270 frames at iir_low = 0.05), where RGBA8
 * outputs meet the parity bar (<= 1 LSB on <= 0.1 % of values; tests/test_ring_c.py).
 * Nothing crosses the ring in this mode.  mm_ring_step refuses IIR handles.
 * Cost: every rank re-runs halo_frames frames per chunk, i.e. halo_frames /
 * chunk extra work (90 % at the default 270-frame halo and 300-frame chunks);
 * the halo buffer the caller keeps is halo_frames frames.
 * mm_ring_halo_frames: ceil(ln 1e-6 / ln(1 - iir_low)) in closed form, 0 for
 * a non-IIR ring; MM_ERR_UNSUPPORTED above MM_RING_HALO_MAX frames (iir_low
 * below about 0.0067: the halo would dwarf any chunk). */
#define MM_RING_HALO_MAX 2048
int mm_ring_step_halo(mm_ring *r, int step, const void *halo, int halo_frames, const void *in, void *out,
                      void *hip_stream);
int mm_ring_halo_frames(const mm_ring *r, int *frames);

/* Path of the libmm355 this library's mm_* calls are bound to (dladdr), for
 * callers that load a specific build of the operator (mm355/ring.py refuses
 * a ring bound to another build than the one it loaded).  NULL if unknown. */
const char *mm_ring_core_library(void);

/* Waits for every posted shift (a shift posted for a step that is never run
 * included) and releases the ring. */
void mm_ring_destroy(mm_ring *r);

const char *mm_ring_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MM_RING_H */
