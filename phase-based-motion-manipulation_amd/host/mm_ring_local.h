/*
 * mm_ring_local.h — TEST-ONLY transport of the C ring (host/mm_ring.c).
 *
 * The product ring (include/mm_ring.h) shifts the temporal state between
 * ranks with RCCL, one process per GPU.  A one-GPU box cannot run that at
 * world > 1 (RCCL refuses two ranks on one device), so the multi-rank step
 * logic of mm_ring_step — rank 0's carry of the state received one step
 * earlier, the two state slots reused across steps, the shift of step s+1
 * posted under step s — would first run on an 8-GPU node.  This transport
 * runs that same code with the ranks as threads of one process sharing one
 * device: the shift is a device-to-device copy on each rank's ring stream,
 * ordered by events and two host barriers per shift (mm_ring.c, "local
 * transport").  Everything above the shift is the product code path.
 *
 * Usage: one hub per world; each of `world` threads creates its own
 * mm_handle and joins with mm_ring_create_local(hub, rank, ...), then calls
 * mm_ring_step / mm_ring_destroy exactly as with mm_ring_create.  All ranks
 * must call mm_ring_step for the same steps with the same next_last
 * NULL-ness (a shift is a collective).  A failed HIP call inside a shift
 * leaves the other ranks waiting at the hub's barrier: test use only.
 */
#ifndef MM_RING_LOCAL_H
#define MM_RING_LOCAL_H

#include "mm_ring.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mm_ring_hub mm_ring_hub;

int mm_ring_hub_create(int world, mm_ring_hub **out);   /* 1 <= world <= 64 */
void mm_ring_hub_destroy(mm_ring_hub *hub);             /* after every rank's mm_ring_destroy */

int mm_ring_create_local(mm_ring_hub *hub, int rank, int hip_device, mm_handle *h, int width, int height,
                         int chunk, int format, mm_ring **out);

#ifdef __cplusplus
}
#endif
#endif /* MM_RING_LOCAL_H */
