"""Frame-sharded processing of one video stream across ranks.

Output frame t depends only on input frames t-1 and t: the temporal state is
the previous frame's spectrum, a pure function of that frame's *input*.  So a
stream shards into contiguous per-rank chunks; the only exchange is one ring
shift per step carrying the chunk-boundary state to the next rank:

    step s, world G, chunk C:  rank g owns frames [s*G*C + g*C, s*G*C + (g+1)*C)
    1. st_out = state of my LAST frame   (computed up-front from my own input,
                                          so no rank waits on another's compute)
    2. ring:  send st_out -> g+1 ;  recv st_in <- g-1        (RCCL over xGMI)
    3. rank g>0: state := st_in ; rank 0: state := st_in of the PREVIOUS step
       (the frame before rank 0's chunk is rank G-1's last frame of step s-1);
       at s == 0 rank 0 has no predecessor: reset (first-frame passthrough).
    4. process my C frames.

The backend does the compute; the GPU backend is a ``Handle`` over the HIP
library.  The collective is ``torch.distributed`` (nccl == RCCL on ROCm; the
CPU tests use gloo with the same code).
"""


def shard_range(step, rank, world, chunk):
    base = step * world * chunk + rank * chunk
    return base, base + chunk


class ShardedStream:
    """backend must provide:
         empty_state() -> tensor      state_of(frame_index) -> tensor
         set_state(tensor)            reset()
         process(first_frame_index, count) -> anything
    """

    def __init__(self, backend, chunk, rank=0, world=1, group=None):
        self.backend, self.chunk = backend, chunk
        self.rank, self.world, self.group = rank, world, group
        self._carry = None

    def exchange(self, step):
        """Steps 1-3 above; returns nothing, leaves the backend's state set."""
        b = self.backend
        if self.world == 1:
            if step == 0:
                b.reset()
            return
        import torch.distributed as dist
        lo, hi = shard_range(step, self.rank, self.world, self.chunk)
        st_out = b.state_of(hi - 1)
        st_in = b.empty_state()
        nxt = (self.rank + 1) % self.world
        prv = (self.rank - 1) % self.world
        ops = [dist.P2POp(dist.isend, st_out, nxt, group=self.group),
               dist.P2POp(dist.irecv, st_in, prv, group=self.group)]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        if self.rank == 0:
            prev_carry, self._carry = self._carry, st_in
            if step == 0:
                b.reset()
            else:
                b.set_state(prev_carry)
        else:
            b.set_state(st_in)

    def step(self, step):
        self.exchange(step)
        lo, hi = shard_range(step, self.rank, self.world, self.chunk)
        return self.backend.process(lo, hi - lo)
