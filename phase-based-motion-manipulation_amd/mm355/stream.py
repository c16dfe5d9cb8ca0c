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

Overlap (``prefetch=True`` in ``step``): steps 1-2 of step s+1 are posted
before step s's frames are processed, so the ring transfer (the state
G_{t-1}, 8.86 MB at 1080p since ABI 8; ~0.06 ms over one xGMI link) runs on
the collective's stream underneath step s's kernels; step s+1 then only
waits for a transfer that has long finished.  This needs step s+1's last
input frame one step early (one chunk of lookahead); ``finish()`` retires a
transfer posted for a step that is never run.

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
        self._posted = {}     # step -> (requests, st_out, st_in)

    # -- the ring shift, split so that it can overlap compute --------------
    def exchange_begin(self, step):
        """Steps 1-2 for `step`: compute my last frame's state, post the ring."""
        if self.world == 1 or step in self._posted:
            return
        import torch.distributed as dist
        b = self.backend
        lo, hi = shard_range(step, self.rank, self.world, self.chunk)
        st_out = b.state_of(hi - 1)
        st_in = b.empty_state()
        nxt = (self.rank + 1) % self.world
        prv = (self.rank - 1) % self.world
        ops = [dist.P2POp(dist.isend, st_out, nxt, group=self.group),
               dist.P2POp(dist.irecv, st_in, prv, group=self.group)]
        self._posted[step] = (dist.batch_isend_irecv(ops), st_out, st_in)

    def exchange_end(self, step):
        """Step 3 for `step`: wait for its ring shift and set the state."""
        b = self.backend
        if self.world == 1:
            if step == 0:
                b.reset()
            return
        self.exchange_begin(step)          # no-op when posted ahead
        reqs, _, st_in = self._posted.pop(step)
        for req in reqs:
            req.wait()
        if self.rank == 0:
            prev_carry, self._carry = self._carry, st_in
            if step == 0:
                b.reset()
            else:
                b.set_state(prev_carry)
        else:
            b.set_state(st_in)

    def exchange(self, step):
        """Steps 1-3 above, serialised; leaves the backend's state set."""
        self.exchange_begin(step)
        self.exchange_end(step)

    def step(self, step, prefetch=False):
        """Run one step.  prefetch: post step+1's ring shift before this
        step's compute (overlap; needs step+1's input one step early)."""
        self.exchange_end(step)
        if prefetch:
            self.exchange_begin(step + 1)
        lo, hi = shard_range(step, self.rank, self.world, self.chunk)
        return self.backend.process(lo, hi - lo)

    def finish(self):
        """Retire ring shifts posted for steps that were not run."""
        for step in sorted(self._posted):
            for req in self._posted[step][0]:
                req.wait()
        self._posted.clear()
