"""Gate scenarios for tests/test_handle.py (run in a fresh process, GPU only).

A stream is held behind a host-mapped flag (hipStreamWaitValue32) until the
scenario releases it, so work queued on it cannot have run before the release,
with no dependence on timing.  Each scenario runs one handle entry
point of handle A in a thread while handle B's 1080p stream is held on such a
gated stream, and requires that the entry point returns (it waited for A's own
work only, never for the device: DESIGN.md §7b), that B's work was still held
when it did, and that B's output after the release is intact.

Two more scenarios hold handle A's OWN stream and require that mm_set_batch
and mm_destroy of A wait for A's queued work before its buffers go back to
the pool (own_set_batch, own_destroy).

usage: python tests/gate_scenarios.py set_params|set_batch|destroy|own_set_batch|own_destroy
"""
import ctypes
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "phase-based-motion-manipulation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mm355  # noqa: E402
import mmtest as T  # noqa: E402


class Gate:
    """hipStreamWaitValue32(stream, flag >= 1) on a host-mapped, coherent flag."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        self.hip.hipHostFree.argtypes = [ctypes.c_void_p]
        self.hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                  ctypes.c_uint, ctypes.c_uint32]
        self.p = ctypes.c_void_p()
        assert self.hip.hipHostMalloc(ctypes.byref(self.p), 4, 0x2 | 0x40000000) == 0   # mapped, coherent
        self._set(0)

    def _set(self, v):
        ctypes.c_uint32.from_address(self.p.value).value = v

    def hold(self, stream_handle):
        assert self.hip.hipStreamWaitValue32(stream_handle, self.p, 1, 0, 0xFFFFFFFF) == 0   # >= 1

    def release(self):
        self._set(1)

    def free(self):
        self.hip.hipHostFree(self.p)


def returns_while_other_stream_gated(op, b_frames=8):
    """Queues handle B's 1080p stream on a gated stream, runs op() in a thread;
    -> (op returned within 20 s, B still held then, B's output == ungated)."""
    W, H = 1920, 1080
    p = mm355.Params.make(phase_scale=25.0)
    b = mm355.Handle(W, H, p)
    b.set_batch(b_frames)
    frames = torch.empty((b_frames, H, W, 4), dtype=torch.uint8, device="cuda")
    b.synth(frames, 0, b_frames)
    ref = torch.empty_like(frames)
    r = mm355.Handle(W, H, p)
    r.process_stream(frames, ref, b_frames, mm355.RGBA8)
    torch.cuda.synchronize()
    outb = torch.zeros_like(frames)
    sb = torch.cuda.Stream()
    gate = Gate()
    th = threading.Thread(target=op)
    try:
        gate.hold(sb.cuda_stream)
        b.process_stream(frames, outb, b_frames, mm355.RGBA8, stream=sb.cuda_stream)
        held = not sb.query()
        th.start()
        th.join(20.0)
        returned = not th.is_alive()
        pending = not sb.query()
    finally:
        gate.release()
    th.join()
    torch.cuda.synchronize()
    gate.free()
    ok_b = torch.equal(outb, ref)
    b.close()
    r.close()
    assert held, "the gate did not hold B's stream (hipStreamWaitValue32)"
    return returned, pending, ok_b


def check(name, returned, pending, ok_b):
    assert returned, f"{name} waited for another handle's stream"
    assert pending, "B's gated work finished before the gate was released"
    assert ok_b, "B's output changed"


def set_params():
    Wa, Ha = 64, 48
    fr = T.synth(Wa, Ha, 3)
    a = mm355.Handle(Wa, Ha, mm355.Params.make(phase_scale=10.0))
    dev = torch.from_numpy(np.stack(fr)).cuda()
    oa = torch.empty_like(dev)
    a.process(dev[0], oa[0], mm355.RGBA32F)
    torch.cuda.synchronize()
    check("mm_set_params", *returns_while_other_stream_gated(
        lambda: a.set_params(mm355.Params.make(phase_scale=10.0, edge_mode=mm355.EDGE_CLAMP))))
    a.process(dev[1], oa[1], mm355.RGBA32F)
    a.process(dev[2], oa[2], mm355.RGBA32F)
    torch.cuda.synchronize()
    # frame 2 and its state (frame 1) both ran on the CLAMP tables (frame 1
    # itself pairs the old REPEAT state with the new tables: the state is the
    # previous frame's resampled rows, include/mm.h mm_set_params)
    ref = T.oracle_run(Wa, Ha, fr, 5, 10.0, edge=1)
    T.assert_close_f32(oa[2].cpu().numpy(), ref[2])
    a.close()


def set_batch():
    W, H = 200, 120
    fr = T.synth(W, H, 8)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    p = mm355.Params.make(phase_scale=25.0)
    rh = mm355.Handle(W, H, p)
    ref = torch.empty_like(dev)
    rh.process_stream(dev, ref, 8, mm355.RGBA32F)
    a = mm355.Handle(W, H, p)
    a.set_batch(2)
    out = torch.empty_like(dev)
    a.process_stream(dev[:3], out[:3], 3, mm355.RGBA32F)
    check("mm_set_batch", *returns_while_other_stream_gated(lambda: a.set_batch(7)))
    a.process_stream(dev[3:], out[3:], 5, mm355.RGBA32F)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "A's stream across the batch change"
    a.close()
    rh.close()


def destroy():
    W, H = 96, 64
    fr = T.synth(W, H, 3)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    a = mm355.Handle(W, H, mm355.Params.make(phase_scale=10.0, show_magnitude=True))
    out = torch.empty_like(dev)
    a.process_stream(dev, out, 3, mm355.RGBA32F)                                      # debug textures
    host_out = np.empty_like(fr[0])
    a.process(np.ascontiguousarray(fr[1]), host_out, mm355.RGBA32F, on_device=False)   # host staging
    torch.cuda.synchronize()
    check("mm_destroy", *returns_while_other_stream_gated(a.close))


def _own_gated(a, sa, queue_work, op):
    """Holds handle A's OWN stream sa behind a gate, queues A's work on it
    (queue_work), runs op() (an entry point that frees or swaps buffers that
    work reads) in a thread -> (op still blocked while A's work was held,
    op returned after the release).  ADVICE r4: the stream-ordered frees
    (hipFreeAsync behind last_ev) must not run ahead of A's queued kernels."""
    import time
    gate = Gate()
    th = threading.Thread(target=op)
    try:
        gate.hold(sa.cuda_stream)
        queue_work()
        th.start()
        time.sleep(1.0)
        blocked = th.is_alive() and not sa.query()
    finally:
        gate.release()
    th.join(20.0)
    returned = not th.is_alive()
    torch.cuda.synchronize()
    gate.free()
    return blocked, returned


def own_set_batch():
    """A's 8-frame 1080p stream is queued behind a gate on A's stream; a
    concurrent mm_set_batch of A (which retires G and Q and moves the state
    slot) must wait for that work, and A's outputs, including the frames after
    the batch change, equal an ungated handle's."""
    W, H = 1920, 1080
    p = mm355.Params.make(phase_scale=25.0)
    n = 8
    frames = torch.empty((2 * n, H, W, 4), dtype=torch.uint8, device="cuda")
    r = mm355.Handle(W, H, p)
    r.set_batch(n)
    r.synth(frames, 0, 2 * n)
    ref = torch.empty_like(frames)
    r.process_stream(frames, ref, 2 * n, mm355.RGBA8)
    torch.cuda.synchronize()
    a = mm355.Handle(W, H, p)
    a.set_batch(n)
    out = torch.zeros_like(frames)
    sa = torch.cuda.Stream()
    blocked, returned = _own_gated(
        a, sa, lambda: a.process_stream(frames[:n], out[:n], n, mm355.RGBA8, stream=sa.cuda_stream),
        lambda: a.set_batch(3))
    assert blocked, "mm_set_batch returned while the handle's own work was still held"
    assert returned, "mm_set_batch did not return after the release"
    a.process_stream(frames[n:], out[n:], n, mm355.RGBA8, stream=sa.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "A's output across a set_batch issued while its work was queued"
    a.close()
    r.close()


def own_destroy():
    """mm_destroy of A while A's own stream is held: it returns only after the
    held work ran (the buffers it reads go back to the pool behind it), and
    that work's output is complete."""
    W, H = 1920, 1080
    p = mm355.Params.make(phase_scale=25.0)
    n = 8
    frames = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    r = mm355.Handle(W, H, p)
    r.set_batch(n)
    r.synth(frames, 0, n)
    ref = torch.empty_like(frames)
    r.process_stream(frames, ref, n, mm355.RGBA8)
    torch.cuda.synchronize()
    a = mm355.Handle(W, H, p)
    a.set_batch(n)
    out = torch.zeros_like(frames)
    sa = torch.cuda.Stream()
    blocked, returned = _own_gated(
        a, sa, lambda: a.process_stream(frames, out, n, mm355.RGBA8, stream=sa.cuda_stream), a.close)
    assert blocked, "mm_destroy returned while the handle's own work was still held"
    assert returned, "mm_destroy did not return after the release"
    assert torch.equal(out, ref), "A's held work lost its buffers"
    r.close()


if __name__ == "__main__":
    {"set_params": set_params, "set_batch": set_batch, "destroy": destroy,
     "own_set_batch": own_set_batch, "own_destroy": own_destroy}[sys.argv[1]]()
    print(f"{sys.argv[1]}: ok")
