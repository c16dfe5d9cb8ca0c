"""Handle lifecycle on the HIP path (through the C-ABI): batch changes,
allocation failure, the G_{t-1} state slots, parameter changes that must not
stall other handles, and the geometries at the edges of the build.

Every comparison is bitwise against an untouched handle or an uninterrupted
stream (the results do not depend on the batch size, include/mm.h), or
against the oracle at the SURVEY.md §8c bars.
"""
import os

import numpy as np
import pytest

import mmtest as T
import oracle_py as O

pytestmark = pytest.mark.gpu


def _dev(frames):
    import torch
    return torch.from_numpy(np.stack(frames)).cuda()


def _stream(h, dev, fmt, chunks):
    """Process dev[0..n) through h in calls of the given frame counts."""
    import torch
    out = torch.empty_like(dev)
    k = 0
    for c in chunks:
        h.process_stream(dev[k:k + c], out[k:k + c], c, fmt)
        k += c
    torch.cuda.synchronize()
    return out


def test_set_batch_oom_keeps_handle_intact():
    """mm_set_batch failure-atomic: with most of the device
    memory taken, a 4096-frame batch at 1080p gets its G buffer but not its Q
    buffer; mm_set_batch returns MM_ERR_OOM and the handle keeps its batch,
    buffers and state: frames after the failure equal an untouched handle's."""
    import torch
    import mm355
    W, H = 1920, 1080
    fr = T.synth(W, H, 6, fmt="u8")
    dev = _dev(fr)
    p = mm355.Params.make(phase_scale=25.0)
    a, b = mm355.Handle(W, H, p), mm355.Handle(W, H, p)
    a.set_batch(4), b.set_batch(4)
    oa, ob = torch.empty_like(dev), torch.empty_like(dev)
    a.process_stream(dev[:3], oa[:3], 3, mm355.RGBA8)
    b.process_stream(dev[:3], ob[:3], 3, mm355.RGBA8)
    torch.cuda.synchronize()
    free, _ = torch.cuda.mem_get_info()
    g_bytes = 4097 * (1024 + 1) * 1080 * 8          # G: 36 GB, Q: 36 GB
    filler = None
    leave = g_bytes + (8 << 30)                       # room for G, not for G + Q
    if free > leave:
        filler = torch.empty(free - leave, dtype=torch.uint8, device="cuda")
    with pytest.raises(mm355.MMError) as ei:
        a.set_batch(4096)
    assert ei.value.code == -5                        # MM_ERR_OOM
    del filler
    torch.cuda.empty_cache()
    assert a.batch == 4
    a.process_stream(dev[3:], oa[3:], 3, mm355.RGBA8)
    b.process_stream(dev[3:], ob[3:], 3, mm355.RGBA8)
    torch.cuda.synchronize()
    assert torch.equal(oa, ob)
    a.close(), b.close()


def test_default_batch_without_yh_and_results_batch_independent():
    """The fused path allocates no Yh: the default batch at
    1080p is 64 (2 GiB of G + Q), and a default-batch stream equals a batch-5
    stream bitwise."""
    import mm355
    W, H = 1920, 1080
    h = mm355.Handle(W, H, mm355.Params.make(phase_scale=25.0))
    assert h.batch == 64
    fr = T.synth(W, H, 12, fmt="u8")
    dev = _dev(fr)
    a = _stream(h, dev, mm355.RGBA8, [12])
    h2 = mm355.Handle(W, H, mm355.Params.make(phase_scale=25.0))
    h2.set_batch(5)
    b = _stream(h2, dev, mm355.RGBA8, [12])
    import torch
    assert torch.equal(a, b)
    h.close(), h2.close()


@pytest.mark.parametrize("batch,chunks", [(1, [1] * 9), (3, [2, 1, 4, 2]), (4, [9]), (8, [5, 4])])
def test_state_slots_any_call_pattern(batch, chunks):
    """G_{t-1} slot placement (place_batch): every mix of call sizes and batch
    sizes, including the one-frame-per-call pattern (slots alternate) and the
    slot copy, gives the uninterrupted single-call stream bitwise."""
    import mm355
    W, H = 200, 120
    fr = T.synth(W, H, 9)
    dev = _dev(fr)
    p = mm355.Params.make(phase_scale=25.0)
    ref_h = mm355.Handle(W, H, p)
    ref_h.set_batch(9)
    ref = _stream(ref_h, dev, mm355.RGBA32F, [9])
    h = mm355.Handle(W, H, p)
    h.set_batch(batch)
    got = _stream(h, dev, mm355.RGBA32F, chunks)
    import torch
    assert torch.equal(got, ref)
    ora = T.oracle_run(W, H, fr, 5, 25.0)
    for k in range(1, 9):
        T.assert_close_f32(got[k].cpu().numpy(), ora[k])
    ref_h.close(), h.close()


def test_set_batch_mid_stream_keeps_state():
    """Changing the batch between frames carries G_{t-1} over."""
    import torch
    import mm355
    W, H = 200, 120
    fr = T.synth(W, H, 8)
    dev = _dev(fr)
    p = mm355.Params.make(phase_scale=25.0)
    ref = _stream(mm355.Handle(W, H, p), dev, mm355.RGBA32F, [8])
    h = mm355.Handle(W, H, p)
    h.set_batch(2)
    out = torch.empty_like(dev)
    h.process_stream(dev[:3], out[:3], 3, mm355.RGBA32F)
    h.set_batch(7)
    h.process_stream(dev[3:], out[3:], 5, mm355.RGBA32F)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    h.close()


def test_debug_view_after_batch_growth():
    """a debug view at batch 1, then batch 8 and an 8-frame
    debug stream: the view textures grow with the batch (no write past them)
    and the frames equal a fresh handle's at batch 8."""
    import torch
    import mm355
    W, H = 64, 48
    fr = T.synth(W, H, 9)
    dev = _dev(fr)
    p = mm355.Params.make(phase_scale=10.0, show_magnitude=True)
    h = mm355.Handle(W, H, p)
    h.set_batch(1)
    out = torch.empty_like(dev)
    h.process(dev[0], out[0], mm355.RGBA32F)
    h.set_batch(8)
    h.process_stream(dev[1:], out[1:], 8, mm355.RGBA32F)
    torch.cuda.synchronize()
    ref = _stream(mm355.Handle(W, H, p), dev, mm355.RGBA32F, [9])
    assert torch.equal(out, ref)
    ora = T.oracle_run(W, H, fr, 5, 10.0, debug=(True, False))
    for k in range(1, 9):
        e = np.abs(out[k].cpu().numpy()[..., 0].astype(np.float64) - ora[k][..., 0])
        assert e.max() < 1e-4
    h.close()


def test_steerable_set_batch_mid_stream():
    """mm_set_batch mid-stream must not drop or corrupt the
    steerable local-phase state: equal, bitwise, to the uninterrupted stream."""
    import torch
    import mm355
    W, H = 96, 64
    fr = T.synth(W, H, 7)
    dev = _dev(fr)
    p = mm355.Params.make(levels=5, phase_scale=10.0, mode=mm355.MODE_STEERABLE, orientations=8)
    ref_h = mm355.Handle(W, H, p)
    ref_h.set_batch(2)
    ref = _stream(ref_h, dev, mm355.RGBA32F, [7])
    h = mm355.Handle(W, H, p)
    h.set_batch(2)
    out = torch.empty_like(dev)
    h.process_stream(dev[:3], out[:3], 3, mm355.RGBA32F)
    h.set_batch(5)                      # grows the per-batch spectra, keeps the planes
    h.process_stream(dev[3:], out[3:], 4, mm355.RGBA32F)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # and with a mm_set_state in between
    st = torch.empty(h.state_bytes, dtype=torch.uint8, device="cuda")
    g = mm355.Handle(W, H, p)
    g.set_batch(3)
    o2 = torch.empty_like(dev)
    g.process_stream(dev[:4], o2[:4], 4, mm355.RGBA32F)
    g.get_state(st)
    g.set_batch(1)
    g.set_state(st)
    g.process_stream(dev[4:], o2[4:], 3, mm355.RGBA32F)
    torch.cuda.synchronize()
    assert torch.equal(o2, ref)
    ref_h.close(), h.close(), g.close()


def _gate_scenario(name):
    """Runs tests/gate_scenarios.py NAME in a fresh process with enough HIP
    hardware queues that every stream gets its own (GPU_MAX_HW_QUEUES=16):
    at the default of 4, streams share hardware queues round-robin, and a
    stream held behind a gate then also holds every stream on its queue — a
    property of the runtime's queue mapping, not of the entry point under
    test."""
    import subprocess
    import sys
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16", PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gate_scenarios.py"), name],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_set_params_does_not_stall_other_streams():
    """mm_set_params waits only for its own handle's work:
    while handle B's stream is held behind a gate, A's edge-mode change
    returns; A's next frames use the new tables (tests/gate_scenarios.py)."""
    _gate_scenario("set_params")


def test_set_batch_does_not_stall_other_streams():
    """mm_set_batch of handle A returns while handle B's work
    is held behind a gate on another stream; A's stream across the batch
    change equals an uninterrupted one, and B's output is intact."""
    _gate_scenario("set_batch")


def test_destroy_does_not_stall_other_streams():
    """mm_destroy of handle A (with lazily grown debug-view and
    host-staging buffers) returns while handle B's work is held behind a gate
    on another stream; B's output is intact."""
    _gate_scenario("destroy")


def test_set_batch_waits_for_own_queued_work():
    """mm_set_batch issued while the handle's own work is held on
    its stream returns only after that work ran; outputs equal an ungated
    handle's across the batch change (tests/gate_scenarios.py own_set_batch)."""
    _gate_scenario("own_set_batch")


def test_destroy_waits_for_own_queued_work():
    """mm_destroy with the handle's own work held on its stream
    frees the buffers only behind that work (own_destroy)."""
    _gate_scenario("own_destroy")


def test_steerable_set_state_then_pyramid_passes_through():
    """a steerable mm_set_state sets only the local-phase planes;
    after switching that handle to pyramid mode the G_{t-1} slot holds no
    state, so the next frame passes through (as after a reset) and the
    following frames equal a fresh pyramid handle's."""
    import torch
    import mm355
    W, H = 96, 64
    fr = T.synth(W, H, 4)
    dev = _dev(fr)
    ps = mm355.Params.make(levels=5, phase_scale=10.0, mode=mm355.MODE_STEERABLE, orientations=4)
    pp = mm355.Params.make(levels=5, phase_scale=10.0)
    s = mm355.Handle(W, H, ps)
    o = torch.empty_like(dev)
    s.process_stream(dev[:2], o[:2], 2, mm355.RGBA32F)
    st = torch.empty(s.state_bytes, dtype=torch.uint8, device="cuda")
    s.get_state(st)
    h = mm355.Handle(W, H, ps)
    h.set_state(st)
    h.set_params(pp)
    got = _stream(h, dev, mm355.RGBA32F, [4])
    ref = _stream(mm355.Handle(W, H, pp), dev, mm355.RGBA32F, [4])
    assert torch.equal(got[0], dev[0])
    assert torch.equal(got, ref)
    # a handle that HAS run frames (its G slot holds an old frame)
    # must not pair the next pyramid frame with that stale slot either
    u = mm355.Handle(W, H, ps)
    junk = _dev(T.synth(W, H, 3, seed=7))
    _stream(u, junk, mm355.RGBA32F, [3])
    u.set_state(st)
    u.set_params(pp)
    got = _stream(u, dev, mm355.RGBA32F, [4])
    assert torch.equal(got[0], dev[0]), "first frame after a steerable set_state must pass through"
    assert torch.equal(got, ref)
    # the reverse: a pyramid set_state leaves no stale local-phase planes, so
    # switching to steerable passes the next frame through as well
    pst = torch.empty(mm355.Handle(W, H, pp).state_bytes, dtype=torch.uint8, device="cuda")
    q = mm355.Handle(W, H, pp)
    q.process_stream(dev[:2], torch.empty_like(dev[:2]), 2, mm355.RGBA32F)
    q.get_state(pst)
    v = mm355.Handle(W, H, ps)
    _stream(v, junk, mm355.RGBA32F, [3])
    v.set_params(pp)
    v.set_state(pst)
    v.set_params(ps)
    gs = _stream(v, dev, mm355.RGBA32F, [4])
    rs = _stream(mm355.Handle(W, H, ps), dev, mm355.RGBA32F, [4])
    assert torch.equal(gs[0], dev[0]), "first steerable frame after a pyramid set_state must pass through"
    assert torch.equal(gs, rs)
    u.close(), v.close(), q.close()
    with pytest.raises(mm355.MMError):
        g = mm355.Handle(W, H, ps)
        g.set_state(st)
        g.set_params(pp)
        g.get_state(torch.empty(g.state_bytes, dtype=torch.uint8, device="cuda"))   # no G_{t-1}
    s.close(), h.close()


@pytest.mark.parametrize("W,H,L,S,edge", [(16, 12, 3, 10.0, 0), (12, 10, 4, 25.0, 1), (13, 9, 5, 10.0, 0),
                                          (16, 16, 5, 25.0, 1), (9, 16, 2, 10.0, 0)])
def test_smallest_canvas_n16(W, H, L, S, edge):
    """N = 16, the smallest canvas of the build (9 <= max(W, H) <= 16), on
    the oracle's canvas (no clamp: VERDICT r2 #7), frame and stream calls."""
    fr = T.synth(W, H, 5)
    ref = T.oracle_run(W, H, fr, L, S, edge)
    for mode in ("frame", "stream"):
        got = T.gpu_run(W, H, fr, L, S, edge, mode=mode, batch=2)
        assert np.array_equal(got[0], fr[0])
        for g, r in zip(got[1:], ref[1:]):
            T.assert_close_f32(g, r)


def test_refused_geometries():
    """max(W, H) <= 8 (N <= 8) and max(W, H) > 8192 (N = 16384) are refused
    with MM_ERR_UNSUPPORTED, not computed on another canvas; N = 8192 (5K/8K
    screens, since round 5) is accepted except by the steerable extension."""
    import mm355
    for W, H in ((8, 6), (4, 4), (2, 8), (8193, 2160), (16384, 8640)):
        with pytest.raises(mm355.MMError) as ei:
            mm355.Handle(W, H)
        assert ei.value.code == -2, (W, H)
    h = mm355.Handle(5120, 2880)
    assert h.N == 8192
    h.close()
    with pytest.raises(mm355.MMError) as ei:
        mm355.Handle(5120, 2880, mm355.Params.make(mode=mm355.MODE_STEERABLE, orientations=8))
    assert ei.value.code == -2


@pytest.mark.parametrize("W,H,n", [(1920, 1080, 30), (640, 360, 48)])
def test_k2_second_half_tails_bitwise(W, H, n):
    """k_cols's tail blocks (MM_K2_TAIL2 percent of the second-half blocks'
    frames, each primed with the frame before its first) give the same bits as
    no tails and as a larger share."""
    import os
    import torch
    import mm355
    fr = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    outs = []
    for pct in ("0", "10", "40"):
        old = os.environ.get("MM_K2_TAIL2")
        os.environ["MM_K2_TAIL2"] = pct
        try:
            h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
        finally:
            if old is None:
                del os.environ["MM_K2_TAIL2"]
            else:
                os.environ["MM_K2_TAIL2"] = old
        h.set_batch(n)
        if not outs:
            h.synth(fr, 0, n)
        o = torch.empty_like(fr)
        h.process_stream(fr, o, n, mm355.RGBA8)
        torch.cuda.synchronize()
        h.close()
        outs.append(o)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
