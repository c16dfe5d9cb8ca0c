"""HIP path (through the C-ABI) vs the CPU oracle on the same seeded inputs.

Bars: fp32 max-abs <= 1e-4 and RMSE <= 1e-5 at integer phase
scale; 99.9th percentile <= 1e-4 at non-integer scale; RGBA8 exact except
+-1 LSB on <= 0.1% of values; first frame bitwise.
"""
import os
import numpy as np
import pytest

import mmtest as T
import oracle_py as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,L,S,edge", [
    (64, 48, 5, 10.0, 0), (64, 48, 4, 25.0, 0), (64, 48, 6, 25.0, 1), (64, 48, 5, 9.7, 0),
    (128, 96, 5, 25.0, 0), (200, 120, 5, 25.0, 1), (96, 96, 2, 10.0, 0), (64, 64, 1, 10.0, 1)])
def test_small_f32(W, H, L, S, edge):
    fr = T.synth(W, H, 4)
    ref = T.oracle_run(W, H, fr, L, S, edge)
    got = T.gpu_run(W, H, fr, L, S, edge)
    assert np.array_equal(got[0], fr[0])                   # first frame passthrough
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r, integer_scale=float(S).is_integer())
        assert np.all(g[..., 3] == 1.0)


def test_c1_256_gray_L3():
    """BASELINE config 0: 256x256 gray, 3 levels, PhaseScale 10, 32 frames."""
    fr = T.synth(256, 256, 32, gray=True)
    ref = T.oracle_run(256, 256, fr, 3, 10.0)
    got = T.gpu_run(256, 256, fr, 3, 10.0, mode="stream")
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r)


def test_u8_frames():
    W, H = 128, 96
    fr = T.synth(W, H, 5, fmt="u8")
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    got = T.gpu_run(W, H, fr, 5, 25.0)
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_u8(g, r)


def test_stream_equals_per_frame_bitwise():
    W, H = 200, 120
    fr = T.synth(W, H, 19)                  # crosses the 8-frame batch boundary twice
    a = T.gpu_run(W, H, fr, 5, 25.0, mode="frame")
    b = T.gpu_run(W, H, fr, 5, 25.0, mode="stream")
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_host_pointer_path():
    W, H = 64, 48
    fr = T.synth(W, H, 3)
    a = T.gpu_run(W, H, fr, 5, 10.0, mode="host")
    b = T.gpu_run(W, H, fr, 5, 10.0, mode="frame")
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_apply_off_passthrough_and_state():
    W, H = 64, 48
    fr = T.synth(W, H, 3)
    got = T.gpu_run(W, H, fr, 5, 10.0, apply=False)
    for g, f in zip(got, fr):
        assert np.array_equal(g, f)


def test_forward_spectrum_matches_oracle():
    """K1's forward path alone: mm_compute_state (the state G_t, row half
    spectra) vs the oracle's windowed luma rows (rfft) and, transformed over
    the padded columns, vs the oracle's 2D spectrum F_t."""
    import torch
    import mm355
    W, H = 128, 96
    f0, f1 = T.synth(W, H, 2)
    o = O.Oracle(W, H)
    o.process(f0)
    _, dbg = o.process(f1, dbg=True)
    h = mm355.Handle(W, H)
    N = h.N
    assert h.state_bytes == (N // 2 + 1) * H * 8
    st = torch.empty(h.state_bytes, dtype=torch.uint8, device="cuda")
    h.compute_state(torch.from_numpy(f1).cuda(), mm355.RGBA32F, st)
    torch.cuda.synchronize()
    G = T.state_rows(st, N, H)
    y0 = (N - H) // 2
    rows = np.fft.rfft(dbg["y_cur"][y0:y0 + H].astype(np.float64), axis=1).T
    assert np.abs(G - rows).max() / np.abs(rows).max() < 2e-6
    ref = T.centered_to_half(dbg["F_cur"], N)
    assert np.abs(T.spectrum_from_state(G, N, H) - ref).max() / np.abs(ref).max() < 2e-6
    h.close()


def test_state_get_set_and_reset():
    import torch
    import mm355
    W, H = 64, 48
    fr = T.synth(W, H, 4)
    full = T.gpu_run(W, H, fr, 5, 25.0)
    p = mm355.Params.make(phase_scale=25.0)
    a = mm355.Handle(W, H, p)
    b = mm355.Handle(W, H, p)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    out = torch.empty_like(dev)
    a.process(dev[0], out[0], mm355.RGBA32F)
    a.process(dev[1], out[1], mm355.RGBA32F)
    st = torch.empty(a.state_bytes, dtype=torch.uint8, device="cuda")
    a.get_state(st)
    torch.cuda.synchronize()
    b.set_state(st)
    b.process(dev[2], out[2], mm355.RGBA32F)
    torch.cuda.synchronize()
    assert np.array_equal(out[2].cpu().numpy(), full[2])
    b.reset()
    b.process(dev[3], out[3], mm355.RGBA32F)
    torch.cuda.synchronize()
    assert np.array_equal(out[3].cpu().numpy(), fr[3])   # passthrough after reset
    with pytest.raises(mm355.MMError):
        mm355.Handle(W, H).get_state(st)                 # MM_ERR_NO_STATE
    a.close()
    b.close()


def test_processor_mirror():
    import torch
    import mm355
    W, H = 64, 48
    fr = T.synth(W, H, 3)
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    proc = mm355.MotionMagnificationProcessor(W, H, phase_scale=1.0).Start()
    proc.phase_scale = 25.0
    proc.OnValidate()
    src = torch.from_numpy(np.stack(fr)).cuda()
    dst = torch.empty_like(src)
    for k in range(3):
        proc.OnRenderImage(src[k], dst[k])
    torch.cuda.synchronize()
    for k in range(1, 3):
        T.assert_close_f32(dst[k].cpu().numpy(), ref[k])
    proc.OnDestroy()


@pytest.mark.slow
def test_c2_1080p_vs_oracle():
    """BASELINE config 1 geometry: 1920x1080 RGBA, L=5, PhaseScale=25."""
    W, H = 1920, 1080
    fr = T.synth(W, H, 3, fmt="u8")
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    got = T.gpu_run(W, H, fr, 5, 25.0, mode="stream")
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_u8(g, r)
    ff = [f.astype(np.float32) / np.float32(255) for f in fr[:2]]
    rf = T.oracle_run(W, H, ff, 5, 25.0)
    gf = T.gpu_run(W, H, ff, 5, 25.0)
    T.assert_close_f32(gf[1], rf[1])


@pytest.mark.slow
def test_c3_2160p_vs_oracle():
    """BASELINE config 2 geometry: 3840x2160 RGBA, L=6, PhaseScale=25."""
    W, H = 3840, 2160
    ff = T.synth(W, H, 2)
    rf = T.oracle_run(W, H, ff, 6, 25.0)
    gf = T.gpu_run(W, H, ff, 6, 25.0)
    assert np.array_equal(gf[0], ff[0])
    T.assert_close_f32(gf[1], rf[1])


def test_chunk_boundary_state_handoff():
    """What the multi-GPU ring carries: rank g's state = mm_compute_state of the
    frame before its chunk.  Two handles ("ranks") reproduce one stream bitwise."""
    import torch
    import mm355
    W, H, C = 200, 120, 5
    fr = T.synth(W, H, 2 * C, fmt="u8")
    full = T.gpu_run(W, H, fr, 5, 25.0, mode="stream")
    p = mm355.Params.make(phase_scale=25.0)
    r0, r1 = mm355.Handle(W, H, p), mm355.Handle(W, H, p)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    out = torch.empty_like(dev)
    st = torch.empty(r1.state_bytes, dtype=torch.uint8, device="cuda")
    r0.compute_state(dev[C - 1], mm355.RGBA8, st)          # rank 0's last frame
    torch.cuda.synchronize()
    r1.set_state(st)
    r0.process_stream(dev[:C], out[:C], C, mm355.RGBA8)
    r1.process_stream(dev[C:], out[C:], C, mm355.RGBA8)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for k in range(2 * C):
        assert np.array_equal(got[k], full[k]), k
    r0.close()
    r1.close()


@pytest.mark.parametrize("W,H,S,std", [
    (64, 48, 10.0, {}), (200, 120, 25.0, dict(steep=2.0, high=0.3)),
    (128, 96, 9.7, dict(apply=False)), (96, 96, 25.0, dict(edge=0.0, sens=1.0))])
def test_standard_mode_f32(W, H, S, std):
    """f1: usePyramidDecomposition = false (ProcessFrameWithStandardMagnification)."""
    fr = T.synth(W, H, 4)
    ref = T.oracle_run(W, H, fr, S=S, standard=std)
    got = T.gpu_run(W, H, fr, S=S, standard=std, mode="stream")
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r, integer_scale=float(S).is_integer())


@pytest.mark.slow
def test_standard_mode_1080p_u8():
    W, H = 1920, 1080
    fr = T.synth(W, H, 2, fmt="u8")
    ref = T.oracle_run(W, H, fr, S=25.0, standard={})
    got = T.gpu_run(W, H, fr, S=25.0, standard={})
    T.assert_close_u8(got[1], ref[1])


def test_processor_standard_mode():
    import torch
    import mm355
    W, H = 64, 48
    fr = T.synth(W, H, 3)
    ref = T.oracle_run(W, H, fr, S=25.0, standard={})
    proc = mm355.MotionMagnificationProcessor(W, H, phase_scale=25.0,
                                              use_pyramid_decomposition=False).Start()
    src = torch.from_numpy(np.stack(fr)).cuda()
    dst = torch.empty_like(src)
    for k in range(3):
        proc.OnRenderImage(src[k], dst[k])
    torch.cuda.synchronize()
    for k in range(1, 3):
        T.assert_close_f32(dst[k].cpu().numpy(), ref[k])
    proc.OnDestroy()


# ---- f3 debug views (ProcessDebugView .cs:234-257) ---------------------------

def _debug_close(got, ref, mag_only):
    """R channel.  |spectrum| view log10(10|z|+1)/4: slope <= 1.09 near |z| = 0
    and the fp32 FFT error is absolute (~1e-7 of the spectrum's peak), so
    max <= 1e-4 and 99.9th percentile <= 1e-5.  The |phase| view's error is
    (FFT absolute error) / |z|, unbounded as |z| -> 0 (where even the sign of a
    tiny imaginary part flips): median <= 5e-6 and 99.9th percentile <= 2e-4
    (measured 1.0e-6 and 5.2e-5 at 200x120).  G = B = 0, alpha 1."""
    assert np.array_equal(got[..., 1:3], np.zeros_like(got[..., 1:3]))
    assert np.all(got[..., 3] == 1.0)
    e = np.abs(got[..., 0].astype(np.float64) - ref[..., 0])
    if mag_only:
        assert e.max() < 1e-4 and np.quantile(e, 0.999) < 1e-5, (e.max(), np.quantile(e, 0.999))
    else:
        assert np.quantile(e, 0.999) < 2e-4 and np.median(e) < 5e-6, (np.quantile(e, 0.999), e.max())


@pytest.mark.gpu
@pytest.mark.parametrize("view", [(True, False), (False, True), (True, True)])
@pytest.mark.parametrize("W,H,edge", [(64, 48, 0), (200, 120, 1)])
def test_debug_view_f32(view, W, H, edge):
    fr = T.synth(W, H, 4)
    ref = T.oracle_run(W, H, fr, edge=edge, debug=view)
    got = T.gpu_run(W, H, fr, edge=edge, mode="stream", debug=view)
    assert np.array_equal(got[0], fr[0])
    for k in range(1, 4):
        _debug_close(got[k], ref[k], view == (True, False))


@pytest.mark.gpu
def test_debug_view_u8_and_state():
    """RGBA8 output (saturated R, alpha 255); after switching the view off the
    magnified output matches the oracle (state followed the input)."""
    import mm355
    import torch
    W, H = 96, 64
    fr = T.synth(W, H, 4, fmt="u8")
    o = O.Oracle(W, H, levels=5, phase_scale=10.0)
    o.set_debug(True, False)
    ref = [o.process(fr[0]), o.process(fr[1])]
    o.set_debug(False, False)
    ref += [o.process(fr[2]), o.process(fr[3])]
    p = mm355.Params.make(levels=5, phase_scale=10.0, show_magnitude=True)
    h = mm355.Handle(W, H, p)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    out = torch.empty_like(dev)
    h.process(dev[0], out[0], mm355.RGBA8)
    h.process(dev[1], out[1], mm355.RGBA8)
    h.set_params(mm355.Params.make(levels=5, phase_scale=10.0))
    h.process(dev[2], out[2], mm355.RGBA8)
    h.process(dev[3], out[3], mm355.RGBA8)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    h.close()
    assert np.array_equal(got[0], fr[0])
    d = np.abs(got[1].astype(np.int32) - ref[1].astype(np.int32))
    assert d.max() <= 1 and np.all(got[1][..., 1:3] == 0) and np.all(got[1][..., 3] == 255)
    for k in (2, 3):
        T.assert_close_u8(got[k], ref[k])


@pytest.mark.gpu
def test_processor_debug_view_toggle():
    """showPhase via the mirror: OnValidate switches the view on and off."""
    import mm355
    W, H = 64, 48
    fr = T.synth(W, H, 3)
    ref = T.oracle_run(W, H, fr[:2], debug=(False, True))
    proc = mm355.MotionMagnificationProcessor(W, H, show_phase=True, phase_scale=10.0)
    proc.Start()
    outs = []
    for f in fr[:2]:
        o = np.empty_like(f)
        proc.OnRenderImage(f, o)
        outs.append(o)
    _debug_close(outs[1], ref[1], False)
    proc.show_phase = False
    proc.OnValidate()
    o = np.empty_like(fr[2])
    proc.OnRenderImage(fr[2], o)
    ref2 = T.oracle_run(W, H, fr[1:3])
    T.assert_close_f32(o, ref2[1])
    proc.OnDestroy()


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,t0,gray", [(64, 48, 0, False), (200, 120, 7, False), (96, 64, 3, True)])
def test_device_synth_matches_oracle(W, H, t0, gray):
    """mm_synth_frames (the bench's input generator) reproduces the oracle's
    synthetic stream: exact except a +-1 step where the double-precision
    sin/cos of device and host libm round v*255+0.5 to different sides."""
    import mm355
    import torch
    h = mm355.Handle(W, H)
    dev = torch.empty((3, H, W, 4), dtype=torch.uint8, device="cuda")
    h.synth(dev, t0, 3, gray=gray)
    torch.cuda.synchronize()
    got = dev.cpu().numpy()
    h.close()
    ref = np.stack([O.synth_frame(W, H, t0 + k, gray=gray) for k in range(3)])
    d = np.abs(got.astype(np.int32) - ref.astype(np.int32))
    assert d.max() <= 1 and (d > 0).mean() < 1e-4, (d.max(), (d > 0).mean())


@pytest.mark.gpu
@pytest.mark.slow
def test_1080p_stream_device_synth_u8():
    """The bench's path end to end: device-generated 1080p RGBA8 stream, one
    multi-frame mm_process_stream call on the default stream (ordered after
    mm_synth_frames), crossing a chunk boundary; against the oracle."""
    import mm355
    import torch
    W, H, n = 1920, 1080, 10
    h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
    h.set_batch(8)
    fr = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    h.synth(fr, 0, n)
    out = torch.empty_like(fr)
    h.process_stream(fr, out, n, mm355.RGBA8)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    h.close()
    O.set_threads(16)
    ref = T.oracle_run(W, H, [O.synth_frame(W, H, t) for t in range(n)], levels=5, S=25.0)
    assert np.array_equal(got[0], ref[0])
    for k in range(1, n):
        T.assert_close_u8(got[k], ref[k])


@pytest.mark.gpu
def test_bench_sharded_ring_equals_single_rank():
    """bench.py's own N>1 path (ShardedStream with prefetch, GpuBackend state
    hand-off via mm_compute_state/mm_set_state) at world 2 over gloo on this
    GPU (the ring state through host memory instead of RCCL): per-frame output
    checksums equal the single-rank run of the same 48 frames bitwise."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(cmd):
        out = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
        assert out.returncode == 0, out.stderr[-2000:]
        return json.loads([l for l in out.stdout.splitlines() if l.startswith('{"')][-1])

    one = run([sys.executable, "bench.py", "--checksum", "--frames-per-step", "12",
               "--steps", "3", "--warmup", "1"])
    two = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", "29541", "bench.py", "--gpus", "2",
               "--dist-backend", "gloo", "--checksum", "--frames-per-step", "6", "--steps", "3",
               "--warmup", "1"])
    assert one["frames"] == two["frames"] == [0, 47]
    assert not one["inputs_wrapped"] and not two["inputs_wrapped"]
    assert one["checksums"] == two["checksums"]


# ---- odd frame sizes (the reference takes any Screen.width/height, .cs:298-302) ----
# N - W odd puts the PadTexture quad half a texel off the grid (.cs:358-381) and
# makes CropTexture sample between two texels; the oracle restates both.
@pytest.mark.parametrize("W,H,L,S,edge,mode", [
    (63, 47, 5, 10.0, 0, "frame"), (63, 48, 5, 25.0, 1, "stream"), (64, 47, 4, 25.0, 0, "frame"),
    (65, 49, 5, 9.7, 0, "stream"), (201, 121, 5, 25.0, 0, "stream"), (33, 17, 3, 10.0, 1, "frame")])
def test_odd_sizes_f32(W, H, L, S, edge, mode):
    fr = T.synth(W, H, 5)
    ref = T.oracle_run(W, H, fr, L, S, edge)
    got = T.gpu_run(W, H, fr, L, S, edge, mode=mode, batch=3)
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r, integer_scale=float(S).is_integer())
        assert np.all(g[..., 3] == 1.0)


def test_odd_size_standard_mode_and_u8():
    W, H = 97, 63
    fr = T.synth(W, H, 4)
    std = dict(apply=True, low=0.05, high=0.4, steep=3.0, sens=1.5, edge=0.8)
    ref = T.oracle_run(W, H, fr, 5, 25.0, standard=std)
    got = T.gpu_run(W, H, fr, 5, 25.0, standard=std)
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r)
    fr8 = T.synth(W, H, 4, fmt="u8")
    ref8 = T.oracle_run(W, H, fr8, 5, 25.0)
    got8 = T.gpu_run(W, H, fr8, 5, 25.0, mode="stream")
    assert np.array_equal(got8[0], fr8[0])
    T.assert_close_u8(np.stack(got8[1:]), np.stack(ref8[1:]))


def test_odd_1919x1079_u8_stream():
    """1080p minus one pixel each way (N = 2048, both offsets fractional)."""
    W, H = 1919, 1079
    fr = T.synth(W, H, 3, fmt="u8")
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    got = T.gpu_run(W, H, fr, 5, 25.0, mode="stream")
    assert np.array_equal(got[0], fr[0])
    T.assert_close_u8(np.stack(got[1:]), np.stack(ref[1:]))




# ---- k_cols_tail: the packed block's last frames as one-frame workgroups ----
@pytest.mark.parametrize("W,H,n,batch,tail", [(1920, 1080, 50, 25, "12"), (640, 360, 60, 30, "25"),
                                              (256, 256, 72, 24, "50")])
def test_k2_tail_bitwise_equals_single_launch(W, H, n, batch, tail, monkeypatch):
    """Frames handed from k_cols's packed block to k_cols_tail (which restarts
    from the previous input frame) give bitwise the single-launch outputs; the
    stream spans several batches, so the state the tail writes is used next."""
    fr = T.synth(W, H, n, fmt="u8")
    monkeypatch.setenv("MM_K2_TAIL", "0")
    a = T.gpu_run(W, H, fr, 5, 25.0, mode="stream", batch=batch)
    monkeypatch.setenv("MM_K2_TAIL", tail)
    b = T.gpu_run(W, H, fr, 5, 25.0, mode="stream", batch=batch)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


# ---- round 4: K2 staging area and the two-band op -----------------------------
@pytest.mark.parametrize("W,H,n,batch", [(1920, 1080, 40, 20), (640, 360, 30, 10), (200, 120, 20, 7)])
def test_k2_dedicated_staging_bitwise_equals_aliased(W, H, n, batch, monkeypatch):
    """k_cols with its own Q staging area in LDS (MM_K2_STGD=1: 2 barriers per
    frame fewer, where it fits beside two workgroups per CU; opt-in) gives
    bitwise the outputs of the default staging that aliases the FFT exchange
    buffers."""
    fr = T.synth(W, H, n, fmt="u8")
    monkeypatch.setenv("MM_K2_STGD", "0")
    a = T.gpu_run(W, H, fr, 5, 25.0, mode="stream", batch=batch)
    monkeypatch.setenv("MM_K2_STGD", "1")
    b = T.gpu_run(W, H, fr, 5, 25.0, mode="stream", batch=batch)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("W,H,S", [(256, 192, 25.0), (320, 200, 9.7)])
def test_two_band_op_l6_vs_oracle(W, H, S):
    """L = 6 (neighbouring middle bands overlap: MM_K2_PYR_TAB2, the branch-
    free two-band op) against the oracle's per-level loop at the §8c bars,
    frame calls and one stream call."""
    fr = T.synth(W, H, 5)
    ref = T.oracle_run(W, H, fr, 6, S)
    for mode in ("frame", "stream"):
        got = T.gpu_run(W, H, fr, 6, S, mode=mode, batch=3)
        assert np.array_equal(got[0], fr[0])
        for k in range(1, 5):
            T.assert_close_f32(got[k], ref[k], integer_scale=float(S).is_integer())


def test_two_band_op_tail_and_batch_bitwise(monkeypatch):
    """The two-band kernel across launch shapes: 1080p L = 6, a 30-frame
    stream in one batch without and with k_cols_tail (40 %: the packed
    block's last 12 frames) and in one-frame calls, all bitwise equal."""
    W, H = 1920, 1080
    fr = T.synth(W, H, 30, fmt="u8")
    monkeypatch.setenv("MM_K2_TAIL", "0")
    a = T.gpu_run(W, H, fr, 6, 25.0, mode="stream", batch=30)
    monkeypatch.setenv("MM_K2_TAIL", "40")
    b = T.gpu_run(W, H, fr, 6, 25.0, mode="stream", batch=30)
    monkeypatch.delenv("MM_K2_TAIL")
    c = T.gpu_run(W, H, fr, 6, 25.0, mode="frame", batch=1)
    for x, y, z in zip(a, b, c):
        assert np.array_equal(x, y) and np.array_equal(x, z)


# ---- round 4: the packed block entirely in k_cols_tail (MM_K2_PKALL) --------------
@pytest.mark.parametrize("W,H,L,n,batch", [(1920, 1080, 5, 30, 30), (1920, 1080, 6, 30, 30),
                                           (640, 360, 5, 60, 25), (2100, 64, 6, 50, 25)])
def test_k2_packed_all_in_tail_bitwise(W, H, L, n, batch, monkeypatch):
    """Batches >= 24 frames with block 0 (the packed group) out of k_cols and
    every one of its frames a k_cols_tail workgroup (frame 0 primed from the
    state slot, the others from the previous input frame): bitwise the
    outputs with block 0 in k_cols and of one-frame calls (2100 x 64: N =
    4096).  Opt-in (MM_K2_PKALL=1): same-call no faster at the default shapes."""
    fr = T.synth(W, H, n, fmt="u8")
    monkeypatch.setenv("MM_K2_PKALL", "0")
    a = T.gpu_run(W, H, fr, L, 25.0, mode="stream", batch=batch)
    monkeypatch.setenv("MM_K2_PKALL", "1")
    b = T.gpu_run(W, H, fr, L, 25.0, mode="stream", batch=batch)
    monkeypatch.delenv("MM_K2_PKALL")
    c = T.gpu_run(W, H, fr, L, 25.0, mode="frame", batch=1)
    for x, y, z in zip(a, b, c):
        assert np.array_equal(x, y) and np.array_equal(x, z)


# ---- K2's generic per-bin op (MM_MODE_PYRAMID instance) ---------------------------
@pytest.mark.parametrize("W,H,L,S,notab", [(200, 120, 7, 25.0, False), (160, 96, 8, 9.7, False),
                                           (200, 120, 5, 25.0, True)])
def test_k2_generic_op_vs_oracle(W, H, L, S, notab, monkeypatch):
    """Band layouts where three middle bands share bins (L >= 7 at the default
    0.05 / 0.45) and MM_K2_NOTAB=1 run K2's generic per-bin op: against the
    oracle in a stream and in one-frame calls, which agree bitwise."""
    if notab:
        monkeypatch.setenv("MM_K2_NOTAB", "1")
    fr = T.synth(W, H, 5)
    ref = T.oracle_run(W, H, fr, L, S)
    st = T.gpu_run(W, H, fr, L, S, mode="stream", batch=3)
    fm = T.gpu_run(W, H, fr, L, S, mode="frame")
    assert np.array_equal(st[0], fr[0])
    for k in range(1, 5):
        T.assert_close_f32(st[k], ref[k], integer_scale=float(S).is_integer())
        assert np.array_equal(st[k], fm[k])


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_c2_1080p_long_stream_vs_oracle():
    """BASELINE C2 over a 96-frame stream in batches of 40 (every K2 launch
    shape of the bench: packed-block tail, second-half tails, the prime from
    the state slot at each batch boundary) against the oracle frame by frame,
    at the RGBA8 bar (max 1 LSB on <= 0.1 % of values)."""
    W, H, n = 1920, 1080, 96
    O.set_threads(16)
    fr = T.synth(W, H, n, fmt="u8")
    got = T.gpu_run(W, H, fr, 5, 25.0, mode="stream", batch=40)
    o = O.Oracle(W, H, levels=5, phase_scale=25.0)
    off = 0
    for k in range(n):
        ref = o.process(fr[k])
        if k == 0:
            assert np.array_equal(got[0], fr[0])
            continue
        T.assert_close_u8(got[k], ref)
        off += int((got[k] != ref).sum())
    assert off <= 1e-3 * (n - 1) * W * H * 4


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_c3_2160p_stream_with_tails_vs_oracle():
    """BASELINE C3 (3840x2160, L = 6: the two-band op at N = 4096) as one
    30-frame batch, so K2 runs its packed-block and second-half tails,
    against the oracle frame by frame at the RGBA8 bar."""
    W, H, n = 3840, 2160, 30
    O.set_threads(16)
    fr = T.synth(W, H, n, fmt="u8")
    got = T.gpu_run(W, H, fr, 6, 25.0, mode="stream", batch=30)
    o = O.Oracle(W, H, levels=6, phase_scale=25.0)
    for k in range(n):
        ref = o.process(fr[k])
        if k == 0:
            assert np.array_equal(got[0], fr[0])
        else:
            T.assert_close_u8(got[k], ref)
