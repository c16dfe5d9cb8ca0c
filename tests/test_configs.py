"""BASELINE.json configurations at full size on the HIP path (SURVEY.md §8(d)
configs C2, C3, C5), plus parameter hot-reload across modes.

  C2  1920x1080 RGBA, L=5, 8-orientation steerable extension, S=25 (DIFF, IIR)
      against the float64 spec oracle (oracle/steerable_ref.py)
  C3  3840x2160 RGBA, L=6: O=1 RGBA8 stream across batch boundaries against
      the reference restatement; O=8 steerable: first frame bitwise, output
      finite, S=25 within the spec tolerance of oracle/steerable_ref.py on a
      2-frame run, and S=0 equal to the reference restatement (the identity
      that pins the extension to the reference's stages)
  C5  independent replica streams: bench.py --mode replicas at world 2 over
      gloo on one GPU, each rank's per-frame checksums equal to a single-rank
      run of that rank's stream
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import mmtest as T
import oracle_py as O
from test_steerable import _close_spec, gpu_steer

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "oracle"))
import steerable_ref as SR  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _f32(W, H, n, t0=0):
    return [O.synth_frame(W, H, t0 + t).astype(np.float32) / np.float32(255) for t in range(n)]


@pytest.mark.slow
@pytest.mark.parametrize("filt", [SR.FILTER_DIFF, SR.FILTER_IIR])
def test_c2_steerable_o8_1080p_vs_spec(filt):
    """C2 at full size: 1920x1080, L=5, O=8, S=25, 3 frames (passthrough + 2
    magnified; batch 2 so the second magnified frame starts a new batch)."""
    W, H, n = 1920, 1080, 3
    fr = _f32(W, H, n)
    got = gpu_steer(W, H, fr, levels=5, S=25.0, Oo=8, filt=filt, batch=2)
    r = SR.SteerableRef(W, H, levels=5, phase_scale=25.0, orientations=8, filt=filt)
    ref = [r.process(f.astype(np.float64)) for f in fr]   # frame 0 seeds the state
    assert np.array_equal(got[0], fr[0])
    for k in range(1, n):
        _close_spec(got[k], ref[k])


@pytest.mark.slow
def test_steerable_o8_1919x1079_vs_spec():
    """An odd full-size screen in the steerable extension (round 5: odd W and
    H accepted): 1919x1079 (N = 2048, the quad half a texel off the grid in
    both directions), L=5, O=8 DIFF, S=25, 3 frames in batches of 2."""
    W, H, n = 1919, 1079, 3
    fr = _f32(W, H, n)
    got = gpu_steer(W, H, fr, levels=5, S=25.0, Oo=8, filt=SR.FILTER_DIFF, batch=2)
    r = SR.SteerableRef(W, H, levels=5, phase_scale=25.0, orientations=8, filt=SR.FILTER_DIFF)
    ref = [r.process(f.astype(np.float64)) for f in fr]
    assert np.array_equal(got[0], fr[0])
    for k in range(1, n):
        _close_spec(got[k], ref[k])


@pytest.mark.slow
def test_c3_2160p_rgba8_stream_across_batches():
    """C3 geometry (N = 4096), reference semantics: an RGBA8 stream of 6 frames
    in batches of 4 (K2's state stored and reloaded at the boundary) against
    the reference restatement."""
    W, H, n = 3840, 2160, 6
    O.set_threads(16)
    fr = [O.synth_frame(W, H, t) for t in range(n)]
    ref = T.oracle_run(W, H, fr, levels=6, S=25.0)
    got = T.gpu_run(W, H, fr, 6, 25.0, mode="stream", batch=4)
    assert np.array_equal(got[0], fr[0])
    for k in range(1, n):
        T.assert_close_u8(got[k], ref[k])


@pytest.mark.slow
@pytest.mark.timeout(600)   # the float64 spec at 4096^2: ~1 min on 16 threads
def test_c3_2160p_steerable_o8():
    """C3 with the 8-orientation extension (L=6: 4 middle levels x 4 band
    pairs + residual = 17 complex IFFTs of 4096^2 per frame): first frame
    bitwise, finite outputs in [0, 1], S = 25 within the spec tolerance of
    oracle/steerable_ref.py on the 2-frame run; at S = 0 the extension reproduces the
    reference pipeline (sum of the orientation masks = 1), checked against the
    reference restatement."""
    W, H, n = 3840, 2160, 2
    O.set_threads(16)
    fr = _f32(W, H, n)
    got = gpu_steer(W, H, fr, levels=6, S=25.0, Oo=8, filt=SR.FILTER_DIFF, batch=2)
    assert np.array_equal(got[0], fr[0])
    assert np.isfinite(got[1]).all() and got[1].min() >= 0.0 and got[1].max() <= 1.0
    # S = 25 against the float64 spec over the 2-frame run (16 subbands of
    # 4096^2, formed one at a time; FFTs on 16 threads)
    SR.WORKERS = 16
    try:
        r = SR.SteerableRef(W, H, levels=6, phase_scale=25.0, orientations=8, filt=SR.FILTER_DIFF)
        r.process(fr[0].astype(np.float64))
        _close_spec(got[1], r.process(fr[1].astype(np.float64)))
    finally:
        SR.WORKERS = 1
    g0 = gpu_steer(W, H, fr, levels=6, S=0.0, Oo=8, filt=SR.FILTER_DIFF, batch=2)
    ref = T.oracle_run(W, H, fr, levels=6, S=0.0)
    T.assert_close_f32(g0[1], ref[1])


def test_mode_switch_steerable_to_pyramid():
    """OnValidate across modes: orientations 8 -> 1 mid-stream.  The
    pyramid frame after the switch is magnified against the last input frame
    (.cs:142), exactly as a fresh pyramid handle seeded with that frame's
    state."""
    import mm355
    import torch
    W, H, n = 96, 64, 6
    fr = _f32(W, H, n)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    steer = mm355.Params.make(levels=5, phase_scale=10.0, mode=mm355.MODE_STEERABLE,
                              orientations=8)
    pyr = mm355.Params.make(levels=5, phase_scale=10.0)
    h = mm355.Handle(W, H, steer)
    out = torch.empty_like(dev)
    h.process_stream(dev[:3], out[:3], 3, mm355.RGBA32F)
    h.set_params(pyr)
    assert h.state_bytes == (h.N // 2 + 1) * (H + (H & 1)) * 8   # follows the mode (G, ABI 8)
    h.process_stream(dev[3:], out[3:], n - 3, mm355.RGBA32F)
    ref = mm355.Handle(W, H, pyr)
    st = torch.empty(ref.state_bytes, dtype=torch.uint8, device="cuda")
    ref.compute_state(dev[2], mm355.RGBA32F, st)
    ref.set_state(st)
    o2 = torch.empty_like(dev[3:])
    ref.process_stream(dev[3:], o2, n - 3, mm355.RGBA32F)
    torch.cuda.synchronize()
    assert torch.equal(out[3:], o2)
    # and back: the steerable state restarts (first steerable frame passes through)
    h.set_params(steer)
    o3 = torch.empty_like(dev[:1])
    h.process_stream(dev[5:6], o3, 1, mm355.RGBA32F)
    torch.cuda.synchronize()
    assert torch.equal(o3[0], dev[5])
    h.close()
    ref.close()


def test_steerable_state_size_follows_filter():
    """DIFF carries one phase plane per band, IIR three."""
    import mm355
    W, H = 64, 48
    p = mm355.Params.make(levels=5, mode=mm355.MODE_STEERABLE, orientations=8, temporal_filter=0)
    h = mm355.Handle(W, H, p)
    nb = 3 * 4   # 3 middle levels x O/2 band pairs
    plane = nb * (H + 4) * (W + 4) * 4
    assert h.state_bytes == plane
    h.set_params(mm355.Params.make(levels=5, mode=mm355.MODE_STEERABLE, orientations=8,
                                   temporal_filter=1))
    assert h.state_bytes == 3 * plane
    h.close()


def test_batch_size_does_not_change_results():
    """mm_set_batch only regroups launches: batch 1, 3 and 16 give bitwise
    equal streams."""
    W, H = 200, 120
    fr = T.synth(W, H, 7, fmt="u8")
    outs = [T.gpu_run(W, H, fr, 5, 25.0, mode="stream", batch=b) for b in (1, 3, 16)]
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert np.array_equal(x, y)


def _bench_checksums(args, world):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONUNBUFFERED="1")
    if world > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
               "--master-port", str(29500 + os.getpid() % 1000), os.path.join(ROOT, "bench.py")]
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
    r = subprocess.run(cmd + args, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    return json.loads(line)


def test_bench_replicas_gloo_world2():
    """C5 rehearsal at its workload size, 1920x1080: bench.py --mode replicas
    at world 2 (gloo, both ranks on this GPU): rank r runs its own stream (seed
    base + r); each rank's per-frame output checksums equal a single-rank run
    of that stream."""
    common = ["--mode", "replicas", "--dist-backend", "gloo", "--checksum", "--steps", "2",
              "--warmup", "1", "--frames-per-step", "6", "--width", "1920", "--height", "1080"]
    both = _bench_checksums(common + ["--gpus", "2"], 2)["checksums_by_rank"]
    for r in (0, 1):
        one = _bench_checksums(common + ["--gpus", "1", "--replica-index", str(r)], 1)
        assert one["checksums_by_rank"]["0"] == both[str(r)], r
    assert both["0"] != both["1"]   # different streams
