"""MM_MODE_STEERABLE (extension f2): the spec oracle's
identities on CPU, and the HIP path against the spec on the GPU.

Parity against the reference is unpinned (no reference implementation exists,
oracle/steerable_ref.py); what is pinned: at S = 0 the whole chain equals the
reference pipeline (C oracle) exactly up to rounding, and the HIP path equals
the float64 spec at every S within the tolerances below.
"""
import os
import sys

import numpy as np
import pytest

import mmtest as T
import np_twin
import oracle_py as O

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import steerable_ref as SR  # noqa: E402


def frames(W, H, n):
    return [O.synth_frame(W, H, t).astype(np.float32) / np.float32(255) for t in range(n)]


# ---- spec identities (CPU) ----------------------------------------------------

@pytest.mark.parametrize("Oo", [4, 6, 8])
def test_angular_partition_and_mirror(Oo):
    N = 64
    a = SR.angular_masks(N, Oo)
    assert np.abs(a.sum(0) - 1).max() < 1e-12
    idx = (N - np.arange(N)) % N
    for o in range(Oo):
        assert np.abs(a[o][np.ix_(idx, idx)] - a[(o + Oo // 2) % Oo]).max() < 1e-12


@pytest.mark.parametrize("filt", [SR.FILTER_DIFF, SR.FILTER_IIR])
def test_spec_s0_is_reference_pipeline(filt):
    W, H = 64, 48
    fr = [f.astype(np.float64) for f in frames(W, H, 3)]
    r = SR.SteerableRef(W, H, levels=5, phase_scale=0.0, orientations=8, filt=filt)
    outs = [r.process(f) for f in fr]
    assert np.array_equal(outs[0], fr[0])
    ref = np_twin.process_frame(fr[2], fr[1], 5, 0.05, 0.45, 0.0)
    assert np.abs(outs[2] - ref).max() < 1e-12


def test_spec_static_scene_unchanged_by_diff():
    """DIFF on a static scene: P = 0 everywhere, output = S=0 output."""
    W, H = 64, 48
    f = frames(W, H, 1)[0].astype(np.float64)
    a = SR.SteerableRef(W, H, phase_scale=25.0, orientations=4)
    b = SR.SteerableRef(W, H, phase_scale=0.0, orientations=4)
    for _ in range(3):
        oa, ob = a.process(f), b.process(f)
    assert np.abs(oa - ob).max() < 1e-12


# ---- HIP path (GPU) -------------------------------------------------------------

def gpu_steer(W, H, fr, levels=5, S=10.0, Oo=8, filt=0, rl=0.05, rh=0.4, edge=0, apply=True,
              batch=4):
    import mm355
    import torch
    p = mm355.Params.make(levels=levels, phase_scale=S, edge_mode=edge, apply_magnification=apply,
                          mode=mm355.MODE_STEERABLE, orientations=Oo, temporal_filter=filt,
                          iir_low=rl, iir_high=rh)
    h = mm355.Handle(W, H, p)
    h.set_batch(batch)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    out = torch.empty_like(dev)
    h.process_stream(dev, out, len(fr), mm355.RGBA32F)
    torch.cuda.synchronize()
    res = out.cpu().numpy()
    h.close()
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("Oo,filt,W,H", [(8, 0, 96, 64), (4, 1, 96, 64), (8, 0, 95, 63), (6, 1, 96, 63)])
def test_gpu_s0_equals_reference_oracle(Oo, filt, W, H):
    fr = frames(W, H, 4)
    got = gpu_steer(W, H, fr, S=0.0, Oo=Oo, filt=filt)
    ref = T.oracle_run(W, H, fr, levels=5, S=0.0)
    assert np.array_equal(got[0], fr[0])
    T.assert_close_f32(got[1:], np.stack(ref[1:]))


def _close_spec(got, ref):
    """fp32 HIP vs float64 spec: amplified local phase S*P (P wraps at +-pi
    where the two sides may fall differently): 99.9th percentile <= 2e-4,
    RMSE <= 2e-5."""
    e = np.abs(got.astype(np.float64) - ref)
    assert np.quantile(e, 0.999) < 2e-4 and np.sqrt((e ** 2).mean()) < 2e-5, (
        e.max(), np.quantile(e, 0.999), np.sqrt((e ** 2).mean()))


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,Oo,filt,S,edge", [(64, 48, 8, 0, 10.0, 0), (96, 64, 4, 1, 25.0, 0),
                                                 (64, 48, 6, 1, 9.7, 1), (200, 120, 8, 0, 25.0, 0),
                                                 # odd sizes: the quad half a texel off the grid
                                                 (63, 47, 8, 0, 10.0, 0), (97, 63, 4, 1, 25.0, 1),
                                                 (65, 48, 6, 0, 9.7, 0), (64, 49, 8, 1, 10.0, 1),
                                                 (199, 121, 8, 0, 25.0, 0),
                                                 # tiny canvases (N = 32, 16): one wave per transform
                                                 (31, 16, 8, 1, 10.0, 0), (15, 9, 4, 0, 10.0, 1)])
def test_gpu_matches_spec(W, H, Oo, filt, S, edge):
    n = 5
    fr = frames(W, H, n)
    got = gpu_steer(W, H, fr, S=S, Oo=Oo, filt=filt, edge=edge)
    r = SR.SteerableRef(W, H, levels=5, phase_scale=S, orientations=Oo, filt=filt, edge=edge)
    ref = [r.process(f.astype(np.float64)) for f in fr]
    assert np.array_equal(got[0], fr[0])
    for k in range(1, n):
        _close_spec(got[k], ref[k])


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(64, 48), (63, 47)])
def test_gpu_chunked_and_state_handoff(W, H):
    """Batch boundaries (mm_set_batch 4) and the DIFF state hand-off:
    a second handle seeded with mm_compute_state(frame k-1) continues the
    stream bitwise; mm_get_state/mm_set_state carry the IIR state."""
    import mm355
    import torch
    n = 11
    fr = frames(W, H, n)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    for filt in (0, 1):
        p = mm355.Params.make(levels=5, phase_scale=10.0, mode=mm355.MODE_STEERABLE,
                              orientations=8, temporal_filter=filt)
        a = mm355.Handle(W, H, p)
        a.set_batch(4)
        full = torch.empty_like(dev)
        a.process_stream(dev, full, n, mm355.RGBA32F)
        b = mm355.Handle(W, H, p)
        b.set_batch(4)
        part = torch.empty_like(dev)
        b.process_stream(dev[:6], part[:6], 6, mm355.RGBA32F)
        st = torch.empty(b.state_bytes, dtype=torch.uint8, device="cuda")
        b.get_state(st)
        c = mm355.Handle(W, H, p)
        c.set_batch(4)
        c.set_state(st)
        c.process_stream(dev[6:], part[6:], n - 6, mm355.RGBA32F)
        torch.cuda.synchronize()
        assert torch.equal(full, part), filt
        if filt == 0:
            d = mm355.Handle(W, H, p)
            d.set_batch(4)
            st2 = torch.empty(d.state_bytes, dtype=torch.uint8, device="cuda")
            d.compute_state(dev[5], mm355.RGBA32F, st2)
            d.set_state(st2)
            o = torch.empty_like(dev[6:])
            d.process_stream(dev[6:], o, n - 6, mm355.RGBA32F)
            torch.cuda.synchronize()
            assert torch.equal(o, full[6:])
            d.close()
        for h in (a, b, c):
            h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("filt", [0, 1])
def test_gpu_frames_per_launch_bitwise(filt):
    """k_sb_rows runs 1, 2 or (DIFF) 4 frames per launch (MM_SB_NF, read at
    mm_create), carrying the band state from one frame to the next in
    registers, and k_sb_cols the band columns of MM_SB_CF frames per launch:
    the same expressions in the same order, so the outputs and the final state
    are bitwise equal for every grouping, including batches (11 of 13 frames)
    whose column chunks (8 + 3, 2 + 1) leave a pair and a single frame."""
    import os
    import mm355
    import torch
    W, H, n = 200, 120, 13
    fr = frames(W, H, n)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    p = mm355.Params.make(levels=5, phase_scale=10.0, mode=mm355.MODE_STEERABLE,
                          orientations=8, temporal_filter=filt)
    combos = [("1", "2"), ("2", "2"), ("2", "8"), ("2", "4")] + ([("4", "8")] if filt == 0 else [])
    res = {}
    old = {k: os.environ.get(k) for k in ("MM_SB_NF", "MM_SB_CF")}
    try:
        for nf, cf in combos:
            os.environ["MM_SB_NF"] = nf
            os.environ["MM_SB_CF"] = cf
            h = mm355.Handle(W, H, p)
            h.set_batch(11)
            out = torch.empty_like(dev)
            h.process_stream(dev, out, n, mm355.RGBA32F)
            st = torch.empty(h.state_bytes, dtype=torch.uint8, device="cuda")
            h.get_state(st)
            torch.cuda.synchronize()
            res[(nf, cf)] = (out.cpu(), st.cpu())
            h.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ref = res[("1", "2")]
    for c in combos[1:]:
        assert torch.equal(res[c][0], ref[0]), c
        assert torch.equal(res[c][1], ref[1]), c


@pytest.mark.gpu
def test_c1_literal_256_gray_L3_O4_S10_32_frames():
    """BASELINE configs[0] literally: 256 x 256 gray, 3 levels,
    4 orientations, PhaseScale 10, a 32-frame clip, in MM_MODE_STEERABLE on
    the GPU.  L = 3 makes the one middle band's centre 0/0 = NaN
    (PyramidOperations.compute:59-64, :71), so its mask is zero everywhere and
    no subband carries anything: the output must be the spec's (float64), the
    reference restatement's (C oracle, O = 1) and the GPU pyramid path's, all
    within the fp32 bar, frame by frame."""
    W = H = 256
    n = 32
    fr = [f.astype(np.float32) / np.float32(255) for f in T.synth(W, H, n, gray=True, fmt="u8")]
    got = gpu_steer(W, H, fr, levels=3, S=10.0, Oo=4, batch=8)
    r = SR.SteerableRef(W, H, levels=3, phase_scale=10.0, orientations=4)
    spec = [r.process(f.astype(np.float64)) for f in fr]
    ref = T.oracle_run(W, H, fr, 3, 10.0)
    pyr = T.gpu_run(W, H, fr, 3, 10.0, mode="stream", batch=8)
    assert np.array_equal(got[0], fr[0])
    for k in range(1, n):
        T.assert_close_f32(got[k], spec[k].astype(np.float32))
        T.assert_close_f32(got[k], ref[k])
        T.assert_close_f32(got[k], pyr[k])
        assert np.abs(got[k][..., 0] - got[k][..., 1]).max() < 1e-6     # gray stays gray


@pytest.mark.gpu
def test_odd_size_steerable_set_params():
    """mm_set_params on an odd-size handle accepts the steerable
    mode (mm_create does since round 5).  63 x 47: a pyramid handle switched
    to steerable O = 4, then its phase scale changed, equals a handle created
    steerable on the same frames (bitwise: the switch passes one frame through
    and seeds the local phases, as a fresh handle's first frame does)."""
    import mm355
    import torch
    W, H = 63, 47
    fr = frames(W, H, 8)
    dev = torch.from_numpy(np.stack(fr)).cuda()
    kw = dict(mode=mm355.MODE_STEERABLE, orientations=4)
    a = mm355.Handle(W, H, mm355.Params.make(phase_scale=10.0))
    oa = torch.empty_like(dev)
    a.process_stream(dev[:3], oa[:3], 3, mm355.RGBA32F)
    a.set_params(mm355.Params.make(phase_scale=10.0, **kw))
    a.process_stream(dev[3:6], oa[3:6], 3, mm355.RGBA32F)
    a.set_params(mm355.Params.make(phase_scale=25.0, **kw))
    a.process_stream(dev[6:], oa[6:], 2, mm355.RGBA32F)
    b = mm355.Handle(W, H, mm355.Params.make(phase_scale=10.0, **kw))
    ob = torch.empty_like(dev)
    b.process_stream(dev[3:6], ob[3:6], 3, mm355.RGBA32F)
    b.set_params(mm355.Params.make(phase_scale=25.0, **kw))
    b.process_stream(dev[6:], ob[6:], 2, mm355.RGBA32F)
    torch.cuda.synchronize()
    ga, gb = oa.cpu().numpy(), ob.cpu().numpy()
    a.close()
    b.close()
    assert np.array_equal(ga[3], fr[3])                  # the switch frame passes through
    assert np.array_equal(ga[3:], gb[3:])
    assert not np.array_equal(ga[6], ga[3])
