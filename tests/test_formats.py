"""The reference camera's own frame formats (ABI 10).

The component sits on a camera that renders HDR (Assets/Scenes/SampleScene.unity:663,
m_HDR: 1) in Linear colour space (ProjectSettings/ProjectSettings.asset:50), so
OnRenderImage's source (.cs:101) is a linear half-float target (values may
exceed 1) that .cs:109 blits into ARGBFloat; an LDR camera's 8-bit target is
sRGB, sampled as linear light and encoded on write.  MM_RGBA16F and
MM_RGBA8_SRGB take those frames directly.

Checks, each through the C-ABI on the HIP path:
* against the oracle (oracle/mm_ref.c mm_ref_process_f16 / _srgb8: exact
  decode, the fp32 pipeline, the destination's rounding) at 1080p, frame calls
  and a stream, with HDR values above 1 in the half input;
* structurally: the RGBA16F output is bitwise the RGBA32F path's output on the
  decoded frames rounded to half (round to nearest even), and the sRGB output
  bitwise the RGBA32F path's output encoded with the exact thresholds — the
  formats change only the two ends of the pipeline;
* odd sizes (k_compose_odd), the steerable extension and the debug views take
  them too; the first frame passes through bitwise.

Bars: RGBA16F decoded outputs within 1e-4 + one half ulp (2^-11 at [0.5, 1))
of the oracle's, differing halves on <= 1 % of values; sRGB8 the RGBA8 bar
(+-1 code on <= 0.1 % of values); first frame bitwise.
"""
import numpy as np
import pytest

import mmtest as T
import oracle_py as O

pytestmark = pytest.mark.gpu

HALF_TOL = 1e-4 + 2.0 ** -11
HALF_FRAC = 1e-2


def _hdr_frames(W, H, n, gain=1.6):
    """Synthetic stream frames as linear half with highlights above 1."""
    out = []
    for f in T.synth(W, H, n):
        g = f.copy()
        g[..., :3] *= np.float32(gain)
        out.append(g.astype(np.float16))
    return out


def _assert_close_f16(got, ref):
    a, b = got.astype(np.float64), ref.astype(np.float64)
    assert np.abs(a - b).max() <= HALF_TOL, np.abs(a - b).max()
    assert (got.view(np.uint16) != ref.view(np.uint16)).mean() <= HALF_FRAC


def _srgb_encode(v):
    """The exact encode of saturated linear values (largest b with v >= thr[b])."""
    _, thr = O.srgb_tables()
    return (np.searchsorted(thr, np.clip(v, 0.0, 1.0), side="right") - 1).astype(np.uint8)


def _srgb_decode(u8):
    dec, _ = O.srgb_tables()
    f = dec[u8]
    f[..., 3] = u8[..., 3].astype(np.float32) / np.float32(255.0)
    return f


@pytest.mark.timeout(600)
def test_rgba16f_1080p_vs_oracle():
    import mm355
    W, H, n = 1920, 1080, 5
    O.set_threads(16)
    fr = _hdr_frames(W, H, n)
    assert max(float(f[..., :3].max()) for f in fr) > 1.2            # HDR highlights
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    for mode, batch in (("frame", 1), ("stream", 8)):
        got = T.gpu_run(W, H, fr, 5, 25.0, mode=mode, batch=batch, fmt=mm355.RGBA16F)
        assert np.array_equal(got[0].view(np.uint16), fr[0].view(np.uint16))
        for k in range(1, n):
            _assert_close_f16(got[k], ref[k])


@pytest.mark.timeout(600)
def test_srgb8_1080p_vs_oracle():
    import mm355
    W, H, n = 1920, 1080, 5
    O.set_threads(16)
    fr = T.synth(W, H, n, fmt="u8")
    o = O.Oracle(W, H, levels=5, phase_scale=25.0)
    ref = [o.process_srgb8(f) for f in fr]
    for mode, batch in (("frame", 1), ("stream", 8)):
        got = T.gpu_run(W, H, fr, 5, 25.0, mode=mode, batch=batch, fmt=mm355.RGBA8_SRGB)
        assert np.array_equal(got[0], fr[0])
        for k in range(1, n):
            T.assert_close_u8(got[k], ref[k])
            assert np.all(got[k][..., 3] == 255)


@pytest.mark.parametrize("W,H,extra", [
    (1920, 1080, {}),                                   # K1 -> K2 -> fused K34
    (97, 63, {}),                                       # odd: general K1 taps, k_compose_odd
    (640, 360, {"mode": 1}),                            # standard mode (f1)
    (256, 192, {"mode": 2, "orientations": 4}),         # steerable (f2): K4 after the band kernels
    (128, 96, {"show_magnitude": 1, "show_phase": 1}),  # debug views (f3): k_dbg_out
])
def test_formats_equal_f32_path_at_both_ends(W, H, extra):
    """RGBA16F = half(RGBA32F path on the decoded frames); RGBA8_SRGB =
    encode(RGBA32F path on the decoded frames): bitwise, every frame, so the
    formats touch only the decode on load and the rounding on store."""
    import mm355
    n = 4
    hdr = _hdr_frames(W, H, n)
    f32 = T.gpu_run(W, H, [f.astype(np.float32) for f in hdr], 5, 25.0, mode="stream", extra=extra)
    f16 = T.gpu_run(W, H, hdr, 5, 25.0, mode="stream", extra=extra, fmt=mm355.RGBA16F)
    assert np.array_equal(f16[0].view(np.uint16), hdr[0].view(np.uint16))
    for k in range(1, n):
        assert np.array_equal(f16[k].view(np.uint16), f32[k].astype(np.float16).view(np.uint16)), k
    u8 = T.synth(W, H, n, fmt="u8")
    f32 = T.gpu_run(W, H, [_srgb_decode(f) for f in u8], 5, 25.0, mode="stream", extra=extra)
    s8 = T.gpu_run(W, H, u8, 5, 25.0, mode="stream", extra=extra, fmt=mm355.RGBA8_SRGB)
    assert np.array_equal(s8[0], u8[0])
    for k in range(1, n):
        want = _srgb_encode(f32[k])
        want[..., 3] = 255
        assert np.array_equal(s8[k], want), (k, int((s8[k] != want).sum()))


def test_processor_takes_half_and_srgb_frames():
    """The Python mirror picks the format from the dtype (float16) or the
    component's colour-space switch (srgb=True for 8-bit targets)."""
    import torch
    import mm355
    W, H, n = 64, 48, 3
    hdr = _hdr_frames(W, H, n)
    u8 = T.synth(W, H, n, fmt="u8")
    for frames, kw, fmt in ((hdr, {}, mm355.RGBA16F), (u8, {"srgb": True}, mm355.RGBA8_SRGB)):
        want = T.gpu_run(W, H, frames, 5, 25.0, mode="frame", fmt=fmt)
        p = mm355.MotionMagnificationProcessor(W, H, phase_scale=25.0, **kw).Start()
        src = torch.from_numpy(np.stack(frames)).cuda()
        dst = torch.empty_like(src)
        for k in range(n):
            p.OnRenderImage(src[k], dst[k])
        torch.cuda.synchronize()
        got = dst.cpu().numpy()
        p.OnDestroy()
        for k in range(n):
            assert np.array_equal(got[k].view(np.uint8), want[k].view(np.uint8))
