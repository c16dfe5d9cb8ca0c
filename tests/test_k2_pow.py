"""K2's power form of the phase factor (k_cols SP > 0: an integer phase scale
with a compiled instance, |S| 25 and 10 at N >= 2048; opt-in, MM_K2_POW=1,
measured slower than the atan2 form):
e^{i S wrap(arg p - arg c)} = z^S with z = p conj(c) / |p||c|
(PyramidPhaseDifference.compute:47-54, 92-98: for integer S the wrap's
multiple of 2 pi drops out).  Against the atan2 + sin/cos form of the same
kernel (the default) and against the oracle's literal atan2f path: one-band
(L = 5) and two-band (L = 6) layouts, S < 0, the stream's batch, tail and
packed-group paths, and the 1080p RGBA8 bench geometry."""
import os

import numpy as np
import pytest

import mmtest as T

pytestmark = pytest.mark.gpu


def _run(W, H, fr, S, atan2_form, L=5, mode="stream", batch=3):
    """atan2_form: the default; else MM_K2_POW=1 (read at mm_create)."""
    old = os.environ.pop("MM_K2_POW", None)
    if not atan2_form:
        os.environ["MM_K2_POW"] = "1"
    try:
        return T.gpu_run(W, H, fr, L, S, mode=mode, batch=batch)
    finally:
        os.environ.pop("MM_K2_POW", None)
        if old is not None:
            os.environ["MM_K2_POW"] = old


@pytest.mark.parametrize("S,L", [(25.0, 5), (10.0, 5), (-25.0, 5), (25.0, 6), (-10.0, 6)])
def test_power_form_matches_atan2_form_and_oracle(S, L):
    W, H = 1100, 48   # N = 2048: the power-form instances
    fr = T.synth(W, H, 5)
    pw = _run(W, H, fr, S, False, L)
    at = _run(W, H, fr, S, True, L)
    ref = T.oracle_run(W, H, fr, L, S)
    assert np.array_equal(pw[0], fr[0])
    for k in range(1, 5):
        T.assert_close_f32(pw[k], ref[k])
        T.assert_close_f32(at[k], ref[k])
        # the two GPU forms agree at least as closely as either with the oracle
        assert np.abs(pw[k] - at[k]).max() <= 1e-4


@pytest.mark.parametrize("S", [7.0, 25.5])
def test_other_scales_keep_the_atan2_form(S):
    """No compiled instance (|S| = 7) or a non-integer S: MM_K2_POW=1 has no effect."""
    W, H = 1100, 48
    fr = T.synth(W, H, 3)
    assert all(np.array_equal(a, b) for a, b in zip(_run(W, H, fr, S, False), _run(W, H, fr, S, True)))


def test_power_form_frame_mode_and_tail():
    """frame-at-a-time (the packed group's one-bin ops every call) and a long
    batch whose last frames run in k_cols_tail: both equal the stream."""
    W, H = 1100, 48
    fr = T.synth(W, H, 30)
    st = _run(W, H, fr, 25.0, False, batch=30)
    fm = _run(W, H, fr, 25.0, False, mode="frame")
    for a, b in zip(st, fm):
        assert np.array_equal(a, b)


def test_power_form_1080p_u8():
    """BASELINE C2 geometry at S = 25 (the bench's phase factor path)."""
    W, H = 1920, 1080
    fr = T.synth(W, H, 3, fmt="u8")
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    got = _run(W, H, fr, 25.0, False)
    for k in range(1, 3):
        T.assert_close_u8(got[k], ref[k])
