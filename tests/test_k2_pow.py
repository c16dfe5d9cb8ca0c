"""K2's power form of the phase factor (MM_K2_PYR_POW, integer phase scale;
opt-in with MM_K2_POW=1: same-call it measured 4 % slower than the atan2 form,
profiles/r03_ab3.txt):
e^{i S wrap(arg p - arg c)} = z^S with z = p conj(c) / |p||c|
(PyramidPhaseDifference.compute:47-54, 92-98: for integer S the wrap's
multiple of 2 pi drops out).  Against the atan2 + sin/cos form of the same
kernel (the default) and against the oracle's literal atan2f path, over
exponents with every bit pattern the square-and-multiply loop takes: 0, 1,
powers of two, odd/even, negative."""
import os

import numpy as np
import pytest

import mmtest as T

pytestmark = pytest.mark.gpu


def _run(W, H, fr, S, nopow, mode="stream"):
    """nopow: the default atan2 form; else MM_K2_POW=1 (read at mm_create)."""
    old = os.environ.pop("MM_K2_POW", None)
    if not nopow:
        os.environ["MM_K2_POW"] = "1"
    try:
        return T.gpu_run(W, H, fr, 5, S, mode=mode, batch=3)
    finally:
        os.environ.pop("MM_K2_POW", None)
        if old is not None:
            os.environ["MM_K2_POW"] = old


@pytest.mark.parametrize("S", [25.0, 10.0, 0.0, 1.0, 2.0, 16.0, 7.0, -3.0, 64.0, 100.0])
def test_power_form_matches_atan2_form_and_oracle(S):
    W, H = 200, 120
    fr = T.synth(W, H, 5)
    pw = _run(W, H, fr, S, False)
    at = _run(W, H, fr, S, True)
    ref = T.oracle_run(W, H, fr, 5, S)
    assert np.array_equal(pw[0], fr[0])
    for k in range(1, 5):
        T.assert_close_f32(pw[k], ref[k])
        T.assert_close_f32(at[k], ref[k])
        # the two GPU forms agree at least as closely as either with the oracle
        assert np.abs(pw[k] - at[k]).max() <= 1e-4


def test_power_form_1080p_u8():
    """BASELINE C2 geometry at S = 25 (the bench's phase factor path)."""
    W, H = 1920, 1080
    fr = T.synth(W, H, 3, fmt="u8")
    ref = T.oracle_run(W, H, fr, 5, 25.0)
    got = _run(W, H, fr, 25.0, False)
    for k in range(1, 3):
        T.assert_close_u8(got[k], ref[k])
