"""K3 + K4 fused (k_rows_inv_compose, csrc/mm_kernels.hpp) against the
unfused k_rows_inv + k_compose pair and against the oracle.

The fused kernel walks strips of MM_K34_ROWS output rows (read at mm_create;
0 selects the unfused pair).  Geometries: several strips with a partial last
strip, strips taller than the image, both edge modes (the chroma rows wrap or
clamp at the image edges), RGBA32F and RGBA8, the rows of a 1080p frame.
The same expressions in the same order run in both forms, so they must agree
bitwise; the oracle bars are tests/mmtest.py's.
"""
import os
import numpy as np
import pytest

import mmtest as T

pytestmark = pytest.mark.gpu


class _env:
    """Sets (value str) or removes (None) environment variables for a block."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _run_env(rows, *args, **kw):
    with _env(MM_K34_ROWS=str(rows)):
        return T.gpu_run(*args, **kw)


def _kernels_ran(rows, W, H, n=2, batch=None, oneshot=None):
    """Names of the kernels an n-frame stream launches at this strip size
    (rows None: the library's own choice by batch size; oneshot "0": short
    launches keep the unfused K3 -> K4 pair)."""
    import torch
    import mm355
    with _env(MM_K34_ROWS=None if rows is None else str(rows), MM_K34_ONESHOT=oneshot):
        h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
    if batch:
        h.set_batch(batch)
    fr = torch.zeros((n, H, W, 4), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(fr)
    h.profile_begin()
    h.process_stream(fr, out, n, mm355.RGBA8)
    torch.cuda.synchronize()
    prof = h.profile_end()
    h.close()
    return {k for k, (ms, n, f) in prof.items() if n}


def test_fused_path_is_selected():
    assert "k_rows_inv_compose" in _kernels_ran(64, 200, 120)
    assert "k_rows_inv_compose" not in _kernels_ran(0, 200, 120)
    # W = 64 at N = 64: x0 = 0 leaves no room for the horizontal blur's taps
    assert "k_rows_inv_compose" not in _kernels_ran(64, 64, 48)


def _fused(ran):
    return "k_rows_inv_compose" in ran and "k_rows_inv" not in ran and "k_compose" not in ran


def _unfused(ran):
    return "k_rows_inv_compose" not in ran and "k_rows_inv" in ran and "k_compose" in ran


def test_strip_policy_by_batch():
    """Default policy: the walking strips for many-frame batches; for short
    launches at N <= 1024 the one-shot form k_rows_inv_compose4 when its 4-row
    strips fit one workgroup round (960x540 at batch 1: 135 strips), else the
    unfused pair (always at N = 2048, where the one-shot measured no faster);
    MM_K34_ONESHOT=0 never, 2 always."""
    assert _fused(_kernels_ran(None, 960, 540, n=2, batch=1))
    assert _unfused(_kernels_ran(None, 960, 540, n=2, batch=1, oneshot="0"))
    assert _unfused(_kernels_ran(None, 1920, 1080, n=2, batch=1))
    assert _fused(_kernels_ran(None, 1920, 1080, n=2, batch=1, oneshot="2"))
    assert _unfused(_kernels_ran(None, 1920, 1080, n=2, batch=8))
    assert _fused(_kernels_ran(None, 1920, 1080, n=40, batch=100))


@pytest.mark.parametrize("W,H,edge,fmt,mode", [
    (200, 120, 0, "f32", "frame"), (200, 118, 1, "u8", "frame"), (240, 136, 1, "u8", "stream"),
    (504, 250, 0, "u8", "frame"), (120, 200, 1, "f32", "stream"), (960, 540, 0, "u8", "frame"),
    (1000, 764, 1, "u8", "stream"), (1920, 1080, 0, "u8", "frame")])
def test_oneshot_equals_unfused_bitwise(W, H, edge, fmt, mode):
    """k_rows_inv_compose4 (forced: MM_K34_ONESHOT=2; one-frame calls and
    8-frame batches: every strip of 4 output rows in one workgroup of four FFT
    groups) against the unfused
    K3 -> K4 pair: the same expressions, so bitwise equal.  H = 118 and 250:
    a partial last strip; W = 504 at N = 512: the tightest canvas margin."""
    fr = T.synth(W, H, 4, fmt=fmt)
    with _env(MM_K34_ROWS=None, MM_K34_ONESHOT="2"):
        a = T.gpu_run(W, H, fr, 5, 25.0, edge, mode=mode)
    b = _run_env(0, W, H, fr, 5, 25.0, edge, mode=mode)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_oneshot_standard_mode_and_oracle():
    W, H = 200, 120
    fr = T.synth(W, H, 4)
    std = {"apply": True}
    with _env(MM_K34_ROWS=None, MM_K34_ONESHOT="2"):
        a = T.gpu_run(W, H, fr, 5, 25.0, 0, mode="frame", standard=std)
        got = T.gpu_run(W, H, fr, 5, 25.0, 1, mode="frame")
    b = _run_env(0, W, H, fr, 5, 25.0, 0, mode="frame", standard=std)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    ref = T.oracle_run(W, H, fr, 5, 25.0, 1)
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r)


@pytest.mark.parametrize("W,H,rows,edge,fmt", [
    (200, 120, 64, 0, "f32"), (200, 120, 8, 1, "f32"), (200, 118, 4, 0, "u8"),
    (240, 136, 12, 1, "u8"), (120, 200, 32, 0, "f32"), (504, 250, 16, 1, "u8"),
    (2100, 300, 128, 0, "u8"), (2100, 300, 256, 1, "f32")])
def test_fused_equals_unfused_bitwise(W, H, rows, edge, fmt):
    fr = T.synth(W, H, 5, fmt=fmt)
    a = _run_env(rows, W, H, fr, 5, 25.0, edge, mode="stream")
    b = _run_env(0, W, H, fr, 5, 25.0, edge, mode="stream")
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("W,H,rows,edge", [(200, 120, 16, 0), (240, 136, 64, 1)])
def test_fused_vs_oracle(W, H, rows, edge):
    fr = T.synth(W, H, 4)
    ref = T.oracle_run(W, H, fr, 5, 25.0, edge)
    got = _run_env(rows, W, H, fr, 5, 25.0, edge)
    assert np.array_equal(got[0], fr[0])
    for g, r in zip(got[1:], ref[1:]):
        T.assert_close_f32(g, r)


def test_fused_equals_unfused_1080p_u8():
    W, H = 1920, 1080
    fr = T.synth(W, H, 3, fmt="u8")
    a = _run_env(64, W, H, fr, 5, 25.0, 0, mode="stream")
    b = _run_env(0, W, H, fr, 5, 25.0, 0, mode="stream")
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_fused_standard_mode():
    W, H = 200, 120
    fr = T.synth(W, H, 4)
    std = {"apply": True}
    a = _run_env(16, W, H, fr, 5, 25.0, 0, mode="stream", standard=std)
    b = _run_env(0, W, H, fr, 5, 25.0, 0, mode="stream", standard=std)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.slow
def test_fused_equals_unfused_2160p_u8():
    """N = 4096: two 512-thread groups per workgroup (1,024 threads) and 73.7 KB
    of dynamic LDS (hipFuncSetAttribute at mm_create)."""
    W, H = 3840, 2160
    fr = T.synth(W, H, 3, fmt="u8")
    b = _run_env(0, W, H, fr, 6, 25.0, 0, mode="stream")
    for rows in (64, 128):   # 128: the N = 4096 default strip (MM_K34_ROWS_4K)
        a = _run_env(rows, W, H, fr, 6, 25.0, 0, mode="stream")
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
