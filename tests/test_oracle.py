"""Known-answer tests of the CPU oracle (SURVEY.md §4 test pyramid, level 1).

The reference ships no tests or fixtures, so the oracle is pinned
by analytic identities plus an independent float64 restatement (np_twin).
"""
import numpy as np
import pytest

import np_twin
import oracle_py as O


def test_fft_impulse_constant_tone():
    n = 64
    y = np.zeros((n, n), np.float32)
    y[0, 0] = 1.0
    F = O.fft_centered(y)              # centred: every bin = +-1 (CenterComplex sign)
    assert np.allclose(np.abs(F), 1.0, atol=1e-6)
    y = np.ones((n, n), np.float32)
    F = O.fft_centered(y)              # DC lands at (N/2, N/2)
    assert abs(F[n // 2, n // 2] - n * n) < 1e-3
    F[n // 2, n // 2] = 0
    assert np.abs(F).max() < 1e-3
    xs = np.arange(n)
    y = np.cos(2 * np.pi * 5 * xs / n)[None, :].repeat(n, 0).astype(np.float32)
    F = np.abs(O.fft_centered(y))
    peaks = sorted(zip(*np.where(F > n * n / 4)))
    assert peaks == [(n // 2, n // 2 - 5), (n // 2, n // 2 + 5)]


def test_fft_matches_numpy():
    rng = np.random.default_rng(1)
    y = rng.random((128, 128)).astype(np.float32)
    F = O.fft_centered(y)
    ref = np.fft.fftshift(np.fft.fft2(y.astype(np.float64)))
    assert np.abs(F - ref).max() / np.abs(ref).max() < 1e-6


def test_ifft_mag_roundtrip():
    rng = np.random.default_rng(2)
    y = rng.random((64, 64)).astype(np.float32)
    back = O.ifft_mag(O.fft_centered(y))
    assert np.abs(back - y).max() < 1e-5


@pytest.mark.parametrize("L", [3, 4, 5, 6])
def test_masks_at_radii(L):
    n = 256
    m = [O.mask(n, L, i, 0.05, 0.45) for i in range(L)]
    tw = np_twin.masks(n, L, 0.05, 0.45)
    for a, b in zip(m, tw):
        assert np.abs(a - b).max() < 1e-5
    c = n // 2
    assert m[L - 1][c, c] == 1.0                     # DC: low-pass only
    assert m[0][0, 0] == 1.0                         # corner radius 0.707 > maxF
    if L == 3:                                       # (i-1)/(L-3) = 0/0 -> NaN band
        assert not m[1].any()
    if L == 5:                                       # band centres 0.45/0.15/0.05
        assert m[2][c, c + int(0.15 * n)] > 0.99
        assert abs(sum(mm.mean() for mm in m) - 1.096) < 0.01   # mean sum 1.096


def test_normalize_phase_wrap():
    pi = np.float32(3.14159265359)
    assert O.normalize_phase(0.5) == np.float32(0.5)
    assert abs(O.normalize_phase(float(pi) + 0.5) - (0.5 - pi)) < 1e-6
    assert abs(O.normalize_phase(-float(pi) - 0.5) - (pi - 0.5)) < 1e-6
    assert O.normalize_phase(float(pi)) == pi        # while (p > PI): PI itself stays


def test_yiq_gray_and_inverse():
    yiq = O.rgb_to_yiq(np.array([0.5, 0.5, 0.5]))
    assert abs(yiq[0] - 0.5) < 1e-6 and abs(yiq[1]) < 1e-6 and abs(yiq[2]) < 1e-6
    rgb = np.array([0.2, 0.6, 0.3], np.float32)
    assert np.abs(O.yiq_to_rgb(O.rgb_to_yiq(rgb)) - rgb).max() < 2e-3  # NTSC matrices, 3 digits
    assert np.all(O.yiq_to_rgb(np.array([2.0, 0, 0])) == 1.0)         # saturate


def test_blur_taps():
    n = 64
    img = np.zeros((n, n), np.float32)
    img[32, 32] = 1.0
    b = O.blur(img)
    row = b[32, 30:35] / b[32, 30:35].sum()
    exp = np.array([0.0432432, 0.2459459, 0.4216216, 0.2459459, 0.0432432])
    assert np.abs(row - exp).max() < 1e-5
    assert abs(b.sum() - 1.0) < 1e-5
    e = np.zeros((n, n), np.float32)
    e[0, 0] = 1.0
    assert O.blur(e, O.EDGE_REPEAT)[n - 1, n - 1] > 0      # repeat wraps around
    assert O.blur(e, O.EDGE_CLAMP)[n - 1, n - 1] == 0


def test_pad_offsets_1080p():
    o = O.Oracle(1920, 1080)
    assert o.N == 2048
    f = O.synth_frame(1920, 1080, 0)[..., :].astype(np.float32) / 255
    canvas = np.zeros((2048, 2048, 4), np.float32)
    O.lib().mm_ref_pad_window(o.h, O._fp(np.ascontiguousarray(f)), O._fp(canvas))
    nz = np.where(np.abs(canvas[..., 0]).sum(1) > 0)[0]
    assert nz[0] == 484 and nz[-1] == 484 + 1079
    nzc = np.where(np.abs(canvas[..., 0]).sum(0) > 0)[0]
    assert nzc[0] == 64 and nzc[-1] == 64 + 1919


def test_first_frame_passthrough_bitwise():
    o = O.Oracle(64, 48, phase_scale=25)
    f = O.synth_frame(64, 48, 0)
    assert np.array_equal(o.process(f), f)
    ff = (f.astype(np.float32) / 255)
    o.reset()
    assert np.array_equal(o.process(ff), ff)
    out = o.process(O.synth_frame(64, 48, 1))
    assert np.all(out[..., 3] == 255)                # combine alpha = 1


def test_L3_no_magnification():
    """L=3: the middle mask is all zero (NaN ratio), so phase_scale and the
    previous frame have no effect."""
    W = H = 64
    f0 = O.synth_frame(W, H, 0, gray=True).astype(np.float32) / 255
    f1 = O.synth_frame(W, H, 5, gray=True).astype(np.float32) / 255
    outs = []
    for S, prev in ((10.0, f0), (25.0, f0), (10.0, f1)):
        o = O.Oracle(W, H, levels=3, phase_scale=S)
        o.process(prev)
        outs.append(o.process(f1))
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    assert np.abs(outs[0][..., 0] - outs[0][..., 1]).max() < 1e-6  # gray -> R=G=B (fp32 I,Q ~ 0)


def test_static_scene_scale_invariant():
    """prev == cur => delta = 0 everywhere => output independent of phase_scale."""
    f = O.synth_frame(64, 48, 3).astype(np.float32) / 255
    res = []
    for S in (1.0, 25.0):
        o = O.Oracle(64, 48, phase_scale=S)
        o.process(f)
        res.append(o.process(f))
    assert np.abs(res[0] - res[1]).max() < 1e-6


def test_apply_off_and_state_roundtrip():
    W, H = 64, 48
    frames = [O.synth_frame(W, H, t).astype(np.float32) / 255 for t in range(4)]
    a = O.Oracle(W, H, phase_scale=10)
    outs = [a.process(f) for f in frames]
    b = O.Oracle(W, H, phase_scale=10)
    b.process(frames[0])
    b.process(frames[1])
    st = b.get_state()
    c = O.Oracle(W, H, phase_scale=10)
    c.set_state(st)
    assert np.array_equal(c.process(frames[2]), outs[2])
    d = O.Oracle(W, H)
    d.set_apply(False)
    d.process(frames[0])
    assert np.array_equal(d.process(frames[1]), frames[1])


@pytest.mark.parametrize("W,H,L,S,gray,edge", [
    (64, 48, 5, 10.0, False, 0), (64, 48, 4, 25.0, False, 0), (64, 48, 6, 9.7, False, 1),
    (256, 256, 3, 10.0, True, 0), (200, 120, 5, 25.0, False, 0), (96, 96, 5, 25.0, False, 1)])
def test_oracle_vs_float64_twin(W, H, L, S, gray, edge):
    o = O.Oracle(W, H, levels=L, phase_scale=S, edge_mode=edge)
    f0 = O.synth_frame(W, H, 0, gray=gray).astype(np.float32) / 255
    f1 = O.synth_frame(W, H, 3, gray=gray).astype(np.float32) / 255
    o.process(f0)
    a1 = o.process(f1)
    b1 = np_twin.process_frame(f1.astype(np.float64), f0.astype(np.float64), L, 0.05, 0.45, S,
                               edge=edge)
    e = np.abs(a1 - b1)
    assert e.max() < 5e-6 and np.sqrt((e ** 2).mean()) < 1e-6


# ---- standard (non-pyramid) mode, f1: PhaseDifferenceComputeShader.compute ----

def test_bandpass_weights_known_values():
    w = O.bandpass_weights(128)                      # defaults .cs:35-43
    assert w[64, 64] == 0.0                          # DC: pow(0, steepness) = 0
    assert abs(w.max() - 1.5 * 1.8) < 1e-3           # sens * (1 + edge) at the band centre
    assert np.abs(w - np_twin.bandpass_weights(128)).max() < 1e-5
    assert np.all(O.bandpass_weights(64, apply=False) == 1.0)


@pytest.mark.parametrize("W,H,S,std", [
    (64, 48, 10.0, {}), (200, 120, 25.0, dict(steep=2.0, high=0.3)),
    (96, 96, 9.7, dict(apply=False)), (64, 48, 25.0, dict(edge=0.0, sens=1.0))])
def test_standard_mode_vs_float64_twin(W, H, S, std):
    o = O.Oracle(W, H, phase_scale=S)
    o.set_standard(True, **std)
    f0 = O.synth_frame(W, H, 0).astype(np.float32) / 255
    f1 = O.synth_frame(W, H, 3).astype(np.float32) / 255
    o.process(f0)
    a = o.process(f1)
    b = np_twin.process_frame(f1.astype(np.float64), f0.astype(np.float64), 5, 0.05, 0.45, S,
                              standard=std)
    e = np.abs(a - b)
    assert e.max() < 5e-6 and np.sqrt((e ** 2).mean()) < 1e-6


def test_standard_mode_static_scene_is_identity_spectrum():
    """prev == cur: delta = 0, so A = F and the output is the unmagnified
    reconstruction -- independent of phase scale and band-pass settings."""
    f = O.synth_frame(64, 48, 2).astype(np.float32) / 255
    outs = []
    for S, std in ((1.0, {}), (25.0, dict(steep=1.0, sens=3.0))):
        o = O.Oracle(64, 48, phase_scale=S)
        o.set_standard(True, **std)
        o.process(f)
        outs.append(o.process(f))
    assert np.abs(outs[0] - outs[1]).max() < 1e-6


# ---- f3 debug views (ProcessDebugView, .cs:234-257) -------------------------

def test_fft_buffer1_is_penultimate_column_stage():
    """complexBuffer1 after the radix-2 ping-pong = even/odd-row N/2-point column
    DFTs of the fully row-transformed, centred image (twin, np.fft)."""
    for n in (16, 32, 256):
        y = np.random.default_rng(n).standard_normal((n, n)).astype(np.float32)
        b = O.fft_buffer1(y)
        t = np_twin.debug_buffer1(y.astype(np.float64))
        assert np.abs(b - t).max() / np.abs(t).max() < 2e-6
        # and it is NOT the finished spectrum
        assert np.abs(b - O.fft_centered(y)).max() > 1e-2 * np.abs(t).max()


@pytest.mark.parametrize("mag,pha", [(True, False), (False, True), (True, True)])
def test_debug_view_matches_twin(mag, pha):
    W, H = 64, 48
    f0, f1 = (O.synth_frame(W, H, t).astype(np.float32) / np.float32(255) for t in (0, 1))
    o = O.Oracle(W, H, levels=5, phase_scale=10.0)
    o.set_debug(mag, pha)
    assert np.array_equal(o.process(f0), f0)          # first frame still passes through
    out = o.process(f1)
    ref = np_twin.debug_view(f1.astype(np.float64), o.N, 0, mag, pha)
    assert np.array_equal(out[..., 1:3], np.zeros_like(out[..., 1:3]))
    assert np.all(out[..., 3] == 1.0)
    err = np.abs(out[..., 0] - ref[..., 0])
    if mag and not pha:
        assert err.max() < 1e-5
    else:   # |arg z| is ill-conditioned where |z| ~ 0: judge by percentiles
        assert np.quantile(err, 0.999) < 1e-4 and np.median(err) < 1e-6
    o.close()


def test_debug_view_state_follows_input():
    """While a debug view is on, previousSourceTexture still follows the input
    (.cs:122): switching it off magnifies against the last debug-view frame."""
    W, H = 64, 48
    fr = [O.synth_frame(W, H, t).astype(np.float32) / np.float32(255) for t in range(3)]
    a = O.Oracle(W, H, levels=5, phase_scale=10.0)
    b = O.Oracle(W, H, levels=5, phase_scale=10.0)
    a.process(fr[0])
    a.set_debug(True, False)
    a.process(fr[1])
    a.set_debug(False, False)
    b.process(fr[1])
    assert np.array_equal(a.process(fr[2]), b.process(fr[2]))
    a.close()
    b.close()
