"""Shared helpers for the GPU parity tests (HIP path through the C-ABI)."""
import numpy as np

import oracle_py as O

# Tolerances, RGB in [0, 1]:
TOL_MAX = 1e-4      # max-abs, fp32 HIP vs fp32 oracle, integer phase scale
TOL_RMSE = 1e-5     # RMSE
TOL_P999 = 1e-4     # 99.9th percentile, non-integer phase scale (wrap ties at |d|~pi)
U8_FRAC = 1e-3      # RGBA8: exact except +-1 LSB on <= 0.1% of values


def synth(W, H, n, t0=0, gray=False, seed=0x5EED0000, fmt="f32"):
    fr = [O.synth_frame(W, H, t0 + t, seed=seed, gray=gray) for t in range(n)]
    if fmt == "u8":
        return fr
    return [f.astype(np.float32) / np.float32(255.0) for f in fr]


# standard-mode settings in oracle terms -> mm_params fields
def _std_fields(std):
    return dict(apply_bandpass_filter=std.get("apply", True),
                low_frequency_cutoff=std.get("low", 0.05),
                high_frequency_cutoff=std.get("high", 0.4),
                filter_steepness=std.get("steep", 3.0),
                motion_sensitivity=std.get("sens", 1.5),
                enhance_edges=True, edge_enhancement=std.get("edge", 0.8))


def oracle_run(W, H, frames, levels=5, S=10.0, edge=0, minf=0.05, maxf=0.45, apply=True,
               standard=None, debug=None):
    o = O.Oracle(W, H, levels=levels, min_freq=minf, max_freq=maxf, phase_scale=S,
                 edge_mode=edge)
    o.set_apply(apply)
    if standard is not None:
        o.set_standard(True, **standard)
    if debug is not None:
        o.set_debug(*debug)
    return [o.process(f) for f in frames]


def gpu_run(W, H, frames, levels=5, S=10.0, edge=0, minf=0.05, maxf=0.45, mode="frame",
            apply=True, standard=None, debug=None, batch=8, fmt=None, extra=None):
    """batch: mm_set_batch frames per internal batch (8: multi-frame streams
    cross batch boundaries, where K2's state is stored and reloaded).
    fmt: the frame format (default from the dtype: uint8 RGBA8, float16
    RGBA16F, float32 RGBA32F; RGBA8_SRGB must be named).  extra: more
    mm_params fields."""
    import torch
    import mm355
    extra = dict(extra or {})
    if standard is not None:
        extra.update(mode=mm355.MODE_STANDARD, **_std_fields(standard))
    if debug is not None:
        extra.update(show_magnitude=debug[0], show_phase=debug[1])
    p = mm355.Params.make(levels=levels, min_freq=minf, max_freq=maxf, phase_scale=S,
                          edge_mode=edge, apply_magnification=apply, **extra)
    h = mm355.Handle(W, H, p)
    h.set_batch(batch)
    if fmt is None:
        fmt = {np.dtype(np.uint8): mm355.RGBA8, np.dtype(np.float16): mm355.RGBA16F}.get(
            frames[0].dtype, mm355.RGBA32F)
    dev_in = torch.from_numpy(np.stack(frames)).cuda()
    dev_out = torch.empty_like(dev_in)
    if mode == "frame":
        for k in range(len(frames)):
            h.process(dev_in[k], dev_out[k], fmt)
    elif mode == "stream":
        h.process_stream(dev_in, dev_out, len(frames), fmt)
    elif mode == "host":
        outs = []
        for f in frames:
            o = np.empty_like(f)
            h.process(f, o, fmt, on_device=False)
            outs.append(o)
        h.close()
        return outs
    torch.cuda.synchronize()
    res = dev_out.cpu().numpy()
    h.close()
    return list(res)


def err_stats(a, b):
    e = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return e.max(), float(np.sqrt((e ** 2).mean())), float(np.quantile(e, 0.999))


def assert_close_f32(gpu, ref, integer_scale=True):
    mx, rmse, p999 = err_stats(gpu, ref)
    if integer_scale:
        assert mx <= TOL_MAX and rmse <= TOL_RMSE, (mx, rmse, p999)
    else:
        assert p999 <= TOL_P999 and rmse <= TOL_RMSE * 10, (mx, rmse, p999)


def assert_close_u8(gpu, ref):
    d = np.abs(gpu.astype(np.int32) - ref.astype(np.int32))
    assert d.max() <= 1, d.max()
    assert (d > 0).mean() <= U8_FRAC, (d > 0).mean()


def state_rows(st, N, H):
    """The pyramid/standard state (mm_get_state / mm_compute_state, ABI 8):
    G_{t-1}[f][r], complex fp32, f = 0..N/2, r = 0..H-1 (rows rounded up to
    even in the buffer) -> complex128 [N/2+1][H]."""
    Hg = H + (H & 1)
    a = st.view(np.float32) if isinstance(st, np.ndarray) else st.view(dtype=__import__("torch").float32).cpu().numpy()
    a = a.reshape(N // 2 + 1, Hg, 2).astype(np.float64)
    return (a[..., 0] + 1j * a[..., 1])[:, :H]


def spectrum_from_state(G, N, H):
    """2D half spectrum [fx = 0..N/2][fy = 0..N) (unshifted) of the canvas the
    state's rows sit in (image rows at y0 = (N - H) // 2, zero elsewhere)."""
    y0 = (N - H) // 2
    col = np.zeros((G.shape[0], N), np.complex128)
    col[:, y0:y0 + H] = G
    return np.fft.fft(col, axis=1)


def centered_to_half(Fc, N):
    """Oracle's fftshift-ed 2D spectrum Fc[y][x] -> [fx = 0..N/2][fy = 0..N)."""
    fx = np.arange(N // 2 + 1)
    fy = np.arange(N)
    return Fc[((fy + N // 2) % N)[None, :], ((fx + N // 2) % N)[:, None]]
