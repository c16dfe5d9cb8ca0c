"""Independent float64 numpy restatement of the reference pyramid-mode frame
operator — TEST INFRASTRUCTURE.  Used only to cross-check the literal fp32 C
oracle (oracle/mm_ref.c).

It deliberately uses a different formulation from the C oracle:
  * np.fft.fft2/ifft2 + fftshift instead of the literal radix-2 passes of
    FFT.compute:213-276 (SURVEY.md §8 a8 states the equivalence);
  * vectorised bilinear sampling, float64 throughout;
  * the per-level loop of ProcessPyramidPhaseDifference
    (PyramidPhaseDifference.compute:58-101) evaluated on whole arrays.
Semantics (REPEAT/CLAMP wrap, quad coverage, window, blur) follow the same
engine decisions as the oracle.
"""
import numpy as np

PI = np.float64(np.float32(3.14159265359))  # the shaders' PI, as a float literal


def next_pow2(v):
    n = 1
    while n < v:
        n <<= 1
    return n


def _wrap(i, n, edge):
    return np.clip(i, 0, n - 1) if edge == 1 else np.mod(i, n)


def _bilinear(tex, u, v, edge):
    """tex [h, w, c]; u [..] v [..] normalised coords -> [.., c]"""
    h, w = tex.shape[:2]
    tx = u * w - 0.5
    ty = v * h - 0.5
    x0 = np.floor(tx)
    y0 = np.floor(ty)
    fx = (tx - x0)[..., None]
    fy = (ty - y0)[..., None]
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    xa, xb = _wrap(x0, w, edge), _wrap(x0 + 1, w, edge)
    ya, yb = _wrap(y0, h, edge), _wrap(y0 + 1, h, edge)
    a = (1 - fx) * tex[ya, xa] + fx * tex[ya, xb]
    b = (1 - fx) * tex[yb, xa] + fx * tex[yb, xb]
    return (1 - fy) * a + fy * b


M_RGB2YIQ = np.array([[0.299, 0.587, 0.114],
                      [0.596, -0.274, -0.322],
                      [0.211, -0.523, 0.312]], dtype=np.float64)
M_YIQ2RGB = np.array([[1.0, 0.956, 0.621],
                      [1.0, -0.272, -0.647],
                      [1.0, -1.106, 1.703]], dtype=np.float64)


def pad_window(frame, N, edge):
    """RGB->YIQ stretch blit + PadTexture quad + Hann window -> [N, N, 3] YIQ."""
    H, W = frame.shape[:2]
    c = (np.arange(N) + 0.5) / N
    U, V = np.meshgrid(c, c)
    yiq_full = _bilinear(frame[..., :3].astype(np.float64), U, V, edge) @ M_RGB2YIQ.T
    X = np.arange(N)
    nx = 2 * X + 1 - (N - W)
    ny = 2 * X + 1 - (N - H)
    cov_x = (nx >= 0) & (nx < 2 * W)
    cov_y = (ny >= 0) & (ny < 2 * H)
    u = nx / (2.0 * W)
    v = ny / (2.0 * H)
    UU, VV = np.meshgrid(u, v)
    padded = _bilinear(yiq_full, UU, VV, edge)
    padded *= (cov_y[:, None] & cov_x[None, :])[..., None]
    h = 0.5 * (1 - np.cos(2 * PI * c))
    return padded * (h[:, None] * h[None, :])[..., None]


def smoothstep(x):
    t = np.clip(x, 0.0, 1.0)
    return t * t * (3 - 2 * t)


def masks(N, L, minf, maxf):
    f1 = np.arange(N) / N - 0.5
    FX, FY = np.meshgrid(f1, f1)
    fr = np.sqrt(FX * FX + FY * FY)
    out = []
    for i in range(L):
        m = np.zeros_like(fr)
        if i == 0:
            band = fr > maxf * 0.8
            m[band] = smoothstep((fr[band] - maxf * 0.8) / (maxf * 0.2))
            m[fr > maxf] = 1.0
        elif i == L - 1:
            band = fr < minf * 1.2
            m[band] = 1.0 - smoothstep((fr[band] - minf) / (minf * 0.2))
            m[fr < minf] = 1.0
        else:
            with np.errstate(invalid="ignore", divide="ignore"):
                ratio = np.float64(i - 1) / np.float64(L - 3) if L != 3 else np.nan
            c = minf * (maxf / minf) ** (1.0 - ratio)
            lo, hi = c - 0.5 * c, c + 0.5 * c
            if np.isfinite(c):
                band = (fr >= lo) & (fr <= hi)
                nrm = (fr[band] - lo) / (hi - lo)
                m[band] = 0.5 * (1 + np.cos(2 * PI * (nrm - 0.5)))
        out.append(m)
    return out


def wrap_phase(p):
    p = np.where(p > PI, p - 2 * PI, p)
    return np.where(p < -PI, p + 2 * PI, p)


def blur(img, edge):
    N = img.shape[0]
    taps = [(0.0, 0.2270270270), (1.3846153846, 0.3162162162), (-1.3846153846, 0.3162162162),
            (3.2307692308, 0.0702702703), (-3.2307692308, 0.0702702703)]

    def one(im, axis):
        out = np.zeros_like(im)
        base = np.arange(N, dtype=np.float64)
        for off, w in taps:
            t = base + 0.5 * off
            i0 = np.floor(t)
            f = t - i0
            i0 = i0.astype(np.int64)
            a, b = _wrap(i0, N, edge), _wrap(i0 + 1, N, edge)
            if axis == 1:
                out += w * ((1 - f)[None, :] * im[:, a] + f[None, :] * im[:, b])
            else:
                out += w * ((1 - f)[:, None] * im[a, :] + f[:, None] * im[b, :])
        return out

    return one(one(img, 1), 0)


def bandpass_weights(N, apply=True, low=0.05, high=0.4, steep=3.0, sens=1.5, edge=0.8):
    """calculate_spatial_frequency + calculate_bandpass_weight
    (PhaseDifferenceComputeShader.compute:74-122), float64."""
    f1 = np.arange(N) / N - 0.5
    FX, FY = np.meshgrid(f1, f1)
    sf = np.minimum(np.sqrt(FX * FX + FY * FY) / np.float64(np.float32(0.707)), 1.0)
    if not apply:
        return np.ones_like(sf)
    w = np.ones_like(sf)
    lo = sf < low
    w[lo] *= (sf[lo] / max(low, 0.001)) ** steep
    hi = sf > high
    w[hi] *= ((1.0 - sf[hi]) / max(1.0 - high, 0.001)) ** steep
    w *= sens
    mid = (sf > low) & (sf < high)
    w[mid] *= 1.0 + edge * np.sin(PI * (sf[mid] - low) / (high - low))
    return np.maximum(w, 0.0)


def process_frame(cur, prev, L, minf, maxf, S, tau=0.01, edge=0, dbg=None, standard=None):
    """One non-first OnRenderImage call on float RGBA frames [H, W, 4].
    standard: None (pyramid mode) or dict of bandpass_weights() arguments
    (ProcessFrameWithStandardMagnification, .cs:208-232)."""
    H, W = cur.shape[:2]
    N = next_pow2(max(W, H))
    pc = pad_window(cur, N, edge)
    pp = pad_window(prev, N, edge)
    Fc = np.fft.fftshift(np.fft.fft2(pc[..., 0]))
    Fp = np.fft.fftshift(np.fft.fft2(pp[..., 0]))
    acc = np.zeros_like(Fc)
    if standard is not None:
        gate = (np.abs(Fc) < tau) | (np.abs(Fp) < tau)
        d = wrap_phase(np.angle(Fp) - np.angle(Fc))
        w = bandpass_weights(N, **standard)
        acc = np.where(gate, Fc, Fc * np.exp(1j * S * w * d))
    for i, m in enumerate(masks(N, L, minf, maxf) if standard is None else []):
        c = Fc * m
        p = Fp * m
        if i == 0 or i == L - 1:
            acc += c
            continue
        gate = (np.abs(c) < tau) | (np.abs(p) < tau)
        d = wrap_phase(np.angle(p) - np.angle(c))
        acc += np.where(gate, c, c * np.exp(1j * S * d))
    # PerformIFFT: the centre flip of FFT.compute:175-189 cancels under |.|
    ymag = np.abs(np.fft.ifft2(np.fft.ifftshift(acc)))
    yb = blur(ymag, edge)
    yiq = np.stack([yb, pc[..., 1], pc[..., 2]], axis=-1)
    rgb = np.clip(yiq @ M_YIQ2RGB.T, 0.0, 1.0)
    # crop (integer or half-integer offsets): bilinear at texel x0+i
    tx = ((N - W) + 2 * np.arange(W)) / 2.0
    ty = ((N - H) + 2 * np.arange(H)) / 2.0
    out = np.ones((H, W, 4))
    TX, TY = np.meshgrid((tx + 0.5) / N, (ty + 0.5) / N)
    out[..., :3] = _bilinear(rgb, TX, TY, edge)
    if dbg is not None:
        dbg.update(y_cur=pc[..., 0], F_cur=Fc, F_prev=Fp, A=acc, y_mag=ymag, y_blur=yb)
    return out


def debug_buffer1(y):
    """complexBuffer1 after PerformFFT, formulated independently of the radix-2
    ping-pong: centred rows transformed along x, then the N/2-point column DFTs
    of the even rows (rows [0, N/2)) and of the odd rows (rows [N/2, N)) -- the
    state one radix-2 DIT stage before the full column transform."""
    N = y.shape[0]
    sgn = np.where((np.add.outer(np.arange(N), np.arange(N)) & 1) == 1, -1.0, 1.0)
    r = np.fft.fft(y * sgn, axis=1)
    return np.vstack([np.fft.fft(r[0::2], axis=0), np.fft.fft(r[1::2], axis=0)])


def debug_view(frame, N, edge, show_mag, show_phase):
    """ProcessDebugView (.cs:234-257) in float64: RFloat view textures sampled
    as (v, 0, 0, 1); crop for one view, bilinear split screen for both."""
    H, W = frame.shape[:2]
    y = pad_window(frame, N, edge)[..., 0]
    b = debug_buffer1(y)
    mag = np.log10(np.abs(b) * 10.0 + 1.0) / 4.0
    pha = np.abs(np.angle(b)) / 1.57079632679
    out = np.zeros((H, W, 4))
    out[..., 3] = 1.0
    if show_mag and show_phase:
        X = np.arange(W)
        right = 2 * X + 1 >= W
        u = (2 * X + 1 - np.where(right, W, 0)) / W
        v = (2 * np.arange(H) + 1) / (2.0 * H)
        UU, VV = np.meshgrid(u, v)
        lm = _bilinear(mag[..., None], UU, VV, edge)[..., 0]
        lp = _bilinear(pha[..., None], UU, VV, edge)[..., 0]
        out[..., 0] = np.where(right[None, :], lp, lm)
    else:
        x0, y0 = (N - W) // 2, (N - H) // 2
        out[..., 0] = (mag if show_mag else pha)[y0:y0 + H, x0:x0 + W]
    return out
