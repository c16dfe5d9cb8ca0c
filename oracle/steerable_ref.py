"""MM_MODE_STEERABLE — specification and CPU oracle of this repository's
orientation + temporal-IIR extension.  TEST
INFRASTRUCTURE: only tests/ import it, as the checker.

PARITY UNPINNED BY THE REFERENCE.  The shipping reference has no orientations
and no IIR: its only precedent, the deleted SteerablePyramid.compute (kept in
Library/Artifacts/f5/f51395e5...), was never driven by any C# code and applies
frequency-domain masks to spatial pixels.  This file is therefore the spec the
HIP path is tested against; it reuses the reference's stages everywhere else.

Per non-first frame (float64, centred spectra as in tests/np_twin.py):
  y  = windowed, padded luma (pad_window: .cs:147-153)
  F  = fftshift(fft2(y))
  residual  r = ifft2(F (m_0 + m_{L-1}))           levels 0, L-1 always pass
  subbands  s_{i,o} = ifft2(F m_i a_o)              middle levels i, o < O/2
      m_i: GeneratePyramidFilters (PyramidOperations.compute:25-87)
      a_o = c_o / sum_k c_k,  c_k = max(0, cos(theta - 2 pi k / O))^4 over
            O orientations (the deleted shader's cos^4 lobes, normalised to a
            partition of unity); a_o = 1/O at DC and on the Nyquist row/column
            (no orientation there), so a_o(-f) = a_{o+O/2}(f) on every bin.
  temporal filter on the local phase phi = arg s (state per coefficient):
      DIFF (reference rule per coefficient): P = wrap(phi_prev - phi)
           (PyramidPhaseDifference.compute:88-98: prev - cur)
      IIR  (band-pass of the unwrapped phase Phi, d = wrap(phi - phi_prev)):
           u_h <- (1 - r_h)(u_h + d),  u_l <- (1 - r_l)(u_l + d),
           P = u_l - u_h  (= L_h - L_l for L <- L + r (Phi - L), kept as the
           bounded deviations u = Phi - L)
  gate:     |s| < tau  ->  s' = s  (state still updated)
  else      s' = s exp(i S P)
  y' = r + sum_{i,o<O/2} 2 Re(s'_{i,o})   (o + O/2 is the conjugate of o)
  then the reference's |.| (ConvertComplexMagToTex), blur, YIQ recombine,
  YIQ->RGB, crop (np_twin).  First frame: passthrough; state <- frame 0.
At S = 0 the output equals the reference pipeline at S = 0 exactly (identity
sum_o a_o = 1), which pins the whole chain to the reference's stages.
"""
import os
import sys

import numpy as np
from scipy import fft as sfft

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests"))
import np_twin as T  # noqa: E402

FILTER_DIFF = 0
FILTER_IIR = 1
# threads of the float64 FFTs (scipy.fft workers); the 2160p case sets 16
WORKERS = 1


def angular_masks(N, O):
    """a_o on the centred N x N grid for all O orientations: [O, N, N]."""
    assert O >= 2 and O % 2 == 0
    f1 = np.arange(N) / N - 0.5
    FX, FY = np.meshgrid(f1, f1)
    r = np.hypot(FX, FY)
    with np.errstate(invalid="ignore", divide="ignore"):
        cx, sy = FX / r, FY / r
    c = np.stack([np.maximum(0.0, cx * np.cos(2 * np.pi * k / O) + sy * np.sin(2 * np.pi * k / O))
                  for k in range(O)]) ** 4
    s = c.sum(axis=0)
    a = c / np.where(s > 0, s, 1.0)
    flat = (r == 0) | (FX == -0.5) | (FY == -0.5)
    a[:, flat] = 1.0 / O
    return a


def finish(pc, ymag, edge):
    """Blur, YIQ recombine, YIQ->RGB, crop: the reference's post stages (np_twin)."""
    N = pc.shape[0]
    yb = T.blur(ymag, edge)
    yiq = np.stack([yb, pc[..., 1], pc[..., 2]], axis=-1)
    rgb = np.clip(yiq @ T.M_YIQ2RGB.T, 0.0, 1.0)
    return rgb, yb


class SteerableRef:
    def __init__(self, W, H, levels=5, min_freq=0.05, max_freq=0.45, phase_scale=10.0,
                 orientations=8, filt=FILTER_DIFF, r_low=0.05, r_high=0.4, tau=0.01, edge=0):
        self.W, self.H = W, H
        self.N = T.next_pow2(max(W, H))
        self.L, self.S, self.O = levels, phase_scale, orientations
        self.filt, self.rl, self.rh, self.tau, self.edge = filt, r_low, r_high, tau, edge
        m = T.masks(self.N, levels, min_freq, max_freq)
        self.res = m[0] + (m[-1] if levels > 1 else 0)
        a = angular_masks(self.N, orientations)
        self.bands = [(i, o) for i in range(1, levels - 1) for o in range(orientations // 2)]
        self.m, self.a = m, a
        self.state = None

    def _ifft2c(self, X):
        return sfft.ifft2(sfft.ifftshift(X), workers=1 if WORKERS > 1 else None)

    def _band(self, F, i, o, st):
        """One subband: (2 Re s', its new state), or the first frame's state."""
        s = self._ifft2c(F * (self.m[i] * self.a[o]))
        ph = np.arctan2(s.imag, s.real)
        if st is None:
            z = np.zeros(s.shape) if self.filt == FILTER_IIR else None
            return None, (ph, z, None if z is None else z.copy())
        ph_prev, uh, ul = st
        if self.filt == FILTER_DIFF:
            P = T.wrap_phase(ph_prev - ph)
        else:
            d = T.wrap_phase(ph - ph_prev)
            uh = (1.0 - self.rh) * (uh + d)
            ul = (1.0 - self.rl) * (ul + d)
            P = ul - uh
        # Re(s e^{i S P}) where |s| >= tau, Re(s) elsewhere
        SP = self.S * P
        re = np.where(np.hypot(s.real, s.imag) < self.tau, s.real, s.real * np.cos(SP) - s.imag * np.sin(SP))
        return 2.0 * re, (ph, uh, ul)

    def process(self, frame):
        """frame: float RGBA [H, W, 4] in [0, 1]; returns the output frame.
        The subbands are formed one per task (the 2160p, O = 8 case holds 16
        of them: 4 GB at once otherwise), WORKERS tasks at a time."""
        pc = T.pad_window(frame.astype(np.float64), self.N, self.edge)
        F = sfft.fftshift(sfft.fft2(pc[..., 0], workers=WORKERS))
        first = self.state is None
        prev = [None] * len(self.bands) if first else self.state
        jobs = [(i, o, st) for (i, o), st in zip(self.bands, prev)]
        if WORKERS > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(WORKERS) as ex:
                res = list(ex.map(lambda j: self._band(F, *j), jobs))
        else:
            res = [self._band(F, *j) for j in jobs]
        self.state = [r[1] for r in res]
        if first:                                   # first frame: passthrough
            return frame.copy()
        y = np.real(self._ifft2c(F * self.res))
        for r in res:
            y = y + r[0]
        rgb, _ = finish(pc, np.abs(y), self.edge)
        N, W, H = self.N, self.W, self.H
        tx = ((N - W) + 2 * np.arange(W)) / 2.0
        ty = ((N - H) + 2 * np.arange(H)) / 2.0
        TX, TY = np.meshgrid((tx + 0.5) / N, (ty + 0.5) / N)
        out = np.ones((H, W, 4))
        out[..., :3] = T._bilinear(rgb, TX, TY, self.edge)
        return out
