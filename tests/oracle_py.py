"""ctypes binding of the CPU oracle (oracle/libmm_ref.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "libmm_ref.so")

EDGE_REPEAT = 0
EDGE_CLAMP = 1

_lib = None


class Dbg(ctypes.Structure):
    _fields_ = [(n, ctypes.POINTER(ctypes.c_float)) for n in
                ("y_cur", "F_cur", "F_prev", "A", "y_mag", "y_blur")]


def build():
    src = os.path.join(ORACLE_DIR, "mm_ref.c")
    if (not os.path.exists(LIB_PATH)
            or os.path.getmtime(LIB_PATH) < os.path.getmtime(src)):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        vp = ctypes.c_void_p
        L.mm_ref_create.restype = vp
        L.mm_ref_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                    ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.mm_ref_destroy.argtypes = [vp]
        L.mm_ref_padded_size.argtypes = [vp]
        L.mm_ref_set_params.argtypes = [vp, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.mm_ref_set_apply.argtypes = [vp, ctypes.c_int]
        cf = ctypes.c_float
        L.mm_ref_set_standard.argtypes = [vp, ctypes.c_int, ctypes.c_int, cf, cf, cf, cf, cf]
        L.mm_ref_bandpass_weights.argtypes = [ctypes.c_int, ctypes.c_int, cf, cf, cf, cf, cf, fp]
        L.mm_ref_reset.argtypes = [vp]
        L.mm_ref_state_size.restype = ctypes.c_size_t
        L.mm_ref_state_size.argtypes = [vp]
        L.mm_ref_get_state.argtypes = [vp, vp]
        L.mm_ref_set_state.argtypes = [vp, vp]
        L.mm_ref_process.argtypes = [vp, fp, fp, ctypes.POINTER(Dbg)]
        L.mm_ref_process_u8.argtypes = [vp, u8p, u8p]
        L.mm_ref_process_f16.argtypes = [vp, vp, vp]
        L.mm_ref_process_srgb8.argtypes = [vp, u8p, u8p]
        L.mm_ref_srgb_tables.argtypes = [fp, fp]
        L.mm_ref_half_to_float.restype = ctypes.c_float
        L.mm_ref_half_to_float.argtypes = [ctypes.c_uint16]
        L.mm_ref_float_to_half.restype = ctypes.c_uint16
        L.mm_ref_float_to_half.argtypes = [ctypes.c_float]
        L.mm_ref_fft_centered.argtypes = [ctypes.c_int, fp, fp]
        L.mm_ref_ifft_mag.argtypes = [ctypes.c_int, fp, fp]
        L.mm_ref_mask.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                  ctypes.c_float, fp]
        L.mm_ref_normalize_phase.restype = ctypes.c_float
        L.mm_ref_normalize_phase.argtypes = [ctypes.c_float]
        L.mm_ref_rgb_to_yiq.argtypes = [fp, fp]
        L.mm_ref_yiq_to_rgb.argtypes = [fp, fp]
        L.mm_ref_pad_window.argtypes = [vp, fp, fp]
        L.mm_ref_blur.argtypes = [ctypes.c_int, ctypes.c_int, fp]
        L.mm_ref_synth_frame.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_uint64, ctypes.c_int, u8p]
        L.mm_ref_set_debug.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.mm_ref_fft_buffer1.argtypes = [ctypes.c_int, fp, fp]
        L.mm_ref_set_threads.argtypes = [ctypes.c_int]
        L.mm_ref_set_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _fp(a):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u8p(a):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def set_threads(n):
    return lib().mm_ref_set_threads(n)


def synth_frame(width, height, t, seed=0x5EED0000, gray=False):
    out = np.empty((height, width, 4), np.uint8)
    lib().mm_ref_synth_frame(width, height, t, seed, 1 if gray else 0, _u8p(out))
    return out


def srgb_tables():
    """(dec[256], thr[257]) of MM_RGBA8_SRGB (include/mm.h), as the oracle builds them."""
    dec = np.empty(256, np.float32)
    thr = np.empty(257, np.float32)
    lib().mm_ref_srgb_tables(_fp(dec), _fp(thr))
    return dec, thr


def float_to_half_bits(v):
    return lib().mm_ref_float_to_half(v)


def half_bits_to_float(b):
    return lib().mm_ref_half_to_float(b)


def fft_centered(y):
    y = np.ascontiguousarray(y, np.float32)
    n = y.shape[0]
    out = np.empty((n, n, 2), np.float32)
    lib().mm_ref_fft_centered(n, _fp(y), _fp(out))
    return out[..., 0] + 1j * out[..., 1].astype(np.complex64)


def fft_buffer1(y):
    """complexBuffer1 after PerformFFT (what ProcessDebugView reads)."""
    y = np.ascontiguousarray(y, np.float32)
    n = y.shape[0]
    out = np.empty((n, n, 2), np.float32)
    lib().mm_ref_fft_buffer1(n, _fp(y), _fp(out))
    return out[..., 0] + 1j * out[..., 1].astype(np.complex64)


def ifft_mag(A):
    n = A.shape[0]
    a = np.ascontiguousarray(np.stack([A.real, A.imag], -1).astype(np.float32))
    out = np.empty((n, n), np.float32)
    lib().mm_ref_ifft_mag(n, _fp(a), _fp(out))
    return out


def mask(n, levels, index, minf, maxf):
    out = np.empty((n, n), np.float32)
    lib().mm_ref_mask(n, levels, index, minf, maxf, _fp(out))
    return out


def normalize_phase(p):
    return lib().mm_ref_normalize_phase(p)


def rgb_to_yiq(rgb):
    a = np.ascontiguousarray(rgb, np.float32)
    o = np.empty(3, np.float32)
    lib().mm_ref_rgb_to_yiq(_fp(a), _fp(o))
    return o


def yiq_to_rgb(yiq):
    a = np.ascontiguousarray(yiq, np.float32)
    o = np.empty(3, np.float32)
    lib().mm_ref_yiq_to_rgb(_fp(a), _fp(o))
    return o


def bandpass_weights(n, apply=True, low=0.05, high=0.4, steep=3.0, sens=1.5, edge=0.8):
    out = np.empty((n, n), np.float32)
    lib().mm_ref_bandpass_weights(n, 1 if apply else 0, low, high, steep, sens, edge, _fp(out))
    return out


def blur(img, edge=EDGE_REPEAT):
    a = np.ascontiguousarray(img, np.float32).copy()
    lib().mm_ref_blur(a.shape[0], edge, _fp(a))
    return a


class Oracle:
    """The reference operator on the CPU (one handle = one camera stream)."""

    def __init__(self, width, height, levels=5, min_freq=0.05, max_freq=0.45,
                 phase_scale=10.0, mag_threshold=0.01, edge_mode=EDGE_REPEAT):
        self.W, self.H = width, height
        self.h = lib().mm_ref_create(width, height, levels, min_freq, max_freq,
                                     phase_scale, mag_threshold, edge_mode)
        if not self.h:
            raise ValueError("mm_ref_create failed")
        self.N = lib().mm_ref_padded_size(self.h)

    def close(self):
        if self.h:
            lib().mm_ref_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def set_params(self, levels, min_freq, max_freq, phase_scale, mag_threshold=0.01,
                   edge_mode=EDGE_REPEAT):
        lib().mm_ref_set_params(self.h, levels, min_freq, max_freq, phase_scale,
                                mag_threshold, edge_mode)

    def set_apply(self, on):
        lib().mm_ref_set_apply(self.h, 1 if on else 0)

    def set_standard(self, on=True, apply=True, low=0.05, high=0.4, steep=3.0, sens=1.5,
                     edge=0.8):
        """usePyramidDecomposition = false; edge = enhanceEdges ? edgeEnhancement : 0."""
        lib().mm_ref_set_standard(self.h, 1 if on else 0, 1 if apply else 0, low, high, steep,
                                  sens, edge)

    def set_debug(self, show_magnitude=False, show_phase=False):
        """showMagnitude / showPhase (.cs:13-14): ProcessDebugView output."""
        lib().mm_ref_set_debug(self.h, 1 if show_magnitude else 0, 1 if show_phase else 0)

    def reset(self):
        lib().mm_ref_reset(self.h)

    def get_state(self):
        buf = np.empty(lib().mm_ref_state_size(self.h), np.uint8)
        lib().mm_ref_get_state(self.h, buf.ctypes.data)
        return buf

    def set_state(self, buf):
        buf = np.ascontiguousarray(buf, np.uint8)
        lib().mm_ref_set_state(self.h, buf.ctypes.data)

    def process_srgb8(self, frame):
        """frame: uint8 [H,W,4] sRGB-encoded (MM_RGBA8_SRGB); returns the same."""
        a = np.ascontiguousarray(frame, np.uint8)
        out = np.empty_like(a)
        lib().mm_ref_process_srgb8(self.h, _u8p(a), _u8p(out))
        return out

    def process(self, frame, dbg=False):
        """frame: float32, float16 (MM_RGBA16F) or uint8 (UNORM) [H,W,4];
        returns the same dtype."""
        if frame.dtype == np.float16:
            a = np.ascontiguousarray(frame)
            out = np.empty_like(a)
            lib().mm_ref_process_f16(self.h, a.ctypes.data, out.ctypes.data)
            return out
        if frame.dtype == np.uint8:
            a = np.ascontiguousarray(frame)
            out = np.empty_like(a)
            lib().mm_ref_process_u8(self.h, _u8p(a), _u8p(out))
            return out
        a = np.ascontiguousarray(frame, np.float32)
        out = np.empty_like(a)
        if not dbg:
            lib().mm_ref_process(self.h, _fp(a), _fp(out), None)
            return out
        N = self.N
        bufs = dict(y_cur=np.zeros((N, N), np.float32), F_cur=np.zeros((N, N, 2), np.float32),
                    F_prev=np.zeros((N, N, 2), np.float32), A=np.zeros((N, N, 2), np.float32),
                    y_mag=np.zeros((N, N), np.float32), y_blur=np.zeros((N, N), np.float32))
        d = Dbg(**{k: _fp(v) for k, v in bufs.items()})
        lib().mm_ref_process(self.h, _fp(a), _fp(out), ctypes.byref(d))
        for k in ("F_cur", "F_prev", "A"):
            bufs[k] = bufs[k][..., 0] + 1j * bufs[k][..., 1].astype(np.complex64)
        return out, bufs
