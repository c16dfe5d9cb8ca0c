"""ctypes binding of include/mm.h (lib/libmm355.so)."""
import ctypes
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "lib", "libmm355.so")
HEADER = os.path.join(REPO_ROOT, "include", "mm.h")

RGBA8 = 0
RGBA32F = 1
RGBA16F = 2         # linear half (the reference camera's HDR target), ABI 10
RGBA8_SRGB = 3      # 8-bit sRGB target in Linear colour space, ABI 10
FORMAT_BPP = {RGBA8: 4, RGBA32F: 16, RGBA16F: 8, RGBA8_SRGB: 4}
EDGE_REPEAT = 0
EDGE_CLAMP = 1
MODE_PYRAMID = 0
MODE_STANDARD = 1
MODE_STEERABLE = 2      # extension f2 (oracle/steerable_ref.py)
FILTER_DIFF = 0
FILTER_IIR = 1
FRAMES_ON_DEVICE = 1

KERNELS = ("k_rows_fwd", "k_cols", "k_rows_inv", "k_compose",
           "k_rows_inv_compose")   # MM_K_* ids 0..4

ERRORS = {0: "MM_OK", -1: "MM_ERR_INVALID", -2: "MM_ERR_UNSUPPORTED", -3: "MM_ERR_HIP",
          -4: "MM_ERR_NO_DEVICE", -5: "MM_ERR_OOM", -6: "MM_ERR_NO_STATE"}


class MMError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        name = ERRORS.get(code, str(code))
        super().__init__(f"{what}: {name} ({strerror(code) if _lib else ''})")


class Params(ctypes.Structure):
    """mm_params — the inspector fields of the reference (.cs:12-31)."""
    _fields_ = [("levels", ctypes.c_int), ("min_freq", ctypes.c_float),
                ("max_freq", ctypes.c_float), ("phase_scale", ctypes.c_float),
                ("magnitude_threshold", ctypes.c_float), ("orientations", ctypes.c_int),
                ("mode", ctypes.c_int), ("edge_mode", ctypes.c_int),
                ("apply_magnification", ctypes.c_int),
                ("apply_bandpass_filter", ctypes.c_int), ("low_frequency_cutoff", ctypes.c_float),
                ("high_frequency_cutoff", ctypes.c_float), ("filter_steepness", ctypes.c_float),
                ("motion_sensitivity", ctypes.c_float), ("enhance_edges", ctypes.c_int),
                ("edge_enhancement", ctypes.c_float),
                ("show_magnitude", ctypes.c_int), ("show_phase", ctypes.c_int),
                ("temporal_filter", ctypes.c_int), ("iir_low", ctypes.c_float),
                ("iir_high", ctypes.c_float)]

    @classmethod
    def make(cls, levels=5, min_freq=0.05, max_freq=0.45, phase_scale=10.0,
             magnitude_threshold=0.01, edge_mode=EDGE_REPEAT, apply_magnification=True,
             mode=MODE_PYRAMID, **standard):
        """other mm.h fields by keyword: the standard-mode band-pass
        (apply_bandpass_filter, low_frequency_cutoff, high_frequency_cutoff,
        filter_steepness, motion_sensitivity, enhance_edges, edge_enhancement)
        the debug views (show_magnitude, show_phase) and the steerable
        extension (orientations, temporal_filter, iir_low, iir_high)."""
        p = cls()
        lib().mm_params_default(ctypes.byref(p))
        p.levels, p.min_freq, p.max_freq = levels, min_freq, max_freq
        p.phase_scale, p.magnitude_threshold = phase_scale, magnitude_threshold
        p.edge_mode, p.apply_magnification = edge_mode, 1 if apply_magnification else 0
        p.mode = mode
        for k, v in standard.items():
            if k not in dict(cls._fields_):
                raise TypeError(f"unknown mm_params field {k}")
            setattr(p, k, int(v) if k in ("apply_bandpass_filter", "enhance_edges",
                                          "show_magnitude", "show_phase", "orientations",
                                          "temporal_filter") else v)
        return p


_lib = None
_lib_path = None
ABI_VERSION = 10  # include/mm.h MM_ABI_VERSION


def load_library(path=None):
    """Load the HIP product library; raises if it is missing (no fallback).
    MM355_LIB overrides the path (A/B builds of the same library)."""
    global _lib, _lib_path
    if _lib is not None:
        return _lib
    path = path or os.environ.get("MM355_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise MMError(-3, f"HIP library not built: {path} (run __graft_entry__.build())")
    L = ctypes.CDLL(path)
    vp, ci, cf, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    pp = ctypes.POINTER(Params)
    sigs = {
        "mm_abi_version": (ci, []),
        "mm_strerror": (ctypes.c_char_p, [ci]),
        "mm_params_default": (ci, [pp]),
        "mm_create": (ci, [ci, ci, pp, ci, ctypes.POINTER(vp)]),
        "mm_set_params": (ci, [vp, pp]),
        "mm_get_params": (ci, [vp, pp]),
        "mm_padded_size": (ci, [vp, ctypes.POINTER(ci)]),
        "mm_frame_bytes": (ci, [ci, ci, ci, ctypes.POINTER(sz)]),
        "mm_process": (ci, [vp, vp, vp, ci, ci, vp]),
        "mm_process_stream": (ci, [vp, vp, vp, ci, ci, vp]),
        "mm_reset": (ci, [vp]),
        "mm_state_size": (ci, [vp, ctypes.POINTER(sz)]),
        "mm_get_state": (ci, [vp, vp, sz, vp]),
        "mm_set_state": (ci, [vp, vp, sz, vp]),
        "mm_compute_state": (ci, [vp, vp, ci, vp, sz, vp]),
        "mm_stream": (vp, [vp]),
        "mm_set_batch": (ci, [vp, ci]),
        "mm_get_batch": (ci, [vp, ctypes.POINTER(ci)]),
        "mm_destroy": (None, [vp]),
        "mm_synth_frames": (ci, [vp, ci, ci, ci, ci, ctypes.c_uint64, ci, vp]),
        "mm_resample_table": (ci, [ci, ci, ci, ci, ctypes.POINTER(ctypes.c_int32),
                                   ctypes.POINTER(cf)]),
        "mm_import_frames": (ci, [vp, ci, sz, sz, ctypes.POINTER(vp)]),
        "mm_ext_frames_ptr": (vp, [vp]),
        "mm_release_frames": (ci, [vp]),
        "mm_profile_begin": (ci, [vp]),
        "mm_profile_end": (ci, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ci),
                                ctypes.POINTER(ci)]),
    }
    abi = L.mm_abi_version()
    for name, (res, args) in sigs.items():
        if abi < 5 and name in ("mm_set_batch", "mm_get_batch"):
            continue
        if abi < 6 and name in ("mm_import_frames", "mm_ext_frames_ptr", "mm_release_frames"):
            continue
        if abi < 10 and name == "mm_frame_bytes":
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    # mm_params grows only at its end: an older library (ABI >= 2) reads a prefix
    # of Params (A/B builds); a newer one than this binding is refused.
    if abi > ABI_VERSION or abi < 2:
        raise MMError(-1, f"{path}: ABI {abi}, binding expects <= {ABI_VERSION}")
    _lib = L
    _lib_path = os.path.realpath(path)
    return L


def library_path():
    """Real path of the libmm355 build this process loaded (MM355_LIB or the tree's)."""
    load_library()
    return _lib_path


def lib():
    return load_library()


def strerror(code):
    return lib().mm_strerror(code).decode()


def check(rc, what):
    if rc != 0:
        raise MMError(rc, what)


def abi_symbols():
    """Function names declared in include/mm.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mm_[a-z_0-9]+)\s*\(", txt)))


def frame_bytes(width, height, fmt):
    """mm_frame_bytes: bytes of one W x H frame of `fmt`."""
    n = ctypes.c_size_t()
    check(lib().mm_frame_bytes(width, height, fmt, ctypes.byref(n)), "mm_frame_bytes")
    return n.value


def resample_table(width, height, axis, edge_mode=EDGE_REPEAT):
    n = width if axis == 0 else height
    idx = np.zeros((n, 4), np.int32)
    w = np.zeros((n, 4), np.float32)
    check(lib().mm_resample_table(width, height, axis, edge_mode,
                                  idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                  w.ctypes.data_as(ctypes.POINTER(ctypes.c_float))),
          "mm_resample_table")
    return idx, w


def _ptr(x):
    """Device/host address of a torch tensor, numpy array or int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take the address of {type(x)}")


class Handle:
    """One mm_handle (one video stream on one GPU)."""

    def __init__(self, width, height, params=None, device=0):
        self.width, self.height = width, height
        self.params = params if params is not None else Params.make()
        h = ctypes.c_void_p()
        check(lib().mm_create(width, height, ctypes.byref(self.params), device, ctypes.byref(h)),
              "mm_create")
        self.h = h
        n = ctypes.c_int()
        check(lib().mm_padded_size(self.h, ctypes.byref(n)), "mm_padded_size")
        self.N = n.value

    @property
    def state_bytes(self):
        """mm_state_size: follows the current parameters (the steerable mode's
        state depends on levels, orientations and temporal filter)."""
        s = ctypes.c_size_t()
        check(lib().mm_state_size(self.h, ctypes.byref(s)), "mm_state_size")
        return s.value

    def set_batch(self, frames):
        check(lib().mm_set_batch(self.h, int(frames)), "mm_set_batch")

    @property
    def batch(self):
        n = ctypes.c_int()
        check(lib().mm_get_batch(self.h, ctypes.byref(n)), "mm_get_batch")
        return n.value

    def close(self):
        if getattr(self, "h", None):
            lib().mm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib().mm_stream(self.h)

    def set_params(self, params):
        self.params = params
        check(lib().mm_set_params(self.h, ctypes.byref(params)), "mm_set_params")

    def process(self, src, dst, fmt, on_device=True, stream=None):
        check(lib().mm_process(self.h, _ptr(src), _ptr(dst), fmt,
                               FRAMES_ON_DEVICE if on_device else 0, _ptr(stream)),
              "mm_process")

    def process_stream(self, src, dst, count, fmt, stream=None):
        check(lib().mm_process_stream(self.h, _ptr(src), _ptr(dst), count, fmt, _ptr(stream)),
              "mm_process_stream")

    def reset(self):
        check(lib().mm_reset(self.h), "mm_reset")

    def get_state(self, dev_buf, stream=None):
        check(lib().mm_get_state(self.h, _ptr(dev_buf), self.state_bytes, _ptr(stream)),
              "mm_get_state")

    def set_state(self, dev_buf, stream=None):
        check(lib().mm_set_state(self.h, _ptr(dev_buf), self.state_bytes, _ptr(stream)),
              "mm_set_state")

    def compute_state(self, src, fmt, dev_buf, stream=None):
        check(lib().mm_compute_state(self.h, _ptr(src), fmt, _ptr(dev_buf), self.state_bytes,
                                     _ptr(stream)), "mm_compute_state")

    def profile_begin(self):
        check(lib().mm_profile_begin(self.h), "mm_profile_begin")

    def profile_end(self):
        """-> {kernel: (total_ms, launches, frames)} for every kernel of the path."""
        k = len(KERNELS)
        ms = (ctypes.c_double * k)()
        n = (ctypes.c_int * k)()
        f = (ctypes.c_int * k)()
        check(lib().mm_profile_end(self.h, ms, n, f), "mm_profile_end")
        return {name: (ms[k], n[k], f[k]) for k, name in enumerate(KERNELS)}

    def synth(self, dev_out, t0, count, seed=0x5EED0000, gray=False, stream=None):
        check(lib().mm_synth_frames(_ptr(dev_out), self.width, self.height, t0, count, seed,
                                    1 if gray else 0, _ptr(stream)), "mm_synth_frames")
