"""ctypes binding of include/mm_ring.h (lib/libmm_ring.so): the C host's
frame-sharded stream over an RCCL ring.

The ring library owns the data path (one ncclSend/ncclRecv of the state per
step, on its own HIP stream); Python only hands the 128-byte ring id from
rank 0 to the other ranks (any out-of-band channel: bench.py uses its
torch.distributed process group) and calls mm_ring_step per step.
"""
import ctypes
import os

from .binding import MMError, PKG_DIR, _ptr, library_path

RING_LIB_PATH = os.path.join(PKG_DIR, "lib", "libmm_ring.so")


def ring_lib_path(core=None):
    """The ring library that belongs to the libmm355 build `core` (default: the
    one this process loaded): MM355_RING_LIB, else beside it — libmm_ring.so
    next to libmm355.so, <name>_ring.so next to an A/B variant <name>.so
    (scripts/build_variants.sh builds both, the ring linked to its variant)."""
    if os.environ.get("MM355_RING_LIB"):
        return os.environ["MM355_RING_LIB"]
    core = core or library_path()
    d, b = os.path.split(core)
    if b == "libmm355.so":
        return os.path.join(d, "libmm_ring.so")
    return os.path.join(d, os.path.splitext(b)[0] + "_ring.so")
ID_BYTES = 128   # MM_RING_ID_BYTES == NCCL_UNIQUE_ID_BYTES

_rl = None


def ring_lib():
    """Load the ring library of the loaded libmm355 build (ring_lib_path);
    raises if it is not built (no fallback to another transport) or if its
    mm_* calls resolve to another libmm355 than the one this process loaded
    (two builds mixed in one process: the ring would run the other build's
    kernels on this build's handles)."""
    global _rl
    if _rl is not None:
        return _rl
    core = library_path()
    path = ring_lib_path(core)
    if not os.path.exists(path):
        raise MMError(-3, f"ring library not built: {path} (run __graft_entry__.build())")
    L = ctypes.CDLL(path)
    L.mm_ring_core_library.restype = ctypes.c_char_p
    L.mm_ring_core_library.argtypes = []
    bound = L.mm_ring_core_library()
    bound = os.path.realpath(bound.decode()) if bound else None
    if bound != core:
        raise MMError(-1, f"{path} is bound to {bound}, but this process loaded {core}: "
                          "load the ring library built with that libmm355 (MM355_RING_LIB)")
    vp, ci = ctypes.c_void_p, ctypes.c_int
    for name, res, args in (
            ("mm_ring_get_id", ci, [ctypes.c_char_p]),
            ("mm_ring_create", ci, [ci, ci, ctypes.c_char_p, ci, vp, ci, ci, ci, ci,
                                    ctypes.POINTER(vp)]),
            ("mm_ring_step", ci, [vp, ci, vp, vp, vp, vp]),
            ("mm_ring_destroy", None, [vp]),
            ("mm_ring_last_error", ctypes.c_char_p, [])):
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    _rl = L
    return L


def _check(rc, what):
    if rc != 0:
        msg = ring_lib().mm_ring_last_error() or b""
        raise MMError(rc, f"{what} [{msg.decode(errors='replace')}]")


def new_ring_id():
    """mm_ring_get_id: rank 0's ring id (bytes) for every rank."""
    buf = ctypes.create_string_buffer(ID_BYTES)
    _check(ring_lib().mm_ring_get_id(buf), "mm_ring_get_id")
    return buf.raw


class Ring:
    """One rank of the ring over a Handle's stream: `chunk` frames per step."""

    def __init__(self, world, rank, ring_id, device, handle, chunk, fmt):
        if len(ring_id) != ID_BYTES:
            raise ValueError("ring id must be 128 bytes")
        r = ctypes.c_void_p()
        _check(ring_lib().mm_ring_create(world, rank, ring_id, device, handle.h, handle.width,
                                         handle.height, chunk, fmt, ctypes.byref(r)),
               "mm_ring_create")
        self.r = r

    def step(self, step, src, dst, next_last=None, stream=None):
        """Step `step` (in order from 0): src/dst = this rank's chunk of input
        and output frames; next_last = the last input frame of this rank's
        chunk of step+1 (posts that shift ahead) or None for the last step."""
        _check(ring_lib().mm_ring_step(self.r, step, _ptr(src), _ptr(dst), _ptr(next_last),
                                       _ptr(stream)), "mm_ring_step")

    def close(self):
        if getattr(self, "r", None):
            ring_lib().mm_ring_destroy(self.r)
            self.r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
