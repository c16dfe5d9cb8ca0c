"""C-ABI library checks that need no GPU: it loads, exports every symbol that
include/mm.h declares, reports errors without crashing, and its host-side
geometry tables match the oracle's literal two-step resample."""
import ctypes
import subprocess

import numpy as np
import pytest

import mm355
import oracle_py as O


def test_library_loads_and_exports_header_symbols():
    L = mm355.load_library()
    syms = mm355.abi_symbols()
    assert len(syms) >= 18
    out = subprocess.run(["nm", "-D", "--defined-only", mm355.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    for s in syms:
        assert hasattr(L, s)
    assert L.mm_abi_version() == 10


def test_strerror_and_defaults():
    assert mm355.strerror(0) == "ok"
    assert "state" in mm355.strerror(-6)
    p = mm355.Params()
    assert mm355.lib().mm_params_default(ctypes.byref(p)) == 0
    assert (p.levels, round(p.min_freq, 3), round(p.max_freq, 3), p.phase_scale) == (5, 0.05, 0.45, 10.0)
    assert abs(p.magnitude_threshold - 0.01) < 1e-9 and p.orientations == 1


def test_create_rejects_bad_arguments_without_gpu():
    p = mm355.Params.make()
    h = ctypes.c_void_p()
    L = mm355.lib()
    st = mm355.Params.make(mode=mm355.MODE_STEERABLE, orientations=8)
    assert L.mm_create(8193, 48, ctypes.byref(p), 0, ctypes.byref(h)) == -2  # N > 8192
    assert L.mm_create(5120, 48, ctypes.byref(st), 0, ctypes.byref(h)) == -2  # steerable: N <= 4096
    assert L.mm_create(16385, 2160, ctypes.byref(p), 0, ctypes.byref(h)) == -2  # N = 32768
    assert L.mm_create(8, 6, ctypes.byref(p), 0, ctypes.byref(h)) == -2      # N = 8 < 16
    assert L.mm_create(2, 2, ctypes.byref(p), 0, ctypes.byref(h)) == -2      # N = 2
    assert not h.value                                                       # nothing created
    # odd sizes are accepted in steerable mode too (round 5): only the device is missing here
    assert L.mm_create(63, 47, ctypes.byref(st), 0, ctypes.byref(h)) in (-4, 0)
    if h.value:
        L.mm_destroy(h)
        h = ctypes.c_void_p()
    bad = mm355.Params.make()
    bad.orientations = 8
    assert L.mm_create(64, 48, ctypes.byref(bad), 0, ctypes.byref(h)) == -2
    assert L.mm_create(64, 48, None, 0, ctypes.byref(h)) == -1
    assert L.mm_process(None, None, None, 0, 0, None) == -1
    assert L.mm_reset(None) == -1


def test_create_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(mm355.MMError) as ei:
        mm355.Handle(64, 48)
    assert ei.value.code == -4                     # MM_ERR_NO_DEVICE, no CPU fallback


@pytest.mark.parametrize("W,H,edge", [(64, 48, 0), (64, 48, 1), (1920, 1080, 0), (200, 120, 1),
                                      (256, 256, 0), (63, 47, 0), (65, 49, 1), (1919, 1079, 0)])
def test_resample_table_matches_oracle_pad(W, H, edge):
    """The composite (stretch x pad x Hann) taps reproduce the oracle's literal
    two-step bilinear pad of a separable test image."""
    o = O.Oracle(W, H, edge_mode=edge)
    N = o.N
    rng = np.random.default_rng(3)
    cx, cy = rng.random(W).astype(np.float32), rng.random(H).astype(np.float32)
    img = np.zeros((H, W, 4), np.float32)
    img[..., 0] = img[..., 1] = img[..., 2] = cy[:, None] * cx[None, :]
    img[..., 3] = 1
    canvas = np.zeros((N, N, 4), np.float32)
    O.lib().mm_ref_pad_window(o.h, O._fp(img), O._fp(canvas))
    ix, wx = mm355.resample_table(W, H, 0, edge)
    iy, wy = mm355.resample_table(W, H, 1, edge)
    rx = (wx * cx[ix]).sum(1)
    ry = (wy * cy[iy]).sum(1)
    x0, y0 = (N - W) // 2, (N - H) // 2
    got = ry[:, None] * rx[None, :]
    ref = canvas[y0:y0 + H, x0:x0 + W, 0]      # luma of gray = value
    assert np.abs(got - ref).max() < 2e-6


def test_processor_params_mirror_inspector_fields():
    """MotionMagnificationProcessor fields -> mm_params (host only, no handle)."""
    P = mm355.MotionMagnificationProcessor
    p = P(64, 48, pyramid_levels=4, phase_scale=25.0)._params()
    assert (p.mode, p.levels, p.orientations) == (mm355.MODE_PYRAMID, 4, 1)
    assert abs(p.phase_scale - 25.0) < 1e-6
    assert P(64, 48, use_pyramid_decomposition=False)._params().mode == mm355.MODE_STANDARD
    d = mm355.Params.make()
    s = P(64, 48, orientations=8)._params()
    assert (s.mode, s.orientations, s.temporal_filter) == (mm355.MODE_STEERABLE, 8, mm355.FILTER_DIFF)
    assert (s.iir_low, s.iir_high) == (d.iir_low, d.iir_high)
    s = P(64, 48, orientations=4, temporal_filter=mm355.FILTER_IIR, iir_low=0.1, iir_high=0.5)._params()
    assert (s.mode, s.orientations, s.temporal_filter) == (mm355.MODE_STEERABLE, 4, mm355.FILTER_IIR)
    assert abs(s.iir_low - 0.1) < 1e-7 and abs(s.iir_high - 0.5) < 1e-7


def test_unity_shim_calls_only_declared_entry_points():
    """The Unity rendering-plugin shim (source only: no Unity/Vulkan SDK here)
    calls only entry points include/mm.h declares and the library exports."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(mm355.LIB_PATH), "..", "unity", "mm_unity_plugin.c")).read()
    body = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    called = set(re.findall(r"\b(mm_[a-z_0-9]+)\s*\(", body))
    own = {"mm_unity_create", "mm_unity_event_func", "mm_unity_event_ok", "mm_unity_destroy"}
    declared = set(mm355.abi_symbols())
    assert own <= called
    assert called - own <= declared, called - own - declared
    for s in called - own:
        assert hasattr(mm355.lib(), s)
    for entry in ("UnityPluginLoad", "UnityPluginUnload", "IssuePluginEventAndData"):
        assert entry in src


def test_frame_formats_and_sizes():
    """MM_RGBA16F / MM_RGBA8_SRGB (ABI 10): format codes, bytes per frame, and
    unknown formats refused by every frame entry point (no GPU needed)."""
    assert (mm355.RGBA8, mm355.RGBA32F, mm355.RGBA16F, mm355.RGBA8_SRGB) == (0, 1, 2, 3)
    for f, bpp in mm355.FORMAT_BPP.items():
        assert mm355.frame_bytes(1920, 1080, f) == 1920 * 1080 * bpp
    with pytest.raises(mm355.MMError):
        mm355.frame_bytes(64, 48, 4)
    with pytest.raises(mm355.MMError):
        mm355.frame_bytes(0, 48, 0)
    hdr = open(mm355.binding.HEADER).read()
    assert "#define MM_RGBA16F    2" in hdr and "#define MM_RGBA8_SRGB 3" in hdr
    P = mm355.processor._fmt_of
    assert P(np.zeros(1, np.uint8)) == mm355.RGBA8 and P(np.zeros(1, np.uint8), True) == mm355.RGBA8_SRGB
    assert P(np.zeros(1, np.float16)) == mm355.RGBA16F and P(np.zeros(1, np.float32)) == mm355.RGBA32F


def test_srgb_tables_kernel_header_equals_oracle():
    """The kernels' sRGB tables (csrc/mm_srgb.hpp, tools/gen_srgb.py) are the
    oracle's bit for bit, and encode(decode(b)) == b for every byte."""
    import os
    import re
    txt = open(os.path.join(os.path.dirname(mm355.LIB_PATH), "..", "csrc", "mm_srgb.hpp")).read()
    vals = np.array([float.fromhex(v) for v in re.findall(r"(-?0x[0-9a-f.p+-]+)f", txt)], np.float32)
    dec, thr = O.srgb_tables()
    assert vals.size == 256 + 255
    assert np.array_equal(vals[:256].view(np.uint32), dec.view(np.uint32))
    assert np.array_equal(vals[256:].view(np.uint32), thr[1:256].view(np.uint32))
    assert np.isneginf(thr[0]) and np.isposinf(thr[256]) and np.all(np.diff(thr) > 0)
    enc = np.searchsorted(thr, dec, side="right") - 1      # largest b with dec >= thr[b]
    assert np.array_equal(enc, np.arange(256))
    # the curve's known points: 0 -> 0, 255 -> 1, byte 188 ~ 0.5 linear (IEC 61966-2-1)
    assert dec[0] == 0.0 and dec[255] == 1.0 and abs(dec[188] - 0.50289) < 1e-4


def test_oracle_half_conversions_match_ieee():
    """The oracle's binary16 codecs (MM_RGBA16F) against numpy's IEEE ones:
    every half decodes exactly, floats round to nearest even (subnormals,
    the overflow edge and ties included)."""
    h = np.arange(0, 65536, 257, dtype=np.uint16)
    got = np.array([O.half_bits_to_float(int(b)) for b in h], np.float32)
    ref = h.view(np.float16).astype(np.float32)
    fin = ~np.isnan(ref)
    assert np.array_equal(got[fin], ref[fin]) and np.all(np.isnan(got[~fin]))
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(4000) * 10.0 ** rng.integers(-9, 5, 4000)).astype(np.float32)
    ties = (np.arange(1, 200, dtype=np.float32) + np.float32(0.5)) * np.float32(2.0 ** -24)
    x = np.concatenate([x, ties, np.array([65504, 65519.99, 65520, 6.1e-5, 5.96e-8, 2.98e-8], np.float32)])
    got = np.array([O.float_to_half_bits(float(v)) for v in x], np.uint16)
    with np.errstate(over="ignore"):
        assert np.array_equal(got, x.astype(np.float16).view(np.uint16))


def _build_variant(tmp, name):
    """A copy of the tree's libmm355.so as an A/B variant <name>.so and its
    ring library <name>_ring.so, built as scripts/build_variants.sh does."""
    import os
    import shutil
    pkg = os.path.dirname(os.path.dirname(mm355.LIB_PATH))
    shutil.copy(mm355.LIB_PATH, os.path.join(tmp, name + ".so"))
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-shared", "-I" + os.path.join(pkg, "..", "include"),
                    "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-o", os.path.join(tmp, name + "_ring.so"),
                    os.path.join(pkg, "host", "mm_ring.c"), "-L" + tmp, "-l:" + name + ".so", "-L/opt/rocm/lib",
                    "-lrccl", "-lamdhip64", "-lpthread", "-ldl", "-lm", "-Wl,-rpath,$ORIGIN",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return os.path.join(tmp, name + ".so")


_RING_PROBE = """
import os, sys
sys.path.insert(0, {pkg!r})
import mm355
try:
    mm355.ring_lib()
    print("BOUND", mm355.ring.ring_lib_path(), mm355.binding.library_path())
except mm355.MMError as e:
    print("REFUSED", e)
"""


def test_ring_library_binds_the_loaded_build(tmp_path):
    """with MM355_LIB naming an A/B variant, the ring library
    that loads is the variant's own and resolves its mm_* calls to that same
    build; a ring library bound to another build (the tree's) is refused
    instead of silently running the other build's kernels."""
    import os
    import sys
    var = _build_variant(str(tmp_path), "abvar")
    pkg = os.path.dirname(os.path.dirname(mm355.LIB_PATH))
    code = _RING_PROBE.format(pkg=pkg)

    def run(**env):
        e = {k: v for k, v in os.environ.items() if k not in ("MM355_LIB", "MM355_RING_LIB")}
        e.update(env)
        return subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True,
                              check=True).stdout.strip()

    out = run(MM355_LIB=var)
    assert out.startswith("BOUND"), out
    _, ring_path, core = out.split()
    assert ring_path == os.path.join(str(tmp_path), "abvar_ring.so") and core == os.path.realpath(var)
    tree_ring = os.path.join(os.path.dirname(mm355.LIB_PATH), "libmm_ring.so")
    out = run(MM355_LIB=var, MM355_RING_LIB=tree_ring)
    assert out.startswith("REFUSED") and "bound to" in out, out
    out = run()                                   # the tree's pair
    assert out.startswith("BOUND"), out
