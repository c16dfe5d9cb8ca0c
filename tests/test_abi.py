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
    assert L.mm_abi_version() == 9


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
