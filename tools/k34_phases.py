#!/usr/bin/env python3
"""k_rows_inv_compose phase breakdown from a diagnostic build (-DMM_K34_STAMPS):
cycles per strip step of each phase, averaged over waves (s_memtime deltas taken
by every wave).

usage: MM355_LIB=lib/variants/k34st.so python3 tools/k34_phases.py [frames]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-based-motion-manipulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mm355  # noqa: E402

PHASES = ["Q loads+unpack", "inv FFT", "|z| + barrier", "blur + barrier", "chroma loads", "compose+stores"]
W, H = 1920, 1080
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
h.set_batch(n)
fr = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
out = torch.empty_like(fr)
h.synth(fr, 0, n)
h.process_stream(fr, out, n, mm355.RGBA8)
torch.cuda.synchronize()
h.process_stream(fr, out, n, mm355.RGBA8)      # the launch whose stamps are read
torch.cuda.synchronize()
L = mm355.lib()
nw = 65536
buf = (ctypes.c_ulonglong * (nw * 8))()
L.mm_debug_k34_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.mm_debug_k34_stamps(buf, nw * 8) == 0
raw = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 8)
live = raw[raw[:, 6] > 0]
steps = live[:, 6].astype(np.float64)
a = live[:, :len(PHASES)].astype(np.float64) / steps[:, None]
dur = (live[:, 7] >> 32).astype(np.float64) * 10.0
res = {"frames": n, "waves": int(live.shape[0]), "steps": int(steps[0]),
       "cycles_per_step_mean": {p: round(float(a[:, i].mean()), 1) for i, p in enumerate(PHASES)},
       "total_per_step_mean": round(float(a.sum(axis=1).mean()), 1),
       "walk_duration_us": {q: round(float(np.percentile(dur, q)) / 1e3, 2) for q in (0, 50, 90, 100)}}
print(json.dumps(res))
