#!/usr/bin/env python3
"""The reference's call pattern alone (OnRenderImage once per frame,
.cs:101-143): one mm_process per frame on device pointers at batch 1, for a
rocprofv3 kernel summary of the drop-in path (no HIP events around the
launches: bench.py's per-kernel events would lengthen one-frame kernels).

usage: python3 tools/perframe.py [frames] [width height]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-based-motion-manipulation_amd"))
import torch  # noqa: E402
import mm355  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
h.set_batch(1)
fr = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
out = torch.empty((2, H, W, 4), dtype=torch.uint8, device="cuda")
h.synth(fr, 0, n)
st = torch.cuda.current_stream().cuda_stream
for k in range(11):
    h.process(fr[k], out[k & 1], mm355.RGBA8, stream=st)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(11, n):
    h.process(fr[k], out[k & 1], mm355.RGBA8, stream=st)
te = time.perf_counter() - t0   # host time to enqueue every call (CPU-bound if ~ dt)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"frames": n - 11, "frames_per_s": round((n - 11) / dt, 1),
                  "us_per_frame": round(dt / (n - 11) * 1e6, 2),
                  "host_enqueue_us_per_frame": round(te / (n - 11) * 1e6, 2)}))
h.close()
