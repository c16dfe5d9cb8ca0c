#!/usr/bin/env python3
"""Do two streams' frames overlap on the GPU?  H handles (each its own HIP
stream) process C frames each (batch B) at 1920x1080 RGBA8, L = 5, S = 25:
first one after another, then all enqueued before one synchronise.  If the
concurrent time is clearly below the sequential one, K1 / K2 / K34 of
different batches fill each other's idle issue slots and memory waits, and a
handle that pipelines its own batches over two streams would gain the same.

usage: python tools/concurrency_probe.py [H] [C] [B] [reps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "phase-based-motion-manipulation_amd"))
import torch  # noqa: E402
import mm355  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 2
C = int(sys.argv[2]) if len(sys.argv) > 2 else 300
B = int(sys.argv[3]) if len(sys.argv) > 3 else 150
R = int(sys.argv[4]) if len(sys.argv) > 4 else 5
W, Hh = 1920, 1080
hs = []
for i in range(H):
    h = mm355.Handle(W, Hh, mm355.Params.make(levels=5, phase_scale=25.0))
    h.set_batch(B)
    hs.append(h)
src = [torch.empty((C, Hh, W, 4), dtype=torch.uint8, device="cuda") for _ in range(H)]
dst = [torch.empty_like(s) for s in src]
for i, h in enumerate(hs):
    h.synth(src[i], 0, C, seed=0x5EED0000 + i)
torch.cuda.synchronize()


def run(concurrent):
    t0 = time.perf_counter()
    for i, h in enumerate(hs):
        h.process_stream(src[i], dst[i], C, mm355.RGBA8)
        if not concurrent:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


for _ in range(2):   # warm-up: allocations, first launches
    run(False)
    run(True)
res = {"handles": H, "frames_each": C, "batch": B, "seq_s": [], "conc_s": []}
for _ in range(R):
    res["seq_s"].append(run(False))
    res["conc_s"].append(run(True))
s, c = min(res["seq_s"]), min(res["conc_s"])
res["seq_fps"] = H * C / s
res["conc_fps"] = H * C / c
res["gain"] = s / c
print(json.dumps(res))
for h in hs:
    h.close()
