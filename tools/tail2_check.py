#!/usr/bin/env python3
"""Bitwise check of k_cols's second-half tails: the same 1080p stream through
handles created with MM_K2_TAIL2 = 0 and = each given percentage."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "phase-based-motion-manipulation_amd"))
import torch  # noqa: E402
import mm355  # noqa: E402

W, H, n = 1920, 1080, 120
fr = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
outs = {}
for pct in ["0"] + sys.argv[1:]:
    os.environ["MM_K2_TAIL2"] = pct
    h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
    h.set_batch(60)
    if pct == "0":
        h.synth(fr, 0, n)
    o = torch.empty_like(fr)
    h.process_stream(fr, o, n, mm355.RGBA8)
    torch.cuda.synchronize()
    h.close()
    outs[pct] = o
for pct in sys.argv[1:]:
    eq = torch.equal(outs[pct], outs["0"])
    print(f"TAIL2={pct}: bitwise equal to 0: {eq}")
    assert eq
