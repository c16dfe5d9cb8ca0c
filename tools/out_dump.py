"""Diagnostic for same-call A/B builds: run one stream through the library
MM355_LIB names and write its outputs (uint8 frames) to OUT.npy, so two
builds can be compared bitwise.
usage: MM355_LIB=... python tools/out_dump.py OUT W H L O FILTER(0 diff, 1 iir) FRAMES"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "phase-based-motion-manipulation_amd"))
import mm355  # noqa: E402
import mmtest as T  # noqa: E402

out, W, H, L, O, filt, n = sys.argv[1], *map(int, sys.argv[2:8])
fr = T.synth(W, H, n, fmt="u8")
kw = dict(mode=mm355.MODE_STEERABLE, orientations=O, temporal_filter=filt) if O > 1 else {}
h = mm355.Handle(W, H, mm355.Params.make(levels=L, phase_scale=25.0, **kw))
dev = torch.from_numpy(np.stack(fr)).cuda()
o = torch.empty_like(dev)
h.process_stream(dev, o, n, mm355.RGBA8)
torch.cuda.synchronize()
np.save(out, o.cpu().numpy())
print(out, "written")
