#!/usr/bin/env python3
"""k_cols phase breakdown from a diagnostic build (-DMM_K2_STAMPS): cycles per
frame of each frame-loop phase, averaged over waves (s_memtime deltas taken by
every wave; block 0 reported separately).

usage: MM355_LIB=lib/variants/stamps.so python3 tools/k2_phases.py [frames]
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

PHASES = ["top+loads", "stores+barrier", "G wait+setup", "fwd FFT", "op", "inv FFT", "stage+barrier"]
W, H = 1920, 1080
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
h = mm355.Handle(W, H, mm355.Params.make(levels=5, phase_scale=25.0))
h.set_batch(n)
fr = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
out = torch.empty_like(fr)
h.synth(fr, 0, n)
h.process_stream(fr, out, n, mm355.RGBA8)      # warm-up (first frame passthrough)
torch.cuda.synchronize()
h.profile_begin()
h.process_stream(fr, out, n, mm355.RGBA8)      # the launch whose stamps are read
torch.cuda.synchronize()
kprof = h.profile_end()                         # HIP events around each launch on its stream
L = mm355.lib()
nw = 4096
buf = (ctypes.c_ulonglong * (nw * 8))()
L.mm_debug_k2_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert L.mm_debug_k2_stamps(buf, nw * 8) == 0
raw = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 8)
a = raw[:, :len(PHASES)].astype(np.float64) / n
start = (raw[:, 7] & 0xffffffff).astype(np.int64)      # loop start, 100 MHz ticks (low 32 bits)
dur = (raw[:, 7] >> 32).astype(np.float64) * 10.0        # loop duration, ns
waves = (h.N // 2 + 1) // 2 * 8 if False else nw
live = a[a.sum(axis=1) > 0]
res = {"frames": n, "waves": int(live.shape[0]),
       "cycles_per_frame_mean": {p: round(float(live[:, i].mean()), 1) for i, p in enumerate(PHASES)},
       "cycles_per_frame_block0": {p: round(float(a[:8, i].mean()), 1) for i, p in enumerate(PHASES)},
       "total_mean": round(float(live.sum(axis=1).mean()), 1),
       "total_max": round(float(live.sum(axis=1).max()), 1)}
tot = a.sum(axis=1)
blk = np.arange(nw) // 8
bt = np.array([tot[blk == b].max() for b in range(nw // 8)])
res["block_total_pct"] = {q: round(float(np.percentile(bt, q)), 1) for q in (0, 10, 50, 90, 99, 100)}
res["slowest_blocks"] = [int(b) for b in np.argsort(-bt)[:8]]
res["per_xcd_mean_total"] = [round(float(bt[np.arange(nw // 8) % 8 == x].mean()), 1) for x in range(8)]
s0 = start - start.min()
res["loop_start_skew_us"] = {q: round(float(np.percentile(s0, q)) / 100.0, 2) for q in (0, 50, 90, 100)}
res["loop_duration_us"] = {q: round(float(np.percentile(dur, q)) / 1e3, 1) for q in (0, 50, 90, 100)}
res["end_us_max"] = round(float((s0 * 10 + dur).max()) / 1e3, 1)
if hasattr(L, "mm_debug_k2_entry"):   # kernel entry per wave (100 MHz): dispatch skew and prologue
    eb = (ctypes.c_ulonglong * nw)()
    L.mm_debug_k2_entry.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.mm_debug_k2_entry(eb, nw) == 0
    ent = np.frombuffer(eb, dtype=np.uint64).astype(np.int64)
    lo = ent & 0xffffffff
    e0 = lo - lo.min()
    res["entry_skew_us"] = {q: round(float(np.percentile(e0, q)) / 100.0, 2) for q in (0, 50, 90, 100)}
    res["prologue_us"] = {q: round(float(np.percentile(start - lo, q)) / 100.0, 2) for q in (0, 50, 90, 100)}
    if hasattr(L, "mm_debug_k2_exit"):   # after each wave's last stores completed (vmcnt 0)
        xb = (ctypes.c_ulonglong * nw)()
        L.mm_debug_k2_exit.argtypes = [ctypes.c_void_p, ctypes.c_int]
        assert L.mm_debug_k2_exit(xb, nw) == 0
        ex = np.frombuffer(xb, dtype=np.uint64).astype(np.int64) & 0xffffffff
        ok = (ex > 0) & (lo > 0)
        # one 100 MHz clock (s_memrealtime) for entry and exit: the span of the
        # waves' work, first entry to last completed store, against the launch's
        # HIP-event time (which adds the dispatch and the end-of-kernel release)
        res["wave_span_us"] = round(float(ex[ok].max() - lo[ok].min()) / 100.0, 2)
        res["exit_after_loop_us"] = {q: round(float(np.percentile(ex[ok] - (start[ok] + (dur[ok] / 10).astype(np.int64)), q)) / 100.0, 2)
                                    for q in (0, 50, 100)}
        res["kernel_event_us"] = {k: round(v[0] * 1e3 / max(v[1], 1), 2) for k, v in kprof.items() if v[1]}
print(json.dumps(res))
if len(sys.argv) > 2:
    np.save(sys.argv[2], raw)
