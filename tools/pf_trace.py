#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive kernels of a
rocprofv3 kernel trace (run_kernel_trace.csv): for the one-frame-per-call
pattern, where fixed per-launch costs are the frame time.

usage: pf_trace.py run_kernel_trace.csv [skip_first=20]
"""
import collections
import csv
import json
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = [r for r in rows if "k_synth" not in r["Kernel_Name"] and "copyBuffer" not in r["Kernel_Name"]][skip:]


def short(n):
    n = n.split("(")[0].replace("void ", "")
    return n.split("::")[-1]


dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i, r in enumerate(rows):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[short(r["Kernel_Name"])].append((e - s) / 1e3)
    if i:
        pe = int(rows[i - 1]["End_Timestamp"])
        gap[short(rows[i - 1]["Kernel_Name"]) + " -> " + short(r["Kernel_Name"])].append((s - pe) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
res = {"kernels": len(rows), "span_us": round(span, 1),
       "duration_us_p50": {k: round(statistics.median(v), 2) for k, v in dur.items()},
       "gap_us_p50": {k: round(statistics.median(v), 2) for k, v in gap.items() if len(v) > 5}}
print(json.dumps(res, indent=1))
