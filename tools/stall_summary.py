#!/usr/bin/env python3
"""Per-kernel average of SQ counters from rocprofv3 --pmc csv dirs, plus the
derived stall split (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~
SQ_WAVE_CYCLES, MI355X_MICROARCH.md counter table).
usage: stall_summary.py DIR [DIR ...]"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"mm::(k_[a-z_0-9]+)", r["Kernel_Name"])
            if m:
                acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in acc.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in avg:
                avg["frac_" + c] = round(avg[c] / wc, 4)
    if avg.get("SQ_LDS_IDX_ACTIVE"):
        avg["lds_conflict_frac"] = round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / avg["SQ_LDS_IDX_ACTIVE"], 4)
    out[k] = {c: (round(v, 4) if isinstance(v, float) else v) for c, v in sorted(avg.items())}
print(json.dumps(out, indent=1))
