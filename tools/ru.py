#!/usr/bin/env python3
"""Per-kernel register/LDS/occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/ru.py [FILTER]
"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        name = re.sub(r"\(.*", "", name).replace("mm::", "")
        cur = {"name": name}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"),
                     ("spill", r"VGPRs Spill: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name']:<40} vgpr {r.get('vgpr', '?'):>4} agpr {r.get('agpr', '?'):>3} "
              f"spill {r.get('spill', '?'):>4} scratch {r.get('scratch', '?'):>4} "
              f"occ {r.get('occ', '?')} lds {r.get('lds', '?')}")
