#!/usr/bin/env python3
"""s_nop wait states per loop of one kernel in a hipcc -S listing (gfx950
inserts s_nop 0 between a packed-FP32 result and a dependent packed op
issued too close behind it: each costs the wave an issue slot).

usage: nopstat.py LISTING.s KERNEL_SUBSTRING
"""
import re
import sys

L = open(sys.argv[1]).read().split("\n")
i0 = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + re.escape(sys.argv[2]) + r"\S*:", l))
i1 = next(i for i in range(i0, len(L)) if L[i].strip().startswith("s_endpgm"))
body = L[i0:i1]
heads = [l.split(":")[0] for l in body if "Loop Header" in l]
tot = sum(1 for l in body if l.strip().startswith("s_nop"))
print("kernel total s_nop", tot)
for lab in heads:
    name = lab.lstrip(".L")
    inside, n, v = False, 0, 0
    for l in body:
        if re.match(r"^\.?\S+:", l) or l.startswith("; %bb"):
            inside = (l.split(":")[0] == lab) or ("Header=" + name + " ") in l
            continue
        if inside:
            s = l.strip()
            if s.startswith("s_nop"):
                m = re.match(r"s_nop\s+(\d+)", s)
                n += 1 + int(m.group(1)) if m else 1
            elif s.startswith("v_"):
                v += 1
    print(f"{lab:12s} VALU {v:5d}  nop wait states {n}")
