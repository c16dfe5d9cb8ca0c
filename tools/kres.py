#!/usr/bin/env python3
"""Per-kernel VGPR / spill / LDS counts from a hipcc -S listing's metadata.

usage: kres.py LISTING.s [NAME_SUBSTRING...]
"""
import re
import sys

t = open(sys.argv[1]).read()
meta = t[t.find("amdhsa.kernels:"):]
entries = re.split(r"\n  - ", meta)
keys = sys.argv[2:]
for e in entries:
    m = re.search(r"\.name:\s+(\S+)", e)
    if not m:
        continue
    name = m.group(1)
    if keys and not any(k in name for k in keys):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", e) or [None, "?"])[1]
    print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>4} "
          f"sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} priv {g('private_segment_fixed_size')}")
