#!/usr/bin/env python3
"""Static instruction mix of each loop (header label .. last branch back to it)
of one kernel in a hipcc -S listing.

usage: loopstat.py LISTING.s KERNEL_SUBSTRING
"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
i0 = next(i for i, l in enumerate(L) if re.match(r"^_Z\S*" + re.escape(sys.argv[2]) + r"\S*:", l))
i1 = next(i for i in range(i0, len(L)) if L[i].strip().startswith("s_endpgm"))
body = L[i0:i1]
# blocks are annotated "; in Loop: Header=BBx_y Depth=d" (the header itself
# "=>This Inner Loop Header"); a loop is every block carrying its header's name
heads = [l.split(":")[0] for l in body if "Loop Header" in l]
for lab in heads:
    name = lab.lstrip(".L")
    c = collections.Counter()
    inside = False
    for l in body:
        if re.match(r"^\.?\S+:", l) or l.startswith("; %bb"):
            inside = (l.split(":")[0] == lab) or ("Header=" + name + " ") in l
            continue
        if not inside:
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        if op.startswith("v_pk"):
            k = "pk"
        elif re.match(r"v_(sin|cos|rcp|rsq|sqrt|exp|log)_", op):
            k = "trans"
        elif op.startswith(("v_mov", "v_accvgpr")):
            k = "mov"
        elif op.startswith("v_cndmask"):
            k = "cnd"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("ds_"):
            k = "ds"
        elif op.startswith(("buffer", "global", "scratch")):
            k = "vmem"
        elif op.startswith("s_cbranch") or op.startswith("s_branch"):
            k = "br"
        elif op.startswith("s_barrier"):
            k = "bar"
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = "other"
        c[k] += 1
    v = sum(c[k] for k in ("pk", "trans", "mov", "cnd", "valu"))
    print(f"{lab:12s} VALU {v:5d}", dict(sorted(c.items())))
