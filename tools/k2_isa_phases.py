#!/usr/bin/env python3
"""Static instruction mix of k_cols's frame-loop phases in a hipcc -S listing
built with -DMM_ASM_MARKS (marks M1..M4 around the two FFTs).

usage: k2_isa_phases.py LISTING.s [MODE=2] [LOG2N=11]
"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
mode = sys.argv[2] if len(sys.argv) > 2 else "2"
log2n = sys.argv[3] if len(sys.argv) > 3 else "11"
i0 = next(i for i, l in enumerate(L) if re.match(r"^_ZN2mm6k_colsILi%sELi%s(?:ELb[01])?(?:ELi0)?EEEv\S*:" % (log2n, mode), l))
end = next(i for i in range(i0, len(L)) if L[i].strip().startswith("s_endpgm"))
body = L[i0:end]
marks = [(i, l.strip()) for i, l in enumerate(body) if l.strip().startswith("; M")]


def mix(a, b):
    c = collections.Counter()
    for l in body[a:b]:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith("v_pk"):
            k = "pk"
        elif re.match(r"v_(sin|cos|rcp|rsq|sqrt|exp|log)_", op):
            k = "trans"
        elif op.startswith(("v_mov", "v_accvgpr")):
            k = "mov"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("ds_"):
            k = "ds"
        elif op.startswith(("buffer", "global")):
            k = "vmem"
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = "other"
        c[k] += 1
    return dict(sorted(c.items()))


# the marks appear once per frame-loop instantiation (block 0 and the others)
prev = 0
for i, m in marks:
    print(f"{prev:6d}..{i:6d} -> {m:14s}", mix(prev, i))
    prev = i
print(f"{prev:6d}..end   ", mix(prev, len(body)))
