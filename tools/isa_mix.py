#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing.

usage: isa_mix.py LISTING.s SYMBOL_SUBSTRING
Counts vector ALU, packed, transcendental, LDS, global and scalar instructions
between the kernel's label and s_endpgm (static: loop bodies count once).
"""
import re
import sys

text = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
start = next(i for i, l in enumerate(text) if re.match(r"^\S*" + re.escape(key) + r"\S*:\s*(;.*)?$", l))
counts = {}
for l in text[start + 1:]:
    s = l.strip()
    if s.startswith("s_endpgm"):
        break
    if not s or s.startswith((";", ".")) or s.endswith(":"):
        continue
    op = s.split()[0]
    if op.startswith("v_pk_"):
        k = "valu_pk"
    elif re.match(r"v_(sin|cos|rcp|rsq|sqrt|exp|log)_", op):
        k = "valu_trans"
    elif op.startswith(("v_mov", "v_accvgpr")):
        k = "valu_mov"
    elif op.startswith("v_"):
        k = "valu"
    elif op.startswith("ds_"):
        k = "lds"
    elif op.startswith(("global_", "buffer_", "scratch_")):
        k = "vmem"
    elif op.startswith("s_waitcnt"):
        k = "waitcnt"
    elif op.startswith("s_"):
        k = "salu"
    else:
        k = "other"
    counts[k] = counts.get(k, 0) + 1
tot_v = sum(v for k, v in counts.items() if k.startswith("valu"))
issue = counts.get("valu", 0) + counts.get("valu_pk", 0) + counts.get("valu_mov", 0) + 2 * counts.get("valu_trans", 0)
print(key, counts, "valu_total", tot_v, "valu_issue_slots", issue)
