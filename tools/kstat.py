#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy summary and static VALU count of a
hipcc -S listing (the comment block the AMDGPU backend prints after each
function).

usage: kstat.py LISTING.s [NAME_SUBSTRING ...]
"""
import re
import sys

text = open(sys.argv[1]).read().split("\n")
keys = sys.argv[2:]
cur, start = None, 0
for i, l in enumerate(text):
    m = re.match(r"^(_Z\S+):\s", l)
    if m:
        cur, start, valu, ds, mov = m.group(1), i, 0, 0, 0
        continue
    if cur is None:
        continue
    s = l.strip()
    if s.startswith("v_"):
        valu += 1
        mov += s.startswith("v_mov")
    elif s.startswith("ds_"):
        ds += 1
    m = re.match(r"^\s*; NumVgprs: (\d+)", l)
    if m:
        nv = int(m.group(1))
    m = re.match(r"^\s*; ScratchSize: (\d+)", l)
    if m:
        sc = int(m.group(1))
    m = re.match(r"^\s*; Occupancy: (\d+)", l)
    if m:
        if not keys or any(k in cur for k in keys):
            print(f"{cur[:90]:90s} vgpr {nv:3d} scratch {sc:4d} occ {m.group(1)} valu(static) {valu} mov {mov} ds {ds}")
        cur = None
