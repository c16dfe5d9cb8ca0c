#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs into profiles/traffic.json.

FETCH_SIZE and WRITE_SIZE are in KiB (x1024 for bytes).  On gfx950 FETCH_SIZE
under-reads wide streaming loads (MI355X_MICROARCH.md §HBM); each counter is
corrected by the factor measured on tools/pmc_calib (512 MiB streamed at the
access width that dominates the kernel's traffic).

usage: pmc_summary.py FETCH_DIR WRITE_DIR CAL_FETCH_DIR CAL_WRITE_DIR FRAMES_PER_LAUNCH OUT [CONFIG]
(CONFIG: bench.profile_key of the measured configuration, stored as "config")
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

# dominant (read width, write width) in bytes per lane, per kernel
WIDTHS = {"k_rows_fwd": (4, 16), "k_cols": (8, 8), "k_rows_inv": (16, 4), "k_compose": (4, 4),
          "k_rows_inv_compose": (16, 16),
          # steerable extension (mm_steer.hpp): k_cols_fwd once per batch, the
          # band kernels once per frame
          "k_cols_fwd": (8, 8), "k_sb_cols": (8, 16), "k_sb_rows": (8, 4)}
PER_FRAME = {"k_sb_cols", "k_sb_rows"}
CAL_BYTES = 512 << 20


def short(name):
    m = re.search(r"mm::(k_[a-z_]+)", name)
    if m:
        return m.group(1)
    m = re.search(r"\b(rd|wr)<(float|HIP_vector_type<float, (\d)u>)", name)
    if not m:
        return None
    return f"{m.group(1)}_{4 * int(m.group(3) or 1)}"


def frames_of_launch(name):
    """Frames one launch of a per-frame kernel covers: k_sb_rows<L, IIR, NF>
    runs NF frames (round 5: pairs), the band-column kernel one."""
    m = re.search(r"k_sb_rows<\d+, (?:true|false), (\d+)>", name)
    return int(m.group(1)) if m else 1


def read_counter(d, counter):
    """Mean counter value per launch; for the per-frame kernels (PER_FRAME)
    the mean per FRAME (each launch divided by the frames it covers)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            k = short(name)
            if k:
                div = frames_of_launch(name) if k in PER_FRAME else 1
                vals[k].append(float(row["Counter_Value"]) / div)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fdir, wdir, cfdir, cwdir, fpl, out = sys.argv[1:7]
    config = sys.argv[7] if len(sys.argv) > 7 else None
    fpl = int(fpl)
    fetch, write = read_counter(fdir, "FETCH_SIZE"), read_counter(wdir, "WRITE_SIZE")
    cfetch, cwrite = read_counter(cfdir, "FETCH_SIZE"), read_counter(cwdir, "WRITE_SIZE")
    fcorr = {w: CAL_BYTES / (cfetch[f"rd_{w}"] * 1024) for w in (4, 8, 16) if cfetch.get(f"rd_{w}")}
    wcorr = {w: CAL_BYTES / (cwrite[f"wr_{w}"] * 1024) for w in (4, 8, 16) if cwrite.get(f"wr_{w}")}
    kernels = {}
    for k, (rw, ww) in WIDTHS.items():
        if k not in fetch or k not in write:
            continue
        fb, wb = fetch[k] * 1024, write[k] * 1024
        fc, wc = fb * fcorr.get(rw, 1.0), wb * wcorr.get(ww, 1.0)
        kernels[k] = {"fetch_bytes_raw": fb, "write_bytes_raw": wb,
                      "fetch_bytes": fc, "write_bytes": wc,
                      "hbm_bytes_per_launch": fc + wc,   # per frame for PER_FRAME kernels
                      "hbm_bytes_per_frame": (fc + wc) / (1 if k in PER_FRAME else fpl),
                      "read_width": rw, "write_width": ww}
    if "k_sb_cols" in kernels and "k_cols_fwd" in kernels:
        # bench.py's kernel ids (mm_profile_end) of the steerable path: k_cols =
        # k_cols_fwd + k_sb_cols, k_rows_inv = k_sb_rows
        kernels["k_cols"] = {"hbm_bytes_per_frame": kernels["k_cols_fwd"]["hbm_bytes_per_frame"] +
                             kernels["k_sb_cols"]["hbm_bytes_per_frame"], "of": ["k_cols_fwd", "k_sb_cols"]}
    if "k_sb_rows" in kernels:
        kernels["k_rows_inv"] = {"hbm_bytes_per_frame": kernels["k_sb_rows"]["hbm_bytes_per_frame"],
                                 "of": ["k_sb_rows"]}
    res = {"frames_per_launch": fpl, "calibration": {"fetch_factor": fcorr, "write_factor": wcorr},
           "kernels": kernels,
           "frame_hbm_bytes": sum(v["hbm_bytes_per_frame"] for k, v in kernels.items() if "of" not in v)}
    if config:
        res["config"] = config
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
