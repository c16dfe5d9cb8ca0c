# Kernel trace of the one-frame-per-call pattern: per-kernel GPU durations
# and the idle gaps between consecutive kernels (launch overhead).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; TAG=${1:-pf}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --call-pattern per-frame --frames-per-step 100 --steps 2 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_prof.err || { echo PROF FAIL; tail gpurun_out/${TAG}_prof.err; exit 1; }
python3 - gpurun_out/${TAG}_prof/run_kernel_trace.csv <<'PY'
import csv, sys, re, statistics as st
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    m = re.search(r"mm::(k_[a-z_]+)", n); return m.group(1) if m else n[:20]
rows = [r for r in rows if short(r["Kernel_Name"]).startswith("k_") and short(r["Kernel_Name"]) != "k_synth"]
rows = rows[-400:]   # the last 100 frames (4 kernels each)
dur = {}; gap = {}
for a, b in zip(rows, rows[1:]):
    gap.setdefault(short(b["Kernel_Name"]), []).append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in rows:
    dur.setdefault(short(r["Kernel_Name"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in dur:
    print(k, "dur_us median", round(st.median(dur[k]), 2), "gap_before_us median", round(st.median(gap.get(k, [0])), 2))
tot = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 / (len(rows) / 4)
print("us per frame (trace span)", round(tot, 2))
PY
