# SQ counter passes (kernel-trace only) on the bench; summary printed per kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-sq}
export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $R/gpurun_out/${TAG}_$i -o run --output-format csv -- $B > /dev/null 2> gpurun_out/${TAG}_$i.err || { echo PASS $i FAIL; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
done
python3 - "$TAG" <<'PY'
import csv, glob, sys, re
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"mm::(k_[a-z_]+)", r["Kernel_Name"])
        if m: acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v)/len(v)) for c, v in sorted(d.items())})
PY
