# Effective shader clock per kernel and library variant: GRBM_GUI_ACTIVE / 8 /
# kernel time (MI355X_MICROARCH.md DVFS note), kernel-trace only.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; TAG=${1:-clk}
for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
  n=$(basename $V .so)
  MM355_LIB=$R/$V timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/${TAG}_$n -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 1 --warmup 1 > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { echo $n FAIL; tail -5 gpurun_out/${TAG}_$n.err; exit 1; }
  python3 - gpurun_out/${TAG}_$n $n <<'PY'
import csv, glob, sys, re
from collections import defaultdict
d = sys.argv[1]
c = defaultdict(lambda: defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"mm::(k_[a-z_0-9]+)", r["Kernel_Name"])
        if m:
            c[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    hdr = list(csv.DictReader(open(f)))[0].keys()
for k, v in c.items():
    print(sys.argv[2], k, {n: max(x) for n, x in v.items()})
PY
done
