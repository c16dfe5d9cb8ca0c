# One rocprofv3 --pmc pass per counter group over a short bench, per K2 variant;
# prints per-kernel averages.  usage: bash scripts/gpu_pmcset.sh TAG "CNT1 CNT2 ..." [VARIANT_ENV...]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=$1; CNT=$2; shift 2
export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1"
for V in "${@:-MM_X=0}"; do
  export $V
  timeout -k 10 240 rocprofv3 --pmc $CNT -d $R/gpurun_out/${TAG}_$V -o run --output-format csv -- $B > /dev/null 2> gpurun_out/${TAG}_$V.err || { echo PMC $V FAIL; tail -5 gpurun_out/${TAG}_$V.err; exit 1; }
  unset ${V%%=*}
  python3 - "$TAG" "$V" <<'PY'
import csv, glob, sys, re
from collections import defaultdict
tag, v = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"mm::(k_[a-z_]+)", r["Kernel_Name"])
        if m: acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(v, k, {c: round(sum(x)/len(x)) for c, x in sorted(d.items())})
PY
done
