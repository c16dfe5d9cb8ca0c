# counter list + VALU activity counters for two library variants
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1"
for v in a_scalar b_packed_occ4; do
  for CNT in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_BUSY_CYCLES" "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_INSTS_LDS" ; do
    tag=$(echo $CNT | cut -d' ' -f2)
    MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/$v.so timeout -k 10 240 rocprofv3 --pmc $CNT -d $R/gpurun_out/valu_${v}_$tag -o run --output-format csv -- $B > /dev/null 2> gpurun_out/valu_${v}_$tag.err || { echo PMC $v $tag FAIL; tail -3 gpurun_out/valu_${v}_$tag.err; }
  done
done
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
for v in ("a_scalar", "b_packed_occ4"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/valu_{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"mm::(k_[a-z_]+)", r["Kernel_Name"])
            if m: acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in ("k_cols", "k_rows_fwd", "k_rows_inv", "k_compose"):
        print(v, k, {c: round(sum(x)/len(x)) for c, x in sorted(acc[k].items())})
PY
