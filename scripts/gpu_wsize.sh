# K2 write traffic of library variants: rocprofv3 WRITE_SIZE (one counter pass
# each, kernel-trace-free) on a short default bench, per-launch means printed.
# usage: bash scripts/gpu_wsize.sh NAME... (lib/variants/NAME.so, "cur" = tree)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = cur ]; then unset MM355_LIB; else export MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/$n.so; fi
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/ws_$n -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 2 --warmup 1 > /dev/null 2> gpurun_out/ws_$n.err || { echo WS $n FAIL; tail -3 gpurun_out/ws_$n.err; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, sys, collections
n = sys.argv[1]
v = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/ws_{n}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        if r["Counter_Name"].startswith("WRITE_SIZE"):
            v[(k, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
for (k, g), xs in sorted(v.items()):
    if k.startswith(("k_cols", "k_rows")):
        print(n, k, g, len(xs), "mean WRITE_SIZE", round(sum(xs) / len(xs)))
PY
done
