# Round-start baseline: default bench line (no CPU baseline) and a rocprof
# kernel summary of the reference's one-frame-per-call pattern.
# usage: bash scripts/gpu_base.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-base}
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH FAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_pf -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --call-pattern per-frame --frames-per-step 120 --steps 2 --warmup 1 > gpurun_out/${TAG}_pf_bench.json 2> gpurun_out/${TAG}_pf.err || { echo PROF FAIL; tail gpurun_out/${TAG}_pf.err; exit 1; }
cat gpurun_out/${TAG}_pf_bench.json
cut -d, -f1-8 gpurun_out/${TAG}_pf/run_kernel_stats.csv
echo ALL OK
