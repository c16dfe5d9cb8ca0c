# parity tests + bench (no CPU baseline) + rocprof stats; tag in $1
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/test_$TAG.log 2>&1 || { echo TEST FAIL; tail -30 gpurun_out/test_$TAG.log; exit 1; }
tail -2 gpurun_out/test_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAIL; tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 > /dev/null 2> gpurun_out/prof_$TAG.err || { echo PROF FAIL; exit 1; }
cut -d, -f1-4 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-60,200-
