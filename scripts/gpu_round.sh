# Round evidence in one call: smoke, GPU parity suite, default bench (with the
# CPU baseline), rocprofv3 kernel stats of the same bench, PMC traffic passes.
# usage: bash scripts/gpu_round.sh TAG   (outputs under gpurun_out/, TAG-prefixed)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-round}
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; } > gpurun_out/${TAG}_host.txt 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo SMOKE FAIL; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH FAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { echo PROF FAIL; exit 1; }
bash scripts/gpu_pmc.sh ${TAG}_pmc || { echo PMC FAIL; exit 1; }
bash scripts/gpu_stall.sh ${TAG}_st > /dev/null || { echo STALL FAIL; exit 1; }
python3 tools/valu_summary.py gpurun_out/${TAG}_st_1,gpurun_out/${TAG}_st_2 gpurun_out/${TAG}_prof gpurun_out/${TAG}_valu.json
echo ALL OK
