set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo SMOKE FAIL; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo BENCH FAIL; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > gpurun_out/bench1_prof.json 2> gpurun_out/prof1.err || { echo PROF FAIL; exit 1; }
timeout -k 10 120 phase-based-motion-manipulation_amd/bin/mm_cli > gpurun_out/cli1.txt 2>&1 || { echo CLI FAIL; exit 1; }
echo ALL OK
