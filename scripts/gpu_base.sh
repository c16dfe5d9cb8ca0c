# Baseline on a fresh box: smoke, GPU parity suite, default bench.
# usage: bash scripts/gpu_base.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-base}
export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo SMOKE FAIL; tail gpurun_out/${TAG}_smoke.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH FAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
