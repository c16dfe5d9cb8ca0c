# Tests + default bench + C3 bench in one call.
# usage: bash scripts/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-chk}; K=${2:-}
export TMPDIR=/tmp
if [ -n "$K" ]; then KA="-k $K"; else KA=""; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread $KA > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || { grep -B 30 -m1 "^E " gpurun_out/${TAG}_tests.log | tail -40; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH FAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()}, d['drop_in_per_frame']['frames_per_s'])" gpurun_out/${TAG}_bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --drop-in-frames 0 --width 3840 --height 2160 --levels 6 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo C3 FAIL; tail gpurun_out/${TAG}_c3.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3', d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_c3.json
timeout -k 10 300 python bench.py --no-cpu-baseline --drop-in-frames 0 --orientations 8 > gpurun_out/${TAG}_o8.json 2> gpurun_out/${TAG}_o8.err || { echo O8 FAIL; tail gpurun_out/${TAG}_o8.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('o8', d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_o8.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_o8prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --orientations 8 --steps 1 --warmup 1 > /dev/null 2> gpurun_out/${TAG}_o8prof.err || { echo O8 PROF FAIL; exit 1; }
echo CHECK OK
