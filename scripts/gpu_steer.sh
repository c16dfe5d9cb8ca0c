# steerable-extension parity tests + bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-st}
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "steer" > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for cfg in "--orientations 8" "--orientations 8 --temporal-filter iir" "--orientations 4"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline $cfg > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || { echo BENCH FAIL; tail -5 gpurun_out/${TAG}_b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_b.json "$cfg"
done
