# Quick A/B check of a kernel change: the GPU parity file, then the default
# bench twice (no CPU baseline, no drop-in pass), per-kernel us/frame.
# usage: bash scripts/gpu_try.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-try}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err || { echo BENCH FAIL; tail gpurun_out/${TAG}_b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], {k: v['us_per_frame'] for k, v in d['kernels'].items()}, d.get('parity_vs_oracle'))" gpurun_out/${TAG}_b$i.json
done
