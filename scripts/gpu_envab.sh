# A/B of an env knob: parity file once, then the bench per value (per-kernel us/frame).
# usage: bash scripts/gpu_envab.sh VAR "v1 v2 ..."
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; VAR=$1; VALS=$2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/envab_tests.log 2>&1 || { echo TEST FAIL; tail -30 gpurun_out/envab_tests.log; exit 1; }
tail -1 gpurun_out/envab_tests.log
for v in $VALS; do
  env $VAR=$v timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/envab_$v.json 2> gpurun_out/envab_$v.err || { echo BENCH FAIL $v; tail gpurun_out/envab_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/envab_$v.json "$VAR=$v"
done
