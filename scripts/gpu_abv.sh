# parity suite on the default build, then interleaved A/B of lib/variants/*.so
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; TAG=${1:-abv}
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for round in 1 2; do
for v in phase-based-motion-manipulation_amd/lib/variants/*.so; do
  timeout -k 10 200 env MM355_LIB=$R/$v python bench.py --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$(basename $v)', d['value'], {k:v['us_per_frame'] for k,v in d['kernels'].items()})" || { echo "$v FAIL"; exit 1; }
done; done
