# A/B: bench each library variant in lib/variants (interleaved rounds)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for round in 1 2; do
for v in phase-based-motion-manipulation_amd/lib/variants/*.so; do
  timeout -k 10 200 env MM355_LIB=$R/$v python bench.py --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$(basename $v)', d['value'], {k:v['us_per_frame'] for k,v in d['kernels'].items()})" || { echo "$v FAIL"; exit 1; }
done; done
