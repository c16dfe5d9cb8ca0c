set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/tab_tests.log 2>&1 || { echo TEST FAIL; tail -40 gpurun_out/tab_tests.log; exit 1; }
tail -1 gpurun_out/tab_tests.log
MM_K2_NOTAB=1 timeout -k 10 600 python -m pytest tests -q -m gpu -x -k "golden or stream or chunk" > gpurun_out/tab_tests2.log 2>&1 || { echo NOTAB TEST FAIL; tail -40 gpurun_out/tab_tests2.log; exit 1; }
tail -1 gpurun_out/tab_tests2.log
for round in 1 2; do
for v in a_scalar b_table b_table_notab; do
  lib=${v%_notab}; extra=""; [ "$v" = b_table_notab ] && extra="MM_K2_NOTAB=1"
  timeout -k 10 200 env $extra MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/$lib.so python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], {k:v['us_per_frame'] for k,v in d['kernels'].items()})" || { echo "$v FAIL"; exit 1; }
done; done
