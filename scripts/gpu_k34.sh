# K34 experiment: parity subset, same-call A/B of lib/variants, K34 phase stamps
# of lib/stamps/*.so.  usage: bash scripts/gpu_k34.sh TAG ROUNDS "pytest -k expr"
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-k34}; N=${2:-2}; K=${3:-}
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for V in phase-based-motion-manipulation_amd/lib/stamps/*.so; do
  [ -e "$V" ] || continue
  n=$(basename $V .so)
  MM355_LIB=$R/$V timeout -k 10 120 python3 tools/k34_phases.py 100 > gpurun_out/${TAG}_ph_$n.json 2> gpurun_out/${TAG}_ph_$n.err || { echo $n STAMPS FAIL; tail gpurun_out/${TAG}_ph_$n.err; exit 1; }
  echo $n; cat gpurun_out/${TAG}_ph_$n.json
done
bash scripts/gpu_abv.sh $N || exit 1
