# Parity subset then same-call A/B of lib/variants (batch + drop-in), R rounds.
# usage: bash scripts/gpu_tab.sh TAG ROUNDS "pytest -k expr"
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-tab}; N=${2:-2}; K=${3:-}
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
bash scripts/gpu_abv.sh $N pf || exit 1
