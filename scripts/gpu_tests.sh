# GPU parity suite in one process (per-test timeout names a hung test).
# usage: bash scripts/gpu_tests.sh TAG [pytest args...]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-tests}; shift
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" > gpurun_out/${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}.log | tail -80
exit $rc
