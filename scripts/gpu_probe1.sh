# usage: bash scripts/gpu_probe1.sh TAG  -- gate probe + ring-local tests
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-probe}
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/gate_probe.py > gpurun_out/${TAG}_gate.txt 2>&1; cat gpurun_out/${TAG}_gate.txt
timeout -k 10 600 python -u -m pytest tests/test_ring_c.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_ring.log 2>&1 || { echo RING FAIL; tail -30 gpurun_out/${TAG}_ring.log; exit 1; }
tail -3 gpurun_out/${TAG}_ring.log
