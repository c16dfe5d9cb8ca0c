# usage: bash scripts/gpu_probe1.sh TAG  -- gate probe, ring-local tests, bench + C3 profile
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-probe}
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/gate_probe.py > gpurun_out/${TAG}_gate.txt 2>&1; cat gpurun_out/${TAG}_gate.txt
timeout -k 10 600 python -u -m pytest tests/test_ring_c.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_ring.log 2>&1 || { echo RING FAIL; tail -30 gpurun_out/${TAG}_ring.log; }
tail -3 gpurun_out/${TAG}_ring.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH FAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
bash scripts/gpu_profile.sh ${TAG}_c3 --width 3840 --height 2160 --levels 6
