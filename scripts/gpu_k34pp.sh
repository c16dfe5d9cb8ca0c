set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_k34.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k34pp_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/k34pp_tests.log; exit 1; }
tail -1 gpurun_out/k34pp_tests.log
bash scripts/gpu_abv.sh 2 || exit 1
