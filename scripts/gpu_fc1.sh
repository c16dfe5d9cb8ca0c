set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fcache.py tests/test_handle.py tests/test_k34.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fc1_tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/fc1_tests.log; exit 1; }
tail -2 gpurun_out/fc1_tests.log
bash scripts/gpu_pfab.sh 2 || exit 1
MM_K2_NOFC=1 MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/b_cur.so timeout -k 10 120 python3 tools/perframe.py 400 && MM_K2_NOFC=1 MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/b_cur.so timeout -k 10 120 python3 tools/perframe.py 400 || exit 1
bash scripts/gpu_abv.sh 1 || exit 1
