# I-cache probe + K2 one-frame/batch phase stamps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 60 tools/bin/icache_probe > gpurun_out/icache.json 2>&1 || { echo PROBE FAIL; cat gpurun_out/icache.json; exit 1; }
cat gpurun_out/icache.json
bash scripts/gpu_k2pf.sh || exit 1
