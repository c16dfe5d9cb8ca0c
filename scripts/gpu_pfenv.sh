# Per-frame drop-in (tools/perframe.py) under environment variants, R rounds.
# usage: bash scripts/gpu_pfenv.sh ROUNDS "ENV1" "ENV2" ...   ("X=0" = defaults)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=${1:-2}; shift
for i in $(seq $N); do
  for E in "$@"; do
    env $E timeout -k 10 120 python3 tools/perframe.py 400 > gpurun_out/pfenv.json 2> gpurun_out/pfenv.err || { echo PF FAIL "$E"; tail gpurun_out/pfenv.err; exit 1; }
    echo "[$E]" $(cat gpurun_out/pfenv.json)
  done
done
echo ALL OK
