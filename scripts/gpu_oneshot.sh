# One-frame drop-in rate with the one-shot K34 (MM_K34_ONESHOT=1) against the
# unfused K3 -> K4 pair (=0), at several frame sizes, R rounds.
# usage: bash scripts/gpu_oneshot.sh ROUNDS "WxH ..."
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=${1:-2}; SIZES=${2:-"1920x1080 1280x720"}
for i in $(seq $N); do
  for S in $SIZES; do
    for O in 2 0; do
      MM_K34_ONESHOT=$O timeout -k 10 120 python3 tools/perframe.py 400 ${S%x*} ${S#*x} > gpurun_out/os.json 2> gpurun_out/os.err || { echo PF FAIL $S $O; tail gpurun_out/os.err; exit 1; }
      echo "$S oneshot=$O $(cat gpurun_out/os.json)"
    done
  done
done
echo ALL OK
