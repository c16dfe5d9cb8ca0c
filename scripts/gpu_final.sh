# Round-end evidence in one call, part 1: smoke, the GPU suite, the default
# bench (with CPU baseline and parity at the timed launch shape), then the
# profile set of the default configuration (kernel stats, PMC traffic, SQ and
# VALU counters).  usage: bash scripts/gpu_final.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-final}
export TMPDIR=/tmp
bash scripts/gpu_base.sh $TAG || exit 1
bash scripts/gpu_profile.sh ${TAG}_c2 || exit 1
echo FINAL1 OK
