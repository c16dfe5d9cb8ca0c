# Same-call A/B of the working tree against lib/variants/*.so on the default
# configuration, C3 (2160p, L=6) and the steerable O=8 extension.
# usage: bash scripts/gpu_ab_configs.sh [ROUNDS]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=${1:-2}
bash scripts/gpu_libab.sh $N || exit 1
bash scripts/gpu_libab.sh $N --width 3840 --height 2160 --levels 6 || exit 1
bash scripts/gpu_libab.sh 1 --orientations 8 --steps 2 || exit 1
echo AB OK
