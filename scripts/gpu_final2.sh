# Round-end evidence, part 2: profile sets of C3 (2160p L = 6) and the
# steerable O = 8 DIFF path, and the bench lines of every configuration.
# usage: bash scripts/gpu_final2.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-final}
export TMPDIR=/tmp
bash scripts/gpu_profile.sh ${TAG}_c3 --width 3840 --height 2160 --levels 6 || exit 1
bash scripts/gpu_profile.sh ${TAG}_o8 --orientations 8 || exit 1
bash scripts/gpu_configs.sh ${TAG}_cfg || exit 1
echo FINAL2 OK
