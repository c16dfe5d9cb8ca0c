# Round evidence in one call: smoke, GPU parity suite, default bench (with the
# CPU baseline), then the profile set of the default configuration
# (scripts/gpu_profile.sh: kernel stats, PMC traffic, SQ counters, VALU).
# usage: bash scripts/gpu_round.sh TAG   (outputs under gpurun_out/, TAG-prefixed)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-round}
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; } > gpurun_out/${TAG}_host.txt 2>&1
bash scripts/gpu_base.sh $TAG || exit 1
bash scripts/gpu_profile.sh ${TAG}_p || exit 1
echo ALL OK
