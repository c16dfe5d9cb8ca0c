# Experiment builds for same-call A/B (one padded size only: MM_ONLY_LOG2N, fast):
#   build_ab.sh NAME REV|wt "EXTRA FLAGS"   (REV: a git revision; wt: working tree)
set -e
NAME=$1; REV=$2; FL=$3; L2=${L2:-11}
SRC=/root/repo
if [ "$REV" != wt ]; then
  SRC=$(mktemp -d /tmp/rev.XXXXXX)
  git -C /root/repo archive $REV phase-based-motion-manipulation_amd/csrc include | tar -x -C $SRC
fi
mkdir -p /root/repo/phase-based-motion-manipulation_amd/lib/variants
/opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
  -DMM_ONLY_LOG2N=$L2 $FL -shared -o /root/repo/phase-based-motion-manipulation_amd/lib/variants/$NAME.so \
  $SRC/phase-based-motion-manipulation_amd/csrc/mm_api.hip 2>&1 | grep -E 'error' || true
ls -la /root/repo/phase-based-motion-manipulation_amd/lib/variants/$NAME.so
