# Build the library of a git revision as lib/variants/NAME.so (same-call A/B
# against the working tree: device-to-device spread is several percent).
# usage: build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
T=$(mktemp -d /tmp/rev.XXXXXX)
git -C /root/repo archive $REV phase-based-motion-manipulation_amd/csrc include | tar -x -C $T
mkdir -p /root/repo/phase-based-motion-manipulation_amd/lib/variants
for s in $T/phase-based-motion-manipulation_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -ffp-contract=on -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
    -Wno-unused-function -c -o ${s%.hip}.o $s &
done
wait
/opt/rocm/bin/hipcc -fPIC --offload-arch=gfx950 -shared \
  -o /root/repo/phase-based-motion-manipulation_amd/lib/variants/$NAME.so $T/phase-based-motion-manipulation_amd/csrc/*.o
rm -rf $T
ls -la /root/repo/phase-based-motion-manipulation_amd/lib/variants/$NAME.so
