# Build library variants: build_variants.sh name1 "FLAGS1" name2 "FLAGS2" ...
set -e
cd /root/repo/phase-based-motion-manipulation_amd
rm -rf lib/variants; mkdir -p lib/variants
while [ $# -gt 0 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $f -shared -o lib/variants/$n.so csrc/mm_api.hip &
done
wait
ls -la lib/variants
