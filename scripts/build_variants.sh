# Build library variants: build_variants.sh name1 "FLAGS1" name2 "FLAGS2" ...
# (every translation unit of csrc/ with the flags; -DMM_ONLY_LOG2N=L builds
# mm_api.hip alone for one padded size)
set -e
cd /root/repo/phase-based-motion-manipulation_amd
mkdir -p lib/variants
while [ $# -gt 0 ]; do
  n=$1; f=$2; shift 2
  (
    o=/tmp/variant_$n; rm -rf $o; mkdir -p $o
    if echo "$f" | grep -q MM_ONLY_LOG2N; then srcs=csrc/mm_api.hip; else srcs=$(ls csrc/*.hip); fi
    for s in $srcs; do
      /opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -ffp-contract=on -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-function $f -c -o $o/$(basename $s .hip).o $s &
    done
    wait
    /opt/rocm/bin/hipcc -fPIC --offload-arch=gfx950 -shared -o lib/variants/$n.so $o/*.o
    # the variant's own ring library (mm355/ring.py refuses a ring bound to
    # another libmm355 than the one MM355_LIB loaded)
    gcc -O2 -std=gnu11 -fPIC -shared -I../include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
      -o lib/variants/${n}_ring.so host/mm_ring.c -Llib/variants -l:$n.so -L/opt/rocm/lib -lrccl \
      -lamdhip64 -lpthread -ldl -lm -Wl,-rpath,'$ORIGIN' -Wl,-rpath,/opt/rocm/lib
  ) &
done
wait
ls -la lib/variants
