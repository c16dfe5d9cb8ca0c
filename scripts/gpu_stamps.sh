# K2 phase stamps (diagnostic build, -DMM_K2_STAMPS) for a batch of FRAMES
# frames per launch: tools/k2_phases.py against each library in LIBDIR.
# usage: bash scripts/gpu_stamps.sh LIBDIR FRAMES [more FRAMES...]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; D=$1; shift
for V in $D/*.so; do
  n=$(basename $V .so)
  for F in "$@"; do
    MM355_LIB=$R/$V timeout -k 10 120 python3 tools/k2_phases.py $F gpurun_out/k2ph_${n}_$F.npy > gpurun_out/k2ph_${n}_$F.json 2> gpurun_out/k2ph_${n}_$F.err || { echo $n FAIL; tail gpurun_out/k2ph_${n}_$F.err; exit 1; }
    echo $n frames=$F; cat gpurun_out/k2ph_${n}_$F.json
  done
done
