# A/B of lib/variants (non-stamp builds) + phase stamps of st_* builds
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p /tmp/stv && mv phase-based-motion-manipulation_amd/lib/variants/st_*.so /tmp/stv/ 2>/dev/null
bash scripts/gpu_variants.sh ${1:-abs} ${2:-2} --drop-in-frames 0 || exit 1
for V in /tmp/stv/*.so; do
  n=$(basename $V .so)
  MM355_LIB=$V timeout -k 10 120 python3 tools/k2_phases.py 100 gpurun_out/k2ph_$n.npy > gpurun_out/k2ph_$n.json 2> gpurun_out/k2ph_$n.err || { echo $n FAIL; tail gpurun_out/k2ph_$n.err; exit 1; }
  echo $n; cat gpurun_out/k2ph_$n.json
done
