# k_cols phase breakdown of each stamp build in lib/variants (tools/k2_phases.py)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
  n=$(basename $V .so)
  MM355_LIB=$R/$V timeout -k 10 120 python3 tools/k2_phases.py 100 gpurun_out/k2ph_$n.npy > gpurun_out/k2ph_$n.json 2> gpurun_out/k2ph_$n.err || { echo $n FAIL; tail gpurun_out/k2ph_$n.err; exit 1; }
  echo $n; cat gpurun_out/k2ph_$n.json
done
