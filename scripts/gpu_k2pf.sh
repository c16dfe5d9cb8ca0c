# K2 phase stamps of a one-frame call and of a 100-frame batch (lib/stamps/k2st.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for n in 1 100; do
  MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/stamps/k2st.so timeout -k 10 120 python3 tools/k2_phases.py $n > gpurun_out/k2pf_$n.json 2> gpurun_out/k2pf_$n.err || { echo FAIL $n; tail gpurun_out/k2pf_$n.err; exit 1; }
  echo n=$n; cat gpurun_out/k2pf_$n.json
done
echo ALL OK
