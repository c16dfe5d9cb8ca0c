# Same-call A/B of the one-frame-per-call path over lib/variants/*.so:
# perframe.py rate (no events per call), R rounds, then a rocprofv3 kernel
# trace per variant (durations and gaps, tools/pf_trace.py).
# usage: bash scripts/gpu_pfab.sh ROUNDS [trace]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; N=${1:-2}
for i in $(seq $N); do
  for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
    n=$(basename $V .so)
    MM355_LIB=$R/$V timeout -k 10 120 python3 tools/perframe.py 400 > gpurun_out/pfab_$n.json 2> gpurun_out/pfab_$n.err || { echo FAIL $n; tail gpurun_out/pfab_$n.err; exit 1; }
    echo "$n $(cat gpurun_out/pfab_$n.json)"
  done
done
if [ -n "$2" ]; then
  for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
    n=$(basename $V .so)
    MM355_LIB=$R/$V timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pftr_$n -o run --output-format csv -- python3 $R/tools/perframe.py 300 > /dev/null 2> gpurun_out/pftr_$n.err || { echo TRACE FAIL $n; tail gpurun_out/pftr_$n.err; exit 1; }
    echo "== $n"; python3 tools/pf_trace.py gpurun_out/pftr_$n/run_kernel_trace.csv
  done
fi
echo ALL OK
