set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
V=$R/phase-based-motion-manipulation_amd/lib/variants/c_fcnt.so
for i in 1 2; do
MM355_LIB=$V timeout -k 10 120 python3 tools/perframe.py 400 || exit 1
MM_K2_NOFC=1 MM355_LIB=$V timeout -k 10 120 python3 tools/perframe.py 400 || exit 1
done
MM355_LIB=$V timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pftr_fc -o run --output-format csv -- python3 $R/tools/perframe.py 300 > /dev/null 2> gpurun_out/pftr_fc.err && python3 tools/pf_trace.py gpurun_out/pftr_fc/run_kernel_trace.csv || exit 1
MM_K2_NOFC=1 MM355_LIB=$V timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pftr_nofc -o run --output-format csv -- python3 $R/tools/perframe.py 300 > /dev/null 2> gpurun_out/pftr_nofc.err && python3 tools/pf_trace.py gpurun_out/pftr_nofc/run_kernel_trace.csv || exit 1
