# One-frame-per-call path: rate with/without device kernargs, kernel trace gaps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/perframe.py 400 > gpurun_out/pf_base.json 2>gpurun_out/pf_base.err || { echo FAIL base; tail gpurun_out/pf_base.err; exit 1; }
echo base; cat gpurun_out/pf_base.json
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python3 tools/perframe.py 400 > gpurun_out/pf_dk.json 2>gpurun_out/pf_dk.err || { echo FAIL dk; exit 1; }
echo devkernarg; cat gpurun_out/pf_dk.json
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python3 tools/perframe.py 400 > gpurun_out/pf_hk.json 2>gpurun_out/pf_hk.err || { echo FAIL hk; exit 1; }
echo hostkernarg; cat gpurun_out/pf_hk.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pf_tr -o run --output-format csv -- python3 $R/tools/perframe.py 300 > gpurun_out/pf_tr.json 2> gpurun_out/pf_tr.err || { echo PF PROF FAIL; tail gpurun_out/pf_tr.err; exit 1; }
python3 tools/pf_trace.py gpurun_out/pf_tr/run_kernel_trace.csv
echo ALL OK
