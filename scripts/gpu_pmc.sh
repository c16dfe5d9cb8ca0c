# rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs, kernel-trace
# only, no sys/runtime trace) on the bench and on the calibration kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-pmc}
export TMPDIR=/tmp
FPS=100   # frames per K2 launch = bench.py batch
B="python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 1 --warmup 1 --frames-per-step 300 --batch $FPS"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $R/gpurun_out/${TAG}_$C -o run --output-format csv -- $B > /dev/null 2> gpurun_out/${TAG}_$C.err || { echo PMC $C FAIL; tail gpurun_out/${TAG}_$C.err; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $C -d $R/gpurun_out/${TAG}_cal_$C -o run --output-format csv -- $R/tools/bin/pmc_calib > /dev/null 2> gpurun_out/${TAG}_cal_$C.err || { echo CAL $C FAIL; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE gpurun_out/${TAG}_cal_FETCH_SIZE gpurun_out/${TAG}_cal_WRITE_SIZE $FPS gpurun_out/${TAG}_traffic.json
