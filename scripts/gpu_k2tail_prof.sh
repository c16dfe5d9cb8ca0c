# k_cols / k_cols_tail durations per launch for a few MM_K2_TAIL shares.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
for T in ${1:-0 12 20}; do
  MM_K2_TAIL=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k2t_$T -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 3 > gpurun_out/k2t_$T.json 2> gpurun_out/k2t_$T.err || { echo PROF FAIL; tail gpurun_out/k2t_$T.err; exit 1; }
  echo "MM_K2_TAIL=$T"; grep -E "k_cols" gpurun_out/k2t_$T/run_kernel_stats.csv | cut -d, -f1-4 | sed 's/(float __vector.*"/"/'
done
