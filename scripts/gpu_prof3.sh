# K2 phase stamps (stamps variant), SQ stall counters of the default bench,
# rocprof kernel summaries of the batch bench and of the drop-in per-frame path.
# usage: bash scripts/gpu_prof3.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-p3}; export TMPDIR=/tmp
bash scripts/gpu_k2_phases.sh > gpurun_out/${TAG}_k2ph.txt 2>&1 || { echo PHASES FAIL; tail gpurun_out/${TAG}_k2ph.txt; exit 1; }
cat gpurun_out/${TAG}_k2ph.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { echo PROF FAIL; exit 1; }
cut -d, -f1-8 gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-50,150-
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_pf -o run --output-format csv -- python3 $R/tools/perframe.py 300 > gpurun_out/${TAG}_pf.json 2> gpurun_out/${TAG}_pf.err || { echo PF PROF FAIL; tail gpurun_out/${TAG}_pf.err; exit 1; }
cat gpurun_out/${TAG}_pf.json
python3 -c "
import csv,sys
for r in csv.DictReader(open('gpurun_out/${TAG}_pf/run_kernel_stats.csv')): print(r['Name'][:34], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])"
timeout -k 10 120 python3 tools/perframe.py 300 > gpurun_out/${TAG}_pf_noprof.json && cat gpurun_out/${TAG}_pf_noprof.json
bash scripts/gpu_stall.sh ${TAG}_st > /dev/null || { echo STALL FAIL; exit 1; }
cat gpurun_out/${TAG}_st_summary.json
echo ALL OK
