# VALU issue utilisation per kernel: SQ counter passes + a kernel-trace run of
# the same bench, summarised by tools/valu_summary.py.  usage: gpu_valu.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp; TAG=${1:-valu}
bash scripts/gpu_stall.sh ${TAG}_st > /dev/null || { echo STALL FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 2 --warmup 1 > /dev/null 2> gpurun_out/${TAG}_prof.err || { echo PROF FAIL; exit 1; }
python3 tools/valu_summary.py gpurun_out/${TAG}_st_1,gpurun_out/${TAG}_st_2 gpurun_out/${TAG}_prof gpurun_out/${TAG}_valu.json
python3 -c "
import json,sys
v=json.load(open(sys.argv[1])); s=json.load(open(sys.argv[2]))
for k in ('k_rows_fwd','k_cols','k_rows_inv','k_compose','k_rows_inv_compose'):
    print(k, {a: v[k][a] for a in ('valu_insts_per_launch','launch_s','clock_GHz','valu_busy')}, {a: s[k].get(a) for a in ('frac_SQ_WAIT_ANY','frac_SQ_WAIT_INST_ANY','frac_SQ_ACTIVE_INST_ANY','lds_conflict_frac')})
" gpurun_out/${TAG}_valu.json gpurun_out/${TAG}_st_summary.json
