# SQ counter passes per library variant (lib/variants/*.so), kernel-trace only.
# usage: bash scripts/gpu_ab_counters.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
TAG=${1:-abc}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_avail.txt 2>&1 || true
for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
  n=$(basename $V .so)
  i=0
  for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_VMEM"; do
    i=$((i+1))
    MM355_LIB=$R/$V timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/${TAG}_${n}_$i -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 1 --warmup 1 > /dev/null 2> gpurun_out/${TAG}_${n}_$i.err || { echo PMC $n $i FAIL; tail -5 gpurun_out/${TAG}_${n}_$i.err; exit 1; }
  done
  python3 tools/stall_summary.py gpurun_out/${TAG}_${n}_1 gpurun_out/${TAG}_${n}_2 > gpurun_out/${TAG}_${n}_summary.json
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['k_cols']
print(sys.argv[2], {k: d[k] for k in ('SQ_INSTS_VALU','SQ_ACTIVE_INST_VALU','SQ_WAVE_CYCLES','SQ_BUSY_CYCLES','SQ_INSTS_LDS','frac_SQ_WAIT_ANY','frac_SQ_WAIT_INST_ANY','frac_SQ_ACTIVE_INST_ANY','lds_conflict_frac')})" gpurun_out/${TAG}_${n}_summary.json $n
done
