# Stall breakdown per kernel (SQ counters, kernel-trace only; one pass per set).
# usage: bash scripts/gpu_stall.sh TAG [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
TAG=${1:-stall}; shift
B="python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 2 --warmup 1 $*"
i=0
for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/${TAG}_$i -o run --output-format csv -- $B > /dev/null 2> gpurun_out/${TAG}_$i.err || { echo PMC set $i FAIL; tail -5 gpurun_out/${TAG}_$i.err; exit 1; }
done
python3 tools/stall_summary.py gpurun_out/${TAG}_1 gpurun_out/${TAG}_2 > gpurun_out/${TAG}_summary.json
cat gpurun_out/${TAG}_summary.json
