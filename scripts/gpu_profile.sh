# Profile evidence for one bench configuration, in one call: rocprofv3 kernel
# stats of the bench, PMC traffic (FETCH_SIZE and WRITE_SIZE in separate
# kernel-trace-only passes, corrected on tools/pmc_calib), SQ stall and VALU
# counter sets (one pass each), and the VALU summary.
# usage: bash scripts/gpu_profile.sh TAG [bench args...]
#   e.g.  bash scripts/gpu_profile.sh r04c_c3 --width 3840 --height 2160 --levels 6
# The bench batch (frames per K2 launch) is read from the args (--batch, default 150).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
TAG=${1:-prof}; shift
EXTRA="$*"
FPS=$(python3 -c "import sys; a=sys.argv[1:]; print(a[a.index('--batch')+1] if '--batch' in a else 150)" $EXTRA)
KEY=$(python3 -c "
import sys, bench
a = bench.parse_args(sys.argv[1:])
print(bench.profile_key(a.width, a.height, a.levels, a.orientations, a.standard, a.temporal_filter))" $EXTRA)
B="python3 $R/bench.py --no-cpu-baseline --drop-in-frames 0 --steps 2 --warmup 1 $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- $B > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_prof.err || { echo PROF FAIL; tail gpurun_out/${TAG}_prof.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $R/gpurun_out/${TAG}_$C -o run --output-format csv -- $B > /dev/null 2> gpurun_out/${TAG}_$C.err || { echo PMC $C FAIL; tail gpurun_out/${TAG}_$C.err; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/${TAG}_cal_$C -o run --output-format csv -- $R/tools/bin/pmc_calib > /dev/null 2> gpurun_out/${TAG}_cal_$C.err || { echo CAL $C FAIL; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE gpurun_out/${TAG}_cal_FETCH_SIZE gpurun_out/${TAG}_cal_WRITE_SIZE $FPS gpurun_out/${TAG}_traffic.json $KEY || { echo PMC SUMMARY FAIL; exit 1; }
i=0
for CNT in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $R/gpurun_out/${TAG}_st_$i -o run --output-format csv -- $B > /dev/null 2> gpurun_out/${TAG}_st_$i.err || { echo PMC set $i FAIL; tail -5 gpurun_out/${TAG}_st_$i.err; exit 1; }
done
python3 tools/stall_summary.py gpurun_out/${TAG}_st_1 gpurun_out/${TAG}_st_2 > gpurun_out/${TAG}_stall.json || { echo STALL SUMMARY FAIL; exit 1; }
python3 tools/valu_summary.py gpurun_out/${TAG}_st_1,gpurun_out/${TAG}_st_2 gpurun_out/${TAG}_prof gpurun_out/${TAG}_valu.json $KEY || { echo VALU SUMMARY FAIL; exit 1; }
echo PROFILE OK
