# K2 time split (L=1: no middle bands -> no phase op; L=5) + VALU counters of the default bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
for L in 1 5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --levels $L 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('L=$L', d['value'], {k:v['us_per_frame'] for k,v in d['kernels'].items()})" || { echo "L=$L FAIL"; exit 1; }
done
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS -d $R/gpurun_out/split_pmc -o run --output-format csv -- $B > /dev/null 2> gpurun_out/split_pmc.err || { echo PMC FAIL; tail -3 gpurun_out/split_pmc.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/split_kt -o run --output-format csv -- $B > /dev/null 2> gpurun_out/split_kt.err || { echo KT FAIL; exit 1; }
python3 tools/valu_summary.py gpurun_out/split_pmc gpurun_out/split_kt gpurun_out/valu.json
