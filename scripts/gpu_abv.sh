# Same-call A/B of compiled variants lib/variants/*.so (bench batch pattern and
# optionally per-frame), R rounds.  usage: bash scripts/gpu_abv.sh ROUNDS [pf]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=${1:-2}; PF=$2
for i in $(seq $N); do
  for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
    n=$(basename $V .so)
    MM355_LIB=$R/$V timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/abv_$n.json 2> gpurun_out/abv_$n.err || { echo BENCH FAIL $n; tail gpurun_out/abv_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/abv_$n.json $n
    if [ -n "$PF" ]; then
      MM355_LIB=$R/$V timeout -k 10 240 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --frames-per-step 100 > gpurun_out/abvpf_$n.json 2> gpurun_out/abvpf_$n.err || { echo PF FAIL $n; tail gpurun_out/abvpf_$n.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['drop_in_per_frame']; print(sys.argv[2], 'drop-in', d['frames_per_s'], d['latency_ms'])" gpurun_out/abvpf_$n.json $n
    fi
  done
done
echo ALL OK
