# Same-call A/B of the one-frame (drop-in) call under launch-shape variants:
# each "NAME:ENV=VAL,..." runs bench.py's drop-in measurement (300 frame calls)
# R rounds; prints frames/s, p50 and p99 per call.
# usage: bash scripts/gpu_pf_variants.sh R NAME[:ENV=VAL,...] ...
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=$1; shift
for i in $(seq $N); do
  for spec in "$@"; do
    n=${spec%%:*}; envs=""; [ "$spec" != "$n" ] && envs=${spec#*:}
    E=""; for kv in ${envs//,/ }; do E="$E $kv"; done
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --drop-in-frames 300 > gpurun_out/pf_$n.json 2> gpurun_out/pf_$n.err || { echo BENCH FAIL $n; tail gpurun_out/pf_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['drop_in_per_frame']; print(sys.argv[2], d['frames_per_s'], d['latency_ms'])" gpurun_out/pf_$n.json $n
  done
done
