# Same-call A/B of library variants with the drop-in (one call per frame) rate:
# R rounds of NAME=LIB pairs (LIB "cur" = the working-tree library, else
# lib/variants/LIB.so), bench args after "--".
# usage: bash scripts/gpu_abd.sh R VARIANT... -- [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=$1; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
for i in $(seq $N); do
  for spec in "${V[@]}"; do
    n=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*:}
    E=""; [ "$lib" != cur ] && E="MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/$lib.so"
    for kv in ${envs//,/ }; do E="$E $kv"; done
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 "$@" > gpurun_out/abd_${n}_$i.json 2> gpurun_out/abd_${n}_$i.err || { echo BENCH FAIL $n; tail gpurun_out/abd_${n}_$i.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); p=d.get('drop_in_per_frame') or {}
print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()}, 'drop-in', p.get('frames_per_s'), (p.get('latency_ms') or {}).get('p99'))" gpurun_out/abd_${n}_$i.json $n
  done
done
