# Same-call A/B of named variants, each "NAME=LIB[:ENV=VAL,...]" (LIB "cur" =
# the working-tree library), R rounds, bench args after "--".
# usage: bash scripts/gpu_abx.sh R VARIANT... -- [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=$1; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
for i in $(seq $N); do
  for spec in "${V[@]}"; do
    n=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*:}
    E=""; [ "$lib" != cur ] && E="MM355_LIB=$R/phase-based-motion-manipulation_amd/lib/variants/$lib.so"
    for kv in ${envs//,/ }; do E="$E $kv"; done
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 "$@" > gpurun_out/abx_$n.json 2> gpurun_out/abx_$n.err || { echo BENCH FAIL $n; tail gpurun_out/abx_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/abx_$n.json $n
  done
done
