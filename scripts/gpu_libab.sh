# Same-call A/B of library variants: the bench alternately with each
# lib/variants/*.so and the working-tree library ("cur"), R rounds.
# usage: bash scripts/gpu_libab.sh [ROUNDS [bench args...]]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=${1:-2}; shift; EXTRA="$*"
for i in $(seq $N); do
  for V in cur phase-based-motion-manipulation_amd/lib/variants/*.so; do
    n=$(basename $V .so)
    if [ $V = cur ]; then E=""; else E="MM355_LIB=$R/$V"; fi
    env $E timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 $EXTRA > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo BENCH FAIL $n; tail gpurun_out/ab_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/ab_$n.json $n
  done
done
