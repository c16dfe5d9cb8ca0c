# Interleaved A/B of library variants lib/variants/*.so (bench only, no parity).
# usage: bash scripts/gpu_variants.sh TAG ROUNDS [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-var}; ROUNDS=${2:-2}; shift 2
for r in $(seq $ROUNDS); do
  for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
    n=$(basename $V .so)
    MM355_LIB=$R/$V timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { echo BENCH $n FAIL; tail gpurun_out/${TAG}_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_$n.json "$n"
  done
done
