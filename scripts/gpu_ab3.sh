# Same-call A/B: round-2 library vs the working tree, env knobs of the tree,
# batch and per-frame call patterns.  usage: bash scripts/gpu_ab3.sh ROUNDS
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; N=${1:-2}
V=$R/phase-based-motion-manipulation_amd/lib/variants
run() {  # name, env..., -- bench args
  local n=$1; shift; local E=(); while [ "$1" != "--" ]; do E+=("$1"); shift; done; shift
  env "${E[@]}" timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 "$@" > gpurun_out/ab3_$n.json 2> gpurun_out/ab3_$n.err || { echo BENCH FAIL $n; tail gpurun_out/ab3_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/ab3_$n.json $n
}
for i in $(seq $N); do
  run r02 MM355_LIB=$V/r02.so -- --steps 5 || exit 1
  run cur A=1 -- --steps 5 || exit 1
  run nopow MM_K2_NOPOW=1 -- --steps 5 || exit 1
  run pf_r02 MM355_LIB=$V/r02.so -- --call-pattern per-frame --frames-per-step 200 --steps 3 --warmup 1 || exit 1
  run pf_cur A=1 -- --call-pattern per-frame --frames-per-step 200 --steps 3 --warmup 1 || exit 1
  run pf_r4 MM_K34_ROWS=4 -- --call-pattern per-frame --frames-per-step 200 --steps 3 --warmup 1 || exit 1
  run pf_r8 MM_K34_ROWS=8 -- --call-pattern per-frame --frames-per-step 200 --steps 3 --warmup 1 || exit 1
done
echo ALL OK
