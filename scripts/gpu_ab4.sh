# batch bench + per-frame rate per variant, plus MM_K2_TAIL settings for the last variant
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
run() {  # name lib env...
  n=$1; V=$2; shift 2
  env "$@" MM355_LIB=$V timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/ab4_$n.json 2> gpurun_out/ab4_$n.err || { echo BENCH FAIL $n; tail gpurun_out/ab4_$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/ab4_$n.json $n
  env "$@" MM355_LIB=$V timeout -k 10 120 python3 tools/perframe.py 400 | sed "s/^/$n pf /" || return 1
}
L=$R/phase-based-motion-manipulation_amd/lib/variants
for i in 1 2; do
  run base $L/a_base.so || exit 1
  run pkx2 $L/b_pkx2.so || exit 1
  run pkx2_t20 $L/b_pkx2.so MM_K2_TAIL=20 || exit 1
  run pkx2_t10 $L/b_pkx2.so MM_K2_TAIL=10 || exit 1
done
echo ALL OK
