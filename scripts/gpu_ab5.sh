set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
L=$R/phase-based-motion-manipulation_amd/lib/variants
run() { n=$1; V=$2; shift 2
  env "$@" MM355_LIB=$V timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/ab5_$n.json 2> gpurun_out/ab5_$n.err || { echo FAIL $n; tail -5 gpurun_out/ab5_$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()}, d['parity_vs_oracle']['max_abs_lsb'] if 'parity_vs_oracle' in d else '')" gpurun_out/ab5_$n.json $n; }
for i in 1 2; do
  run g2 $L/a_g2.so || exit 1
  run g4 $L/b_g4.so || exit 1
  run g4t15 $L/c_g4t15.so MM_K2_TAIL=15 || exit 1
  run g4t0 $L/c_g4t15.so MM_K2_TAIL=0 || exit 1
done
