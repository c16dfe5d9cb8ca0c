# bench at batch 100 / 150 / 300 (300-frame steps) and K34 strip heights, two rounds
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
one() {  # tag batch env...
  tag=$1; b=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 --batch $b > gpurun_out/bb_$tag.json 2>gpurun_out/bb_$tag.err || return 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/bb_$tag.json $tag
}
for r in 1 2; do
  one b100 100 || exit 1
  one b150 150 || exit 1
  one b300 300 || exit 1
  one b100_r96 100 MM_K34_ROWS=96 || exit 1
  one b100_r128 100 MM_K34_ROWS=128 || exit 1
done
