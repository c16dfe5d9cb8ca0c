set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for c in "30 10" "50 6" "60 5" "100 3" "150 2" "300 1"; do
  set -- $c
  timeout -k 10 240 python bench.py --no-cpu-baseline --frames-per-step $1 --steps $2 --warmup 2 > gpurun_out/ch_$1.json 2> gpurun_out/ch_$1.err || { echo FAIL $1; tail -3 gpurun_out/ch_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/ch_$1.json "$1x$2"
done
