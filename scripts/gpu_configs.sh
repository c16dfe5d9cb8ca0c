# bench lines for the other BASELINE configs and modes (no CPU baseline).
# usage: bash scripts/gpu_configs.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-cfg}
run() {
  n=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { echo BENCH $n FAIL; tail -5 gpurun_out/${TAG}_$n.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['config']['workload'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_$n.json $n
}
run c2 && run c3_4k --width 3840 --height 2160 --levels 6 && run c2_std --standard && \
run c2_o8diff --orientations 8 && run c2_o8iir --orientations 8 --temporal-filter iir && \
run c2_o4 --orientations 4 && run c2_fps60 --frames-per-step 60 --steps 5 && \
run c3_o8diff --width 3840 --height 2160 --levels 6 --orientations 8 --steps 2 --warmup 1 && \
run c5k --width 5120 --height 2880 --frames-per-step 30 --batch 15 --steps 2 --warmup 1
