# Batch-size sweep: per-kernel us/frame at 300-frame steps for several
# mm_set_batch sizes (small batches keep a batch's intermediates G, Q, Yh
# resident in the 256 MiB Infinity Cache between producer and consumer).
# usage: bash scripts/gpu_batch_sweep.sh "8 12 16 25 50 100"
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for b in ${1:-8 16 25 50 100}; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --batch $b --steps 5 --warmup 2 > gpurun_out/bs_$b.json 2> gpurun_out/bs_$b.err || { echo FAIL $b; tail -3 gpurun_out/bs_$b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('batch', sys.argv[2], d['value'], d['ms_per_step'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/bs_$b.json $b
done
