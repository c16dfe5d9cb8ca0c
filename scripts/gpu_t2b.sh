set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
bash scripts/gpu_tests.sh r03i_tests || exit 1
for i in 1 2; do for t in 5 10 15; do
  MM_K2_TAIL2=$t timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/t2_$t.json 2> gpurun_out/t2_$t.err || { echo FAIL; tail gpurun_out/t2_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/t2_$t.json $t
done; done
