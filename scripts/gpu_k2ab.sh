# K2 A/B: parity suite on the default build, then the bench under K2 variants.
# usage: bash scripts/gpu_k2ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-k2ab}
export TMPDIR=/tmp
MM_K2=wave timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for V in "MM_K2=legacy" "MM_NSUB=2" "MM_NSUB=4"; do
  env MM_K2=wave $V timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_$V.json 2> gpurun_out/${TAG}_bench_$V.err || { echo BENCH $V FAIL; tail gpurun_out/${TAG}_bench_$V.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_bench_$V.json $V
done
