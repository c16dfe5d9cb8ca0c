# parity (default K2 and wave K2) + bench per K2 form.  usage: bash scripts/gpu_ab2.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-ab2}
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/${TAG}_tests.log 2>&1 || { echo TEST FAIL; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
MM_K2=wave timeout -k 10 600 python -m pytest tests -q -m gpu -x -k "golden or stream or chunk or standard" > gpurun_out/${TAG}_tests_wave.log 2>&1 || { echo WAVE TEST FAIL; tail -40 gpurun_out/${TAG}_tests_wave.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests_wave.log
for V in "MM_K2=legacy" "MM_K2=wave MM_NSUB=2" "MM_K2=wave MM_NSUB=4"; do
  env $V timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH $V FAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_bench.json "$V"
done
