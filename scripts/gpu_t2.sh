set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
V=$R/phase-based-motion-manipulation_amd/lib/variants/t2.so
MM355_LIB=$V timeout -k 10 120 python3 tools/tail2_check.py 10 20 30 || exit 1
for i in 1 2; do for t in 0 10 20 30; do
  MM_K2_TAIL2=$t MM355_LIB=$V timeout -k 10 240 python bench.py --no-cpu-baseline --drop-in-frames 0 --steps 5 > gpurun_out/t2_$t.json 2> gpurun_out/t2_$t.err || { echo FAIL; tail gpurun_out/t2_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/t2_$t.json $t
done; done
