# A/B of the batch pipeline: variants x (frames per step, batch) configurations
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for cfg in "100 100" "300 100" "300 50" "600 100"; do
  set -- $cfg
  for V in phase-based-motion-manipulation_amd/lib/variants/*.so; do
    n=$(basename $V .so)
    MM355_LIB=$R/$V timeout -k 10 200 python bench.py --no-cpu-baseline --drop-in-frames 0 --frames-per-step $1 --batch $2 > gpurun_out/pipe_${n}_$1_$2.json 2> gpurun_out/pipe_${n}_$1_$2.err || { echo $n FAIL; tail gpurun_out/pipe_${n}_$1_$2.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})" gpurun_out/pipe_${n}_$1_$2.json "$n" "$1/$2"
  done
done
