set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
run() { timeout -k 10 200 env "$@" python bench.py --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(sys.argv[1:], d['value'], {k:round(v['ms_per_launch']/v['frames']*v['launches']*1000,2) for k,v in d['kernels'].items()})" "$@"; }
run MM_X=0
run MM_DIAG_SKIP_NYQUIST=1
run MM_CHUNK=8
run MM_CHUNK=16
