set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
for L in 1 2 5; do timeout -k 10 200 python bench.py --no-cpu-baseline --levels $L 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('L=$L', d['value'], {k:v['us_per_frame'] for k,v in d['kernels'].items()})"; done
