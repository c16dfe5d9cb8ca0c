# gpu_try.sh plus one SQ-counter pass summary (LDS conflicts, VALU count) per kernel.
# usage: bash scripts/gpu_try_st.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; TAG=${1:-try}
bash scripts/gpu_try.sh $TAG || exit 1
bash scripts/gpu_stall.sh ${TAG}_st > /dev/null || { echo STALL FAIL; exit 1; }
python3 -c "
import json, sys
s = json.load(open(sys.argv[1]))
for k in ('k_rows_fwd', 'k_cols', 'k_rows_inv', 'k_compose'):
    print(k, 'lds_conflict', s[k].get('lds_conflict_frac'), 'valu', s[k]['SQ_INSTS_VALU'], 'lds_insts', s[k]['SQ_INSTS_LDS'])
" gpurun_out/${TAG}_st_summary.json
