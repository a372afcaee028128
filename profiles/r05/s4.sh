#!/bin/bash
# r05 step 4: per-rank compute of the 8-way split vs stages per half (virtual ranks), at the
# bench's K=100 and config 4's K=200, plus a bench line of the current HEAD (colstats / k_test
# / solve changes) and a parity subset.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_bias.py > "$O/r05s4_parity.log" 2>&1 \
    || { tail -30 "$O/r05s4_parity.log"; exit 1; }
tail -1 "$O/r05s4_parity.log"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for K in 100 200; do for S in 1 2 4; do
  SBMF_STAGES=$S timeout -k 10 300 python3 "$R/profiles/r05/rank_stages.py" --K $K > "$O/r05s4_rank_stages_k${K}_s${S}.json" 2> "$O/r05s4_rank_stages_k${K}_s${S}.txt"
  python3 -c "
import json; d=json.load(open('$O/r05s4_rank_stages_k${K}_s${S}.json')); print('K=$K stages=$S max user %.3f item %.3f max sweep %.3f' % (d['max_over_ranks']['user'], d['max_over_ranks']['item'], max(x['ms_sweep'] for x in d['per_rank'])))"
done; done
bash "$R/profiles/collect.sh" r05s4 bench
python3 -c "
import json; d=json.load(open('$O/r05s4_bench.json')); c=d['config']; print('bench', d['ms_per_step'], c['ms_user_half'], c['ms_item_half'], c['ms_hyper'], c['ms_eval'])"
