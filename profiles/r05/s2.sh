#!/bin/bash
# r05 step 2: per-rank stage compute of the 8-way split of config 4 (ML-20M K=200, 4 stages
# per half; virtual ranks, exchange skipped), then a rocprofv3 per-dispatch trace of the rank
# holding the longest split item row.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 600 python3 "$R/profiles/r05/rank_stages.py" > "$O/r05s2_rank_stages.json" 2> "$O/r05s2_rank_stages.err"
cat "$O/r05s2_rank_stages.err"
RL=$(python3 -c "
import json,sys
d=json.load(open('$O/r05s2_rank_stages.json'))
print(max(d['per_rank'], key=lambda x: x['halves']['item']['longest_row'])['rank'])")
echo "longest item row on rank $RL"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/r05s2_rank${RL}_trace" -o r05s2 -- \
    python3 "$R/profiles/r05/rank_stages.py" --only "$RL" --sweeps 2 > "$O/r05s2_rank${RL}_trace.log" 2>&1
tail -2 "$O/r05s2_rank${RL}_trace.log"
