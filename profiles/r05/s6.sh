#!/bin/bash
# r05 step 6: stages per half for the 8-way split with the two side streams (default now):
# per-rank compute at 1 / 2 / 4 stages, K=100 and K=200; a per-dispatch trace of rank 0 at
# K=100 with one stage; the default bench line's rocprofv3 trace.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for K in 100 200; do for S in 1 2 4; do
  SBMF_STAGES=$S timeout -k 10 300 python3 "$R/profiles/r05/rank_stages.py" --K $K > "$O/r05s6_rank_k${K}_s${S}.json" 2> "$O/r05s6_rank_k${K}_s${S}.txt"
  python3 -c "
import json; d=json.load(open('$O/r05s6_rank_k${K}_s${S}.json')); print('K=$K stages=$S: max user %.3f item %.3f max sweep %.3f' % (d['max_over_ranks']['user'], d['max_over_ranks']['item'], max(x['ms_sweep'] for x in d['per_rank'])))"
done; done
SBMF_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/r05s6_rank0_k100_s1" -o r05s6 -- \
    python3 "$R/profiles/r05/rank_stages.py" --K 100 --only 0 --sweeps 2 > "$O/r05s6_rank0_trace.log" 2>&1
tail -1 "$O/r05s6_rank0_trace.log"
bash "$R/profiles/collect.sh" r05s6 trace
tail -1 "$O/r05s6_trace.log"
