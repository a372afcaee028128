#!/bin/bash
# r05 step 24: per-rank compute of the 8-way split at the default 2 stages on the final kernels
# (virtual ranks, K=100 and K=200; r05s23's run stopped at the script's old 4-stage default), and the
# biased sampler's line with its roofline on the launch that moves the most bytes.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for K in 100 200; do
  timeout -k 10 300 python3 "$R/profiles/r05/rank_stages.py" --K $K > "$O/r05s24_rank_k${K}_s2.json" 2> "$O/r05s24_rank_k${K}_s2.txt"
  python3 -c "
import json; d=json.load(open('$O/r05s24_rank_k${K}_s2.json')); print('rank K=$K stages=2: max user %.3f item %.3f max sweep %.3f' % (d['max_over_ranks']['user'], d['max_over_ranks']['item'], max(x['ms_sweep'] for x in d['per_rank'])))"
done
# the biased sampler's line again, its roofline now on the launch with the most algorithmic bytes
timeout -k 10 400 python3 "$R/bench.py" --quirks bias2 > "$O/r05s24_bench_bias2.json" 2> "$O/r05s24_bias2.err"
python3 -c "
import json; d=json.load(open('$O/r05s24_bench_bias2.json')); print('bias2', round(d['ms_per_step'],3), d['roofline']['kernel'], round(d['roofline']['frac'],3), d.get('cpu_baseline',{}).get('value'))"
