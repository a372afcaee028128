#!/bin/bash
# r06 step 22: libFM's own MCMC and ALS lines (ML-20M-shaped, K=100) on the final tree, with their
# CPU baselines, and the biased line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for m in libfm als; do
  timeout -k 10 600 python3 "$R/bench.py" --method $m > "$O/r06s22_bench_$m.json" 2> "$O/r06s22_bench_$m.err"
  python3 -c "
import json; d=json.load(open('$O/r06s22_bench_$m.json')); print('$m', round(d['ms_per_step'],2), d['value'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
done
