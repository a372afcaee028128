#!/bin/bash
# r05 step 38: the other lines on the final kernels (item streaming tasks in the 3/4 size class) -- configs 2-4 (ML-1M K=50, ML-10M K=100,
# ML-20M K=200), the biased sampler (bias2), and the per-rank compute of the 8-way split at the
# default 2 stages (virtual ranks, K=100 and K=200).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for cfg in "ml-1m 50" "ml-10m 100" "ml-20m 200"; do
  set -- $cfg
  timeout -k 10 400 python3 "$R/bench.py" --shape $1 --K $2 --no-ttr --no-load > "$O/r05s38_bench_$1_k$2.json" 2> "$O/r05s38_bench_$1_k$2.err"
  python3 -c "
import json; d=json.load(open('$O/r05s38_bench_$1_k$2.json')); print('$1 K$2', round(d['ms_per_step'],3), d['value'], d['f32_ms_per_step'], d['roofline']['frac'])"
done
# the biased line (its roofline on the launch with the most bytes)
timeout -k 10 400 python3 "$R/bench.py" --quirks bias2 > "$O/r05s38_bench_bias2.json" 2> "$O/r05s38_bias2.err"
python3 -c "
import json; d=json.load(open('$O/r05s38_bench_bias2.json')); print('bias2', round(d['ms_per_step'],3), d.get('cpu_baseline',{}).get('value'))"
for K in 100 200; do
  timeout -k 10 300 python3 "$R/profiles/r05/rank_stages.py" --K $K > "$O/r05s38_rank_k${K}_s2.json" 2> "$O/r05s38_rank_k${K}_s2.txt"
  python3 -c "
import json; d=json.load(open('$O/r05s38_rank_k${K}_s2.json')); print('rank K=$K stages=2: max user %.3f item %.3f max sweep %.3f' % (d['max_over_ranks']['user'], d['max_over_ranks']['item'], max(x['ms_sweep'] for x in d['per_rank'])))"
done
cd "$R"
bash profiles/collect.sh r05s38 fetch && bash profiles/collect.sh r05s38 write && bash profiles/collect.sh r05s38 lds
echo pmc done
