#!/bin/bash
# r06 step 5: the item half's two streaming sets one after the other on small stages (below
# 4 M ratings; SBMF_SETS_SIDE_MIN=0 restores side by side everywhere): ML-1M K=50 (config 2) and
# the default ML-20M line, 3 interleaved rounds each; then the per-rank compute of the 8-way split
# (virtual ranks, K=100 and K=200, 2 stages) with both settings.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'hyper', round(c['ms_hyper'],3), 'eval', round(c['ms_eval'],3))"; }
for i in 1 2 3; do
  for m in 4000000 0; do
    SBMF_SETS_SIDE_MIN=$m timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr \
      --no-f32 --no-load > "$O/r06s5_ml1m_m${m}_$i.json" 2> "$O/r06s5_ml1m_m${m}_$i.err"
    show "$O/r06s5_ml1m_m${m}_$i.json" "ml1m min=$m round $i"
  done
done
for i in 1 2; do
  for m in 4000000 0; do
    SBMF_SETS_SIDE_MIN=$m timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s5_ml20m_m${m}_$i.json" 2> "$O/r06s5_ml20m_m${m}_$i.err"
    show "$O/r06s5_ml20m_m${m}_$i.json" "ml20m min=$m round $i"
  done
done
for K in 100 200; do
  for m in 4000000 0; do
    SBMF_SETS_SIDE_MIN=$m timeout -k 10 300 python3 profiles/r05/rank_stages.py --K $K > "$O/r06s5_rank_k${K}_m$m.json" \
      2> "$O/r06s5_rank_k${K}_m$m.txt"
    echo "== K=$K min=$m"; tail -8 "$O/r06s5_rank_k${K}_m$m.txt"
  done
done
