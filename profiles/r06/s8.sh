#!/bin/bash
# r06 step 8: (1) fewer event packets at the half boundaries (the half forks its side streams from,
# and times its first kind by, the event its caller just recorded: the sweep start / the user half's
# end) -- this build against the previous one (build_prev, SBMF_LIB), ML-1M K=50 and ML-20M, 3
# interleaved rounds; (2) the 8-way per-rank compute with smaller streaming tasks (r06s7's plan).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
P=$R/scalable-bayesian-matrix-factorization_amd/build_prev/libsbmf.so
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'hyper', round(c['ms_hyper'],3), 'eval', round(c['ms_eval'],3))"; }
for i in 1 2 3; do
  for v in new prev; do
    L=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so; [ $v = prev ] && L=$P
    SBMF_LIB=$L timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr \
      --no-f32 --no-load > "$O/r06s8_ml1m_${v}_$i.json" 2> "$O/r06s8_ml1m_${v}_$i.err"
    show "$O/r06s8_ml1m_${v}_$i.json" "ml1m $v round $i"
    SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s8_ml20m_${v}_$i.json" 2> "$O/r06s8_ml20m_${v}_$i.err"
    show "$O/r06s8_ml20m_${v}_$i.json" "ml20m $v round $i"
  done
done
bash profiles/r06/s7.sh
