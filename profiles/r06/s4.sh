#!/bin/bash
# r06 step 4: after removing the per-XCD queues and the sweep graph (both measured slower, r06s3):
# the default bench line (every leg), then the wave-0 phase profile (KPROF build, SBMF_KPROF=1) of
# the streaming sets -- set 0: the user 4-wave and item 8-wave sets; set 1: the user 8-wave and
# item 16-wave sets.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
bash profiles/collect.sh r06s4 bench
python3 -c "
import json; d=json.load(open('$O/r06s4_bench.json')); c=d['config']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), d['roofline']['frac'], d['cpu_baseline']['value'], d['f32_ms_per_step'])"
K=$R/scalable-bayesian-matrix-factorization_amd/build_kprof/libsbmf.so
for set in 0 1; do
  SBMF_LIB=$K SBMF_KPROF=1 SBMF_KPROF_SET=$set timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu \
      --no-ttr --no-f32 --no-load > "$O/r06s4_kprof_set$set.json" 2> "$O/r06s4_kprof_set$set.txt"
  echo "== set $set"
  grep "sweep 3 gres" -A 3 "$O/r06s4_kprof_set$set.txt" | head -8
done
