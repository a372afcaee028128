#!/bin/bash
# r06 step 7: the 8-way split's per-rank compute (virtual ranks, 2 stages) with smaller streaming
# tasks for a rank's small stages: all item rows on 8-wave k_gres workgroups (tune bit 27: 1024-rating
# tasks, two workgroups per CU), all user rows on the 4-wave set (bit 13: 512-rating tasks), both;
# K=200 (config 4) and K=100.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
for K in 200 100; do
  for t in 0 134217728 8192 134225920; do
    timeout -k 10 300 python3 profiles/r05/rank_stages.py --K $K --tune $t > "$O/r06s7_rank_k${K}_t$t.json" \
      2> "$O/r06s7_rank_k${K}_t$t.txt"
    python3 - "$O/r06s7_rank_k${K}_t$t.txt" "K=$K tune=$t" <<'PY'
import re, sys
v = [tuple(map(float, re.findall(r"sweep ([\d.]+) ms  user ([\d.]+)  item ([\d.]+)", l)[0])) for l in open(sys.argv[1]) if l.startswith("rank")]
print(sys.argv[2], "max sweep %.3f  max user %.3f  max item %.3f" % tuple(max(x[i] for x in v) for i in range(3)))
PY
  done
done
