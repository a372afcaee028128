#!/bin/bash
# r06 step 15: the item half's two streaming sets one after the other at ML-20M too (set 0, the rows
# of <= 1024 ratings, then set 1; SBMF_SETS_SIDE_MIN above the stage size) against side by side: the
# r06s14 trace has set 0 starved beside set 1 (no VGPR room on a CU that holds a 16-wave set-1
# workgroup), the stage 3.52 ms against 2.95 + 0.45 ms standalone.  3 interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'stage', round(d['roofline']['ms_per_launch'],3))"; }
for i in 1 2 3; do
  for m in 4000000 1000000000; do
    SBMF_SETS_SIDE_MIN=$m timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s15_m${m}_$i.json" 2> "$O/r06s15_m${m}_$i.err"
    show "$O/r06s15_m${m}_$i.json" "sides_min=$m round $i"
  done
done
