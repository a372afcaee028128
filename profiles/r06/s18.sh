#!/bin/bash
# r06 step 18: beside the two streaming sets (ML-20M), the half's last Gram-block kind on the compute
# stream behind stream set 1 (SBMF_LAST_KIND_ON_ST 1 = users, 3 = both) instead of at the end of the
# side stream's chain (the r06s14 trace: the user half ends with that chain, 0.5 ms after set 0).
# 3 interleaved rounds of the default line against 0.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3))"; }
for i in 1 2 3; do
  for v in 0 1 3; do
    SBMF_LAST_KIND_ON_ST=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s18_v${v}_$i.json" 2> "$O/r06s18_v${v}_$i.err"
    show "$O/r06s18_v${v}_$i.json" "last_kind_on_st=$v round $i"
  done
done
