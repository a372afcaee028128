#!/bin/bash
# r06 step 6: the long-row streaming set alone first, every other launch of the half after it
# (SBMF_LONG_FIRST 1 = user half, 2 = item half, 3 = both) against the default (everything side by
# side), 3 interleaved rounds of the default ML-20M line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']; b=d['roofline']['bins']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3))"; }
for i in 1 2 3; do
  for lf in 0 1 2 3; do
    SBMF_LONG_FIRST=$lf timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s6_lf${lf}_$i.json" 2> "$O/r06s6_lf${lf}_$i.err"
    show "$O/r06s6_lf${lf}_$i.json" "long_first=$lf round $i"
  done
done
