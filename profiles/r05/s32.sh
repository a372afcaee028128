#!/bin/bash
# r05 step 32: the halves' two streaming sets one after the other (tune bit 30: set 0 -- item rows
# of 257..1024 ratings, user rows of 257..512 -- then set 1, the Gram-block kinds beside them)
# against side by side (default), 3 interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2 3; do for t in 0 1073741824; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s32_ab_t${t}_$i.json" 2> "$O/r05s32_ab_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s32_ab_t${t}_$i.json')); c=d['config']; print('tune $t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done; done
