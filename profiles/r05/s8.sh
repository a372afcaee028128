#!/bin/bash
# r05 step 8: fewer persistent k_gres workgroups per CU on the user side (4 -> 3 -> 2), so the
# user Gram-block kinds get CU slots beside the streaming launch from its start; 2 rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2; do for u in 4 3 2; do
  SBMF_GRES_PER_CU_U=$u timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > "$O/r05s8_u${u}_$i.json" 2> "$O/r05s8_u${u}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s8_u${u}_$i.json')); c=d['config']; print('user WG/CU $u round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done; done
for i in 1; do
  SBMF_GRES_PER_CU_I=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > "$O/r05s8_i1_$i.json" 2> "$O/r05s8_i1_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s8_i1_$i.json')); c=d['config']; print('item WG/CU 1 round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done
