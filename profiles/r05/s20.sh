#!/bin/bash
# r05 step 20: k_grow with its row's sigma and mu in LDS when Kp <= 128 (KL = 128 instance),
# instead of an L2 load in front of every block's draws; tune bit 12 keeps the KL = 256 form
# (sigma, mu from memory): parity subset, bench A/B, 3 interleaved rounds; K=50 line too.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_cli.py > "$O/r05s20_parity.log" 2>&1 \
    || { tail -30 "$O/r05s20_parity.log"; exit 1; }
tail -1 "$O/r05s20_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2 3; do for t in 4096 0; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s20_ab_t${t}_$i.json" 2> "$O/r05s20_ab_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s20_ab_t${t}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('tune $t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'w16', b['user_gblock_w16']['ms'], 'b4', b['user_gblock_b4']['ms'], 'b8', b['user_gblock_b8']['ms'])"
done; done
for t in 4096 0; do
  timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s20_k50_t${t}.json" 2> "$O/r05s20_k50_t${t}.err"
  python3 -c "
import json; d=json.load(open('$O/r05s20_k50_t${t}.json')); c=d['config']; print('K50 tune $t', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done
