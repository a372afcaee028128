#!/bin/bash
# r05 step 27: f64 user rows above 512 ratings as a second streaming set (tune bit 13: 8-wave
# workgroups, 1024-rating tasks; bit 14: 16-wave, 2048) beside the 4-wave set: the r05s26 phase
# profile puts the 4-wave set's split-row chunks 63 % in the hand-off phase.  Variant parity,
# bench A/B (3 rounds), and the phase profile of the 16-wave user set.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "variants" > "$O/r05s27_parity.log" 2>&1 \
    || { tail -30 "$O/r05s27_parity.log"; exit 1; }
tail -1 "$O/r05s27_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2 3; do for t in 0 8192 16384; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s27_ab_t${t}_$i.json" 2> "$O/r05s27_ab_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s27_ab_t${t}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('tune $t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'ustream', b['user_gres_stage']['ms'])"
done; done
