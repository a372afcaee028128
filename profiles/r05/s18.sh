#!/bin/bash
# r05 step 18: f32 rows of 17..512 ratings on k_grow (tune bit 11): f32 parity, f32 bench A/B
# (2 rounds); then the PMC passes of the default f64 line (FETCH / WRITE / LDS).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "f32" tests/test_gpu_production.py > "$O/r05s18_parity.log" 2>&1 \
    || { tail -30 "$O/r05s18_parity.log"; exit 1; }
tail -1 "$O/r05s18_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2; do for t in 0 2048; do
  timeout -k 10 200 python3 bench.py --precision f32 --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s18_f32_t${t}_$i.json" 2> "$O/r05s18_f32_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s18_f32_t${t}_$i.json')); c=d['config']; print('f32 tune $t round $i', d['dtype'], round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done; done
bash profiles/collect.sh r05s18 fetch && bash profiles/collect.sh r05s18 write && bash profiles/collect.sh r05s18 lds
ls "$O"/r05s18_pmc_*
