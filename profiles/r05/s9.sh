#!/bin/bash
# r05 step 9: k_test keeping the previous rating's user row (test ratings are in user order):
# parity subset, then bench A/B against SBMF_TEST_NOREUSE=1 (2 interleaved rounds).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_bias.py tests/test_gpu_production.py > "$O/r05s9_parity.log" 2>&1 \
    || { tail -30 "$O/r05s9_parity.log"; exit 1; }
tail -1 "$O/r05s9_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2; do for v in 0 1; do
  SBMF_TEST_NOREUSE=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > "$O/r05s9_ab_nr${v}_$i.json" 2> "$O/r05s9_ab_nr${v}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s9_ab_nr${v}_$i.json')); c=d['config']; print('noreuse=$v round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_hyper'],3), round(c['ms_eval'],3))"
done; done
