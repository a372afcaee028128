#!/bin/bash
# r06 step 20: the committed tree end to end after the VB timing change (sbmf_timing grew a field):
# smoke(), the sampler parity and production tests, and the full default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/r06s20_smoke.txt" 2>&1
tail -1 "$O/r06s20_smoke.txt"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_abi.py -x -q \
  --timeout 600 --timeout-method thread > "$O/r06s20_tests.log" 2>&1 || { tail -30 "$O/r06s20_tests.log"; exit 1; }
tail -1 "$O/r06s20_tests.log"
bash profiles/collect.sh r06s20 bench
python3 -c "
import json; d=json.load(open('$O/r06s20_bench.json')); c=d['config']; r=d['roofline']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), r['frac'], r['traffic'], r['traffic_source'], d['cpu_baseline']['value'], d['f32_ms_per_step'])"
