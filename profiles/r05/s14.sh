#!/bin/bash
# r05 step 14: evidence on the k_grow HEAD -- the whole GPU suite, the default bench line,
# the serial schedule's standalone per-launch trace (tune bit 29) and the default trace.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
    > "$O/r05s14_suite.log" 2>&1 || { tail -30 "$O/r05s14_suite.log"; exit 1; }
tail -2 "$O/r05s14_suite.log"
bash profiles/collect.sh r05s14 bench
python3 -c "
import json; d=json.load(open('$O/r05s14_bench.json')); c=d['config']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), d['roofline']['frac'], d['cpu_baseline']['value'])"
BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r05s14_serial trace
tail -2 "$O/r05s14_serial_trace.log"
bash profiles/collect.sh r05s14 trace
tail -2 "$O/r05s14_trace.log"
