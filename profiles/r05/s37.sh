#!/bin/bash
# r05 step 37: evidence on the final kernels (item streaming tasks in the 3/4 size class) -- the whole GPU suite, the default bench
# line (f64 + f32 + CPU baseline + time-to-RMSE + load), the default and serial (tune bit 29)
# per-dispatch traces.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
    > "$O/r05s37_suite.log" 2>&1 || { tail -30 "$O/r05s37_suite.log"; exit 1; }
tail -2 "$O/r05s37_suite.log"
bash profiles/collect.sh r05s37 bench
python3 -c "
import json; d=json.load(open('$O/r05s37_bench.json')); c=d['config']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), d['roofline']['frac'], d['cpu_baseline']['value'], d['f32_ms_per_step'])"
bash profiles/collect.sh r05s37 trace
BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r05s37_serial trace
echo traces done
