#!/bin/bash
# r06 step 1: the libFM transpose input (.xt + .y) through the CLI as bin/libFM -method
# mcmc|als reads it, the rest of the CLI tests, the resource audit with the in-process
# RCCL self-test, and the round's first default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_cli.py tests/test_gpu_resources.py tests/test_gpu_rccl.py -s > "$O/r06s1_new.log" 2>&1 \
    || { tail -60 "$O/r06s1_new.log"; exit 1; }
grep -E "passed|failed|device usage|rccl self-test" "$O/r06s1_new.log" | tail -6
bash profiles/collect.sh r06s1 bench
python3 -c "
import json; d=json.load(open('$O/r06s1_bench.json')); c=d['config']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), d['roofline']['frac'], d['cpu_baseline']['value'], d['f32_ms_per_step'])"
