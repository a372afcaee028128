#!/bin/bash
# r05 step 1b: the rest of the GPU suite after r05s1 stopped at the in-process RCCL test
# (now a fresh worker process), then the serial schedule (tune bit 29, k_gres an ordinary
# launch) under rocprofv3 --kernel-trace --stats with no exit guard, and the default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_rccl.py tests/test_gpu_statistical.py tests/test_gpu_vbo.py > "$O/r05s1b_rest.log" 2>&1 \
    || { tail -40 "$O/r05s1b_rest.log"; exit 1; }
grep -E "passed|failed|rccl self-test" "$O/r05s1b_rest.log" || true
BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r05s1_serial trace
tail -3 "$O/r05s1_serial_trace.log"
bash profiles/collect.sh r05s1 bench
cat "$O/r05s1_bench.json"
