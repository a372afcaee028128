#!/bin/bash
# r05 step 1: the new GPU tests (libFM drop-in CLI on the reference's own files, RCCL
# loopback self-test, virtual ranks, Philox-vs-reference statistics), the whole GPU suite,
# then the serial schedule (tune bit 29; k_gres now an ordinary launch there too) under
# rocprofv3 --kernel-trace --stats with no exit guard, and the default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_cli.py tests/test_gpu_rccl.py tests/test_gpu_statistical.py -s > "$O/r05s1_new.log" 2>&1 \
    || { tail -40 "$O/r05s1_new.log"; exit 1; }
grep -E "passed|failed|rccl self-test|sweep (10|20)" "$O/r05s1_new.log" || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
    > "$O/r05s1_suite.log" 2>&1 || { tail -30 "$O/r05s1_suite.log"; exit 1; }
tail -2 "$O/r05s1_suite.log"
BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r05s1_serial trace
tail -3 "$O/r05s1_serial_trace.log"
bash profiles/collect.sh r05s1 bench
cat "$O/r05s1_bench.json"
