#!/bin/bash
# r05 step 1: the libFM drop-in CLI tests (no -item_offset), the parity suite's launch
# variants (k_gres ordinary launch in every schedule), then the serial schedule (tune bit 29,
# formerly cooperative) under rocprofv3 --kernel-trace --stats with no exit guard.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_cli.py tests/test_gpu_rccl.py tests/test_gpu_parity.py > "$O/r05s1_pytest.log" 2>&1
tail -3 "$O/r05s1_pytest.log" || true
BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r05s1_serial trace
echo "trace exit rc=$?"
tail -5 "$O/r05s1_serial_trace.log"
bash profiles/collect.sh r05s1 bench
cat "$O/r05s1_bench.json"
