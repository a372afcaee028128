#!/bin/bash
# Round 3 (session 2) step 5: Gram-block row setup with unconditional, grouped id / residual loads
# (build) against the previous HEAD (build_prev); parity of the kernel variants and production shapes.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_multirank.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03s5_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s5 "build:0 build_prev:0"
echo s5 done
