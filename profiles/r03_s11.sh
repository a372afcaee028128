#!/bin/bash
# Round 3 (session 2) step 11: a half's Gram-block launches on a second stream beside its
# streaming launch (default) against the serial order (tune bit 29), same library; the GPU
# suite first (the overlap must not change any result).
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03s11_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s11 "build:0 build:536870912"
echo s11 done
