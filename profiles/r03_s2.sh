#!/bin/bash
# Round 3 (session 2) step 2: k_gres solve from a zero-upper image (diagonal kept apart, whole H rows
# read unmasked and pipelined).  Production parity, A/B against the session's starting kernel
# (build_base) with the replicated solve (tune bit 0) and all-8-wave items (bit 27), then the SQ
# instruction-mix pass (MFMA busy cycles) of the new build.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03s2_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s2 "build:0 build_base:0 build:1 build:134217728"
bash profiles/collect.sh r03s2 sq2
echo s2 done
