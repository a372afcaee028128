#!/bin/bash
# Round 3 A/B 4: k_gres block epilogue without per-block geometry / branches / spill reloads (build)
# vs the round's starting kernel (build_noswz); parity of the kernel variants and the production shapes.
set -euo pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1
bash profiles/ab_tune_libs.sh r03e "build:0 build_noswz:0"
echo ab4 done
