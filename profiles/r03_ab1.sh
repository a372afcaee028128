#!/bin/bash
# Round 3 A/B 1: residual-slot swizzle (build vs build_noswz) x tune bits {0, 28 (setprio on the block's
# critical path), 0 (replicated solve), 0|28}; then the GPU suite.  Outputs gpurun_out/r03b_*.
set -euo pipefail
bash profiles/ab_tune_libs.sh r03b "build:0 build_noswz:0 build:268435456 build_noswz:268435456 build:1 build:268435457"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1
echo ab1 done
