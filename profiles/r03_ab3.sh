#!/bin/bash
# Round 3 probe 3: chip-wide f64 MFMA throughput; the double-buffered k_gres (tune bit 25) after its
# last-block vmcnt fix: parity and speed.
set -euo pipefail
timeout -k 10 120 tests/hip/mfma_f64_peak > gpurun_out/r03d_mfma_peak.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "variants" > gpurun_out/r03d_pytest.log 2>&1
bash profiles/ab_tune_libs.sh r03d "build:33554432 build:0"
echo ab3 done
