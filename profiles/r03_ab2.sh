#!/bin/bash
# Round 3 A/B 2: LDS-only barriers in k_gres's block epilogue (build) vs the previous build (build_noswz),
# default kernel and the double-buffered one (tune bit 25); kernel-variant parity; the collapse pin.
set -euo pipefail
bash profiles/ab_tune_libs.sh r03c "build:0 build_noswz:0 build:33554432 build_noswz:33554432"
SBMF_LIB=$PWD/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so timeout -k 10 150 python3 bench.py --steps 5 --warmup 1 --no-cpu --no-ttr --no-f32 --gram-threshold 1024 > gpurun_out/r03c_gram1024.json 2> gpurun_out/r03c_gram1024.err
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_collapse.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r03c_pytest.log 2>&1
echo ab2 done
