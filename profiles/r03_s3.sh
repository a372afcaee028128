#!/bin/bash
# Round 3 (session 2) step 3: candidate kernel changes against the committed HEAD (build):
#   build_v1 + tune bit 28   solving wave of multi-wave Gram-block rows at raised priority
#   build_v2                 two-step block solve (SBMF_SOLVE2: one readlane hop per pair of draws)
#   build_v3                 raw buffer gathers in k_gres / k_gblock (SBMF_GRES_BUF)
#   build_v4                 k_gres accumulates vectors in gather-issue order (SBMF_GRES_ORD)
#   build_v5                 v3 + v4
#   build_v6 / build_v7      v4 + L2 prefetch of the next block's first-gathered 8 / 16 vectors per wave
#                            during a block's exchange and draws (SBMF_GRES_PF)
#   build_v8 / build_v9 + tune bit 31   v4 + long item rows on the wide-register 8-wave k_gres
#                            (96 / 80 vectors per wave at two waves per SIMD: 3072 / 2560-rating tasks)
# Two A/B rounds first, then parity of v8 (wide variant: ML-1M and ML-20M against the oracle) and v6.
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
bash profiles/ab_tune_libs.sh r03s3 "build:0 build_v2:0 build_v4:0 build_v5:0 build_v6:0 build_v8:2147483648 build_v9:2147483648"
echo ab done
SBMF_LIB=$B/build_v8/libsbmf.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_production.py -x -q \
  -k "wide or bench_workload" --timeout 450 --timeout-method thread > gpurun_out/r03s3_pytest_v8.log 2>&1
echo pytest v8 ok
SBMF_LIB=$B/build_v6/libsbmf.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q \
  --timeout 250 --timeout-method thread > gpurun_out/r03s3_pytest_v6.log 2>&1
echo s3 done
