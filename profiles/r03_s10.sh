#!/bin/bash
# Round 3 (session 2) step 10: the user side's streaming rows on 4-wave k_gres workgroups (tune bit 23,
# 512-rating tasks, four workgroups per CU) against the default 8-wave ones, same library (build_v15);
# the two lines' test RMSE after the same sweeps must agree (a consistency check, not the oracle).
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
bash profiles/ab_tune_libs.sh r03s10 "build_v15:0 build_v15:8388608"
echo s10 done
