#!/bin/bash
# Round 3 (session 2) step 1: k_gres solve reads its H row before the serial chain.
# Parity of the kernel variants and production shapes, A/B against the session's
# starting kernel (build_base), then the phase profile (KPROF build) of both item sets.
set -euo pipefail
mkdir -p gpurun_out
B=scalable-bayesian-matrix-factorization_amd
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03s1_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s1 "build:0 build_base:0"
for set in 0 1; do
  SBMF_LIB=$PWD/$B/build_kprof/libsbmf.so SBMF_KPROF=1 SBMF_KPROF_SET=$set timeout -k 10 150 \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 > gpurun_out/r03s1_kprof$set.json 2> gpurun_out/r03s1_kprof$set.log
done
echo s1 done
