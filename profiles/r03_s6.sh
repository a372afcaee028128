#!/bin/bash
# Round 3 (session 2) step 6 (build = HEAD + both changes, build_prev = HEAD):
#  - k_test with the ids and row slices of two ratings loaded before the first product;
#  - libFM's MCMC / ALS chain with the residuals kept in both orders and updated in place (one
#    rank; the other side's last pass applied on read from per-attribute records).
# Parity (sampler, production shapes, libFM chains, multi-rank), then bench A/B: the default
# sampler line and the libFM / ALS lines.
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_libfm.py \
  tests/test_gpu_multirank.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s6_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s6 "build:0 build_prev:0"
for d in build build_prev; do
  for m in libfm als; do
    SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 300 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu \
      > gpurun_out/r03s6_${d}_$m.json 2> gpurun_out/r03s6_${d}_$m.err
  done
done
echo s6 done
