#!/bin/bash
# Round 3 (session 2) step 7 (build = HEAD, build_v11 = HEAD + k_gres task staging by unconditional loads
# + VB v-pass case loads issued before the sums): parity of v11 (sampler, production shapes, VB), then
# the sampler A/B and the VB bench lines of both.
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
SBMF_LIB=$B/build_v11/libsbmf.so timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py \
  tests/test_gpu_vbo.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s7_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s7 "build:0 build_v11:0"
for d in build_v11 build; do
  SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 400 python3 bench.py --method vb --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/r03s7_${d}_vb.json 2> gpurun_out/r03s7_${d}_vb.err
done
echo s7 done
