#!/bin/bash
# Round 3 (session 2) step 8: build_v13 = HEAD + libFM pass case loads issued before the sums (ids /
# residuals, then the partners' values and records) + the biased sampler's row kernels (k_bias_rows,
# k_rowsum2) with eight loads in flight per lane.  libFM, multi-rank and biased-sampler tests of v13,
# then the libFM / ALS and bias2 bench lines of v13 against the previous library (build).
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
SBMF_LIB=$B/build_v13/libsbmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_libfm.py tests/test_gpu_multirank.py \
  tests/test_gpu_bias.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s8_pytest.log 2>&1
echo pytest ok
for d in build_v13 build; do
  for m in libfm als; do
    SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 300 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu \
      > gpurun_out/r03s8_${d}_$m.json 2> gpurun_out/r03s8_${d}_$m.err
  done
  SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 \
    > gpurun_out/r03s8_${d}_bias2.json 2> gpurun_out/r03s8_${d}_bias2.err
done
echo s8 done
