#!/bin/bash
# Round 3 (session 2) step 8: build_v12 = build_v11 + libFM pass case loads issued before the sums
# (ids / residuals, then the partners' values and records); libFM parity, CLI and multi-rank tests,
# then the libFM / ALS bench lines of v12 against HEAD (build).
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
SBMF_LIB=$B/build_v12/libsbmf.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_libfm.py tests/test_gpu_multirank.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s8_pytest.log 2>&1
echo pytest ok
for d in build_v12 build; do
  for m in libfm als; do
    SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 300 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu \
      > gpurun_out/r03s8_${d}_$m.json 2> gpurun_out/r03s8_${d}_$m.err
  done
done
echo s8 done
