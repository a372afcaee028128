#!/bin/bash
# Round 3 (session 2) step 9: online VB user v-pass item records loaded two at a time before use
# (build_v14) against HEAD (build): VB tests, then two VB bench lines each.
set -euo pipefail
mkdir -p gpurun_out
B=$PWD/scalable-bayesian-matrix-factorization_amd
SBMF_LIB=$B/build_v14/libsbmf.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_vbo.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r03s9_pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  for d in build_v14 build; do
    SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 400 python3 bench.py --method vb --steps 5 --warmup 2 --no-cpu \
      > gpurun_out/r03s9_${d}_vb_$i.json 2> gpurun_out/r03s9_${d}_vb_$i.err
  done
done
echo s9 done
