#!/bin/bash
# Round-3 first probe on a 1-GPU box: streaming-kernel phase profile (KPROF build, both item launches),
# a short default bench line, then the GPU test suite.  Outputs: gpurun_out/r03a_*.
set -euo pipefail
B=scalable-bayesian-matrix-factorization_amd
O=gpurun_out; mkdir -p $O
SHORT="--no-cpu --no-ttr --no-f32"
for set in 0 1; do
  SBMF_LIB=$PWD/$B/build_kprof/libsbmf.so SBMF_KPROF=1 SBMF_KPROF_SET=$set timeout -k 10 150 \
    python3 bench.py --steps 3 --warmup 1 $SHORT > $O/r03a_kprof$set.json 2> $O/r03a_kprof$set.err
done
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 $SHORT > $O/r03a_bench.json 2> $O/r03a_bench.err
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/r03a_pytest.log 2>&1
echo probe done
