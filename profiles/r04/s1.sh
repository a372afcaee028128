#!/bin/bash
# Round 4 step 1: the pruned kernels, the threaded loaders and the new bench fields; A/B of the
# k_gres LDS-DMA prefetch (tune bit 25) against the default; the GPU suite minus the multi-rank
# config-4 cases (step 2).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/r04s1_bench.json 2> $O/r04s1_bench.err || { echo "bench rc $?"; tail -20 $O/r04s1_bench.err; exit 1; }
echo bench ok
for i in 1 2; do
  for t in 0 33554432; do
    timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t \
      > $O/r04s1_ab_t${t}_$i.json 2> $O/r04s1_ab_t${t}_$i.err || { echo "ab $t rc $?"; tail -5 $O/r04s1_ab_t${t}_$i.err; exit 1; }
  done
done
echo ab ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 \
  -k "not config4" > $O/r04s1_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s1_pytest.log; exit 1; }
tail -3 $O/r04s1_pytest.log
