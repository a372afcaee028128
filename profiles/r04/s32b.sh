#!/bin/bash
# Round 4 final pass (after the counter-clear, kind-event and test-order changes), part B:
# rocprofv3 kernel trace + FETCH / WRITE / LDS passes of the default line, BASELINE configs 2-4,
# the biased sampler.  (Online VB and libFM MCMC / ALS are unchanged since r04g.)
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for p in trace fetch write lds; do
  bash profiles/collect.sh r04h_ml20m $p || { echo "collect $p failed"; exit 1; }
done
for c in "ml-1m 50" "ml-10m 100" "ml-20m 200"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --shape $1 --K $2 --no-ttr --no-load --no-f32 > $O/r04h_bench_$1_k$2.json 2> $O/r04h_bench_$1_k$2.err \
    || { echo "bench $1 $2 rc $?"; tail -5 $O/r04h_bench_$1_k$2.err; exit 1; }
  echo "bench $1 K=$2 ok"
done
timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-ttr --no-load --no-f32 --no-cpu > $O/r04h_bench_bias2.json 2> $O/r04h_bench_bias2.err || { echo "bias2 rc $?"; exit 1; }
echo s32b done
