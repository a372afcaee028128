#!/bin/bash
# Round 4 step 3: A/B of k_gres with LDS-only task barriers (build) against the previous HEAD
# (build_base); the parity suite on the new kernels; throughput lines for BASELINE configs 2-4
# on one GPU (ML-1M K=50, ML-10M K=100, ML-20M K=200; roofline + CPU baseline each); config 3's
# rocprofv3 kernel trace and FETCH / WRITE passes (ML-10M K=100); a kept per-dispatch kernel
# trace of the default ML-20M K=100 line.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_tune_libs.sh r04s3 "build_base:0 build:0" || { echo "ab failed"; exit 1; }
echo ab ok
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_bias.py -x -q \
  --timeout 500 --timeout-method thread > $O/r04s3_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s3_pytest.log; exit 1; }
tail -1 $O/r04s3_pytest.log
for c in "ml-1m 50" "ml-10m 100" "ml-20m 200"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --shape $1 --K $2 --no-ttr --no-load --no-f32 > $O/r04s3_bench_$1_k$2.json 2> $O/r04s3_bench_$1_k$2.err \
    || { echo "bench $1 $2 rc $?"; tail -5 $O/r04s3_bench_$1_k$2.err; exit 1; }
  echo "bench $1 K=$2 ok"
done
for p in trace fetch write; do
  BENCH_ARGS="--shape ml-10m --K 100" bash profiles/collect.sh r04s3_ml10m $p || { echo "collect $p failed"; exit 1; }
done
bash profiles/collect.sh r04s3_ml20m trace || { echo "collect trace failed"; exit 1; }
echo s3 done
