#!/bin/bash
# Round 4 step 1: the pruned kernels (k_gstream, k_rows, Gram route and tune variants removed),
# the threaded loaders and the new bench fields: bench line, then the GPU suite minus the
# multi-rank config-4 cases (run in step 2).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/r04s1_bench.json 2> $O/r04s1_bench.err || { echo "bench rc $?"; tail -20 $O/r04s1_bench.err; exit 1; }
echo bench ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 \
  -k "not config4" > $O/r04s1_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s1_pytest.log; exit 1; }
tail -3 $O/r04s1_pytest.log
