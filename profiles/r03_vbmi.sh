#!/bin/bash
# VB item-row cases per lane (4 / 8 default / 16), Netflix K=200 GPU ms per epoch, after the VB tests.
# Outputs gpurun_out/r03q_*.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
B=$R/scalable-bayesian-matrix-factorization_amd
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_vbo.py tests/test_gpu_multirank.py -k "vb" -x -v --timeout 600 --timeout-method thread > $O/r03q_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r03q_pytest.log; exit 1; }
VB="python3 $R/bench.py --method vb --no-cpu --steps 1 --warmup 1"
: > $O/r03q_summary.txt
for v in default:build mi4:build_mi4 mi16:build_mi16; do
  t=${v%%:*}; d=${v#*:}
  SBMF_LIB=$B/$d/libsbmf.so timeout -k 10 300 $VB > $O/r03q_$t.json 2> $O/r03q_$t.err || { echo "$t rc $?"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r03q_$t.json').read().strip().splitlines()[-1]); print('$t', round(d['config']['gpu_ms_per_epoch'],1), 'ms/epoch', d['config']['test_rmse_after'])" | tee -a $O/r03q_summary.txt
done
echo vbmi done
