#!/bin/bash
# VB XCD slices by case count: SBMF_VB_SLICES = 1 (default), 8, 4; Netflix K=200 GPU ms per epoch.
# Outputs gpurun_out/r03r_*.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
VB="python3 $R/bench.py --method vb --no-cpu --steps 1 --warmup 1"
: > $O/r03r_summary.txt
for x in 1 8 4; do
  SBMF_VB_SLICES=$x timeout -k 10 300 $VB > $O/r03r_s$x.json 2> $O/r03r_s$x.err || { echo "s$x rc $?"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r03r_s$x.json').read().strip().splitlines()[-1]); print('slices $x', round(d['config']['gpu_ms_per_epoch'],1), 'ms/epoch', d['config']['test_rmse_after'])" | tee -a $O/r03r_summary.txt
done
SBMF_VB_SLICES=8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_vbo.py -x -q --timeout 500 --timeout-method thread > $O/r03r_pytest8.log 2>&1 || { echo "pytest8 rc $?"; exit 1; }
echo vbsl done
