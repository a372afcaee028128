#!/bin/bash
# VB host side per epoch (SBMF_VB_TRACE=1: layout phases on the worker thread, the main thread's wait,
# device allocation and layout upload), Netflix K=200, 3 epochs.  Outputs gpurun_out/r03t_*.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
SBMF_VB_TRACE=1 timeout -k 10 400 python3 bench.py --method vb --no-cpu --steps 2 --warmup 1 > $O/r03t_vb.json 2> $O/r03t_vb.err || { echo "rc $?"; exit 1; }
grep -h "vbo\|bench vb" $O/r03t_vb.err
python3 -c "import json; d=json.loads(open('$O/r03t_vb.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['gpu_ms_per_epoch'])"
nproc
