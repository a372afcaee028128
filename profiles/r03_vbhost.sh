#!/bin/bash
# VB after the host-layout rework: the VB parity tests, then the host side per epoch (SBMF_VB_TRACE=1:
# layout phases on the worker thread, the main thread's wait, the layout upload), Netflix K=200,
# 2 timed epochs.  Outputs gpurun_out/${TAG}_*.
set -uo pipefail
TAG=${TAG:-r03t}
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_vbo.py tests/test_gpu_multirank.py -k "vb" -x -v --timeout 600 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/${TAG}_pytest.log; exit 1; }
SBMF_VB_TRACE=1 timeout -k 10 400 python3 bench.py --method vb --no-cpu --steps 2 --warmup 1 > $O/${TAG}_vb.json 2> $O/${TAG}_vb.err || { echo "rc $?"; exit 1; }
grep -h "vbo\|bench vb" $O/${TAG}_vb.err
python3 -c "import json; d=json.loads(open('$O/${TAG}_vb.json').read().strip().splitlines()[-1]); print('value', d['value'], 'wall ms/epoch', d['ms_per_step'], 'gpu ms/epoch', d['config']['gpu_ms_per_epoch'])"
