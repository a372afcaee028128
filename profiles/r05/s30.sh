#!/bin/bash
# r05 step 30: pipelined sweep boundary (sbmf_config.pipeline: sweep s+1's user half queued
# before the host waits for sweep s and runs the callback): GPU parity (incl. the pipelined-chain
# test, the CLI, the biased sampler, multi-rank), bench A/B against --no-pipeline (3 rounds), and
# the default trace.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_cli.py tests/test_gpu_bias.py tests/test_gpu_multirank.py > "$O/r05s30_parity.log" 2>&1 \
    || { tail -30 "$O/r05s30_parity.log"; exit 1; }
tail -1 "$O/r05s30_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2 3; do for t in nopipe pipe; do
  A=""; [ $t = nopipe ] && A="--no-pipeline"
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load $A > "$O/r05s30_ab_${t}_$i.json" 2> "$O/r05s30_ab_${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s30_ab_${t}_$i.json')); c=d['config']; print('$t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done; done
bash profiles/collect.sh r05s30 trace
echo trace done
