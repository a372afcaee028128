#!/bin/bash
# r05 step 43: config 2 (ML-1M K=50) under the schedule bits -- default overlap against the serial
# schedule (bit 29), one side stream (bit 25) and the two item streaming sets in turn (bit 30):
# does the cross-stream hand-off cost more than the overlap gains at this size? 3 interleaved rounds.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
A=--shape,ml-1m,--K,50
bash profiles/ab_args.sh r05s43 3 "t0=build:$A t29=build:$A,--tune,536870912 t25=build:$A,--tune,33554432 t30=build:$A,--tune,1073741824"
for f in gpurun_out/r05s43_*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['config']; print('$f'.split('/')[-1], round(d['ms_per_step'],4), round(c['ms_user_half'],4), round(c['ms_item_half'],4))"; done
