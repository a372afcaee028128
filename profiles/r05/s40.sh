#!/bin/bash
# r05 step 40: stream threshold 128 / 192 against the default (256, = gkmax) on the final kernels
# (k_grow now serves the 9-256-rating rows; round 4's r04s12 found 128 / 192 within noise), 3 interleaved rounds.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
bash profiles/ab_args.sh r05s40 3 "t0=build: thr128=build:--stream-threshold,128 thr192=build:--stream-threshold,192"
for f in gpurun_out/r05s40_*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['config']; print('$f'.split('/')[-1], round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"; done
