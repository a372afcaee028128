#!/bin/bash
# r05 step 41: streaming task size capped at 1536 / 1280 ratings (only the 16-wave item set's 2048-rating
# tasks shrink; the 3/4 size class makes 1536 a full-speed shape) against the default, 3 interleaved rounds.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
bash profiles/ab_args.sh r05s41 3 "t0=build: c1536=build:--split-chunk,1536 c1280=build:--split-chunk,1280"
for f in gpurun_out/r05s41_*.json; do python3 -c "
import json; d=json.load(open('$f')); c=d['config']; print('$f'.split('/')[-1], round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"; done
