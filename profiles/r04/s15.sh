#!/bin/bash
# Round 4 step 15: user streaming rows above 512 / 1024 ratings as a second stream set on 8-wave
# workgroups (1024-rating tasks: half the chunks per split row), the rest on 4-wave ones
# (SBMF_X_USERSET, experiment), 3 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s15 3 "def=build: u512w8=build:env:SBMF_X_USERSET=512:8 u1024w8=build:env:SBMF_X_USERSET=1024:8" || { echo "ab failed"; exit 1; }
for f in $O/r04s15_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items() if k.startswith('user')})")"; done
echo s15 done
