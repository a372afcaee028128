#!/bin/bash
# Round 4 step 35: host waits spinning (SBMF_SPIN=1, hipDeviceScheduleSpin) against the default,
# 3 interleaved rounds on one box.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s35 3 "def=build: spin=build:env:SBMF_SPIN=1" || { echo "ab failed"; exit 1; }
for f in $O/r04s35_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), c['test_rmse_after'])")"; done
echo s35 done
