#!/bin/bash
# Round 4 step 12: stream threshold 128 / 192 against the default 256 (rows above it leave the
# Gram-block bins for k_gres), 4 interleaved rounds on one box.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s12 4 "def=build: thr192=build:--stream-threshold,192 thr128=build:--stream-threshold,128" || { echo "ab failed"; exit 1; }
for f in $O/r04s12_*_[1234].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))")"; done
echo s12 done
