#!/bin/bash
# Round 4 step 11: is the sweep bound by gather latency?  A timing-only build (SBMF_ABL_GATHER0,
# wrong results) points every partner slice of k_gblock and k_gres at partner row 0 (an L2 hit)
# and keeps everything else; against the default build, 2 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s11 2 "def=build: g0=build_g0:" || { echo "ab failed"; exit 1; }
for f in $O/r04s11_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items()})")"; done
echo s11 done
