#!/bin/bash
# Round 4 step 10: Gram-block occupancy variants (build-time): 8-vector kinds at 6 waves/SIMD
# (80 VGPRs, spills 28-44 B), 16-vector kinds at 3 (142-168 VGPRs) or 5 (96, spills ~200 B)
# against the default (5 / 4), 2 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s10 2 "def=build: occ6=build_occ6: wide3=build_wide3: wide5=build_wide5:" || { echo "ab failed"; exit 1; }
for f in $O/r04s10_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items() if 'gblock' in k})")"; done
echo s10 done
