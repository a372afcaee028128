#!/bin/bash
# Round 4 step 13: clean attribution on the production build flags (timing only, wrong results):
# each build removes ONE component from k_gblock and k_gres -- the MFMAs (SBMF_ABL_NOMFMA), the
# butterfly residual update (SBMF_ABL_NOBFLY), the 16-step recurrence (SBMF_ABL_NOSOLVE), the
# gathers' memory cost (SBMF_ABL_GATHER0: every slice from partner row 0) -- 2 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s13 2 "def=build: nomfma=build_nomfma: nobfly=build_nobfly: nosolve=build_nosolve: g0=build_g0:" || { echo "ab failed"; exit 1; }
for f in $O/r04s13_*_[12].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items()})")"; done
echo s13 done
