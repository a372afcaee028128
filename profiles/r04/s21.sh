#!/bin/bash
# Round 4 step 21: two launch-order experiments, both bitwise-neutral by construction (disjoint
# writes): tune bit 31 = with two stream sets (the item half) the Gram-block launches on the
# second stream ahead of set 0; tune bit 28 = the test evaluation on the second stream beside the
# next sweep's prologue kernels (one rank).  A/B, 3 rounds; the test RMSE must not change.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
bash profiles/ab_args.sh r04s21 3 "def=build: gfirst=build:--tune,2147483648 pareval=build:--tune,268435456 both=build:--tune,2415919104" || { echo "ab failed"; exit 1; }
for f in $O/r04s21_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), round(c['ms_hyper'],3), c['test_rmse_after'])")"; done
echo s21 done
