#!/bin/bash
# Round 4 step 20: with two stream sets (the item half), the Gram-block launches on the second
# stream ahead of set 0 instead of behind it (tune bit 31, experiment): parity of the variant,
# then A/B 3 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_production.py -x -q --timeout 250 --timeout-method thread -k "philox or bench_workload" > $O/r04s20_pytest.log 2>&1 || { echo "pytest rc $?"; tail -20 $O/r04s20_pytest.log; exit 1; }
tail -1 $O/r04s20_pytest.log
bash profiles/ab_args.sh r04s20 3 "def=build: gfirst=build:--tune,2147483648" || { echo "ab failed"; exit 1; }
for f in $O/r04s20_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), c['test_rmse_after'])")"; done
echo s20 done
