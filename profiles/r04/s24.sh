#!/bin/bash
# Round 4 step 24: the item half's Gram-block launches on a third stream beside both streaming
# sets (tune bit 31 = round-3 placement behind set 0); experiment tune bit 25: the user half's
# one-wave Gram-block kinds on the compute stream after the streaming launch.  Parity of the
# variants, then A/B 3 rounds (the test RMSE must not change).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q --timeout 300 --timeout-method thread > $O/r04s24_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s24_pytest.log; exit 1; }
tail -1 $O/r04s24_pytest.log
bash profiles/ab_args.sh r04s24 3 "def=build: b31=build:--tune,2147483648 late=build:--tune,33554432" || { echo "ab failed"; exit 1; }
for f in $O/r04s24_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), c['test_rmse_after'])")"; done
echo s24 done
