#!/bin/bash
# Round 4 step 28: speculative start -- sweep s's test evaluation on a copy of U_s on the second
# stream while sweep s+1's start and user half run (tune bit 25 = off); the evaluation's train
# sum on its own scratch.  Sampler GPU tests, then A/B against HEAD (build_base) and bit 25.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_bias.py tests/test_gpu_collapse.py -x -q --timeout 300 --timeout-method thread > $O/r04s28_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s28_pytest.log; exit 1; }
tail -1 $O/r04s28_pytest.log
bash profiles/ab_args.sh r04s28 3 "base=build_base: new=build: b25=build:--tune,33554432" || { echo "ab failed"; exit 1; }
for f in $O/r04s28_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), c['test_rmse_after'])")"; done
echo s28 done
