#!/bin/bash
# Round 4 step 31: the test set on the device in user order (counting sort at prepare, file order restored in sbmf_predict), so the evaluation reads each user row from cache for its consecutive ratings.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_bias.py tests/test_gpu_collapse.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > $O/r04s31_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s31_pytest.log; exit 1; }
tail -1 $O/r04s31_pytest.log
bash profiles/ab_args.sh r04s31 3 "base=build_base: new=build:" || { echo "ab failed"; exit 1; }
for f in $O/r04s31_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), c['test_rmse_after'])")"; done
echo s31 done
