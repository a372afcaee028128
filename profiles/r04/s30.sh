#!/bin/bash
# Round 4 step 30: the streaming stages' split-row counters cleared at the end of the previous stage (off the path), launch-kind events on the first sweep of a run only (the streaming kind every sweep); bench runs its K sweeps in one call.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_bias.py tests/test_gpu_collapse.py -x -q --timeout 300 --timeout-method thread > $O/r04s30_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s30_pytest.log; exit 1; }
tail -1 $O/r04s30_pytest.log
bash profiles/ab_args.sh r04s30 3 "base=build_base: new=build:" || { echo "ab failed"; exit 1; }
for f in $O/r04s30_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), c['test_rmse_after'])")"; done
echo s30 done
