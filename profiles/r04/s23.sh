#!/bin/bash
# Round 4 step 23: the sweep boundary without host round trips on the device's path: the next
# sweep's hyperparameters uploaded (pinned) and its normals filled at the end of this sweep,
# results / timeout flag read through pinned memory, one timing event per launch boundary.
# GPU tests of the sampler (one and several ranks, bias, production), then A/B against HEAD.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_bias.py tests/test_gpu_production.py tests/test_gpu_collapse.py -x -q --timeout 300 --timeout-method thread > $O/r04s23_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s23_pytest.log; exit 1; }
tail -1 $O/r04s23_pytest.log
bash profiles/ab_args.sh r04s23 3 "base=build_base: new=build:" || { echo "ab failed"; exit 1; }
for f in $O/r04s23_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), round(c['ms_hyper'],3), c['test_rmse_after'])")"; done
echo s23 done
