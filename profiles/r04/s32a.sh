#!/bin/bash
# Round 4 final pass (after the counter-clear, kind-event and test-order changes), part A: the whole GPU suite on the final kernels, then the default bench.py
# line (f64 + f32 + CPU baselines + time-to-RMSE + load / prepare).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=30 \
  > $O/r04h_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04h_pytest.log; exit 1; }
tail -1 $O/r04h_pytest.log
bash profiles/collect.sh r04h bench || { echo "bench failed"; tail -20 $O/r04h_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/r04h_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['config']['ms_user_half'], d['config']['ms_item_half'])"
echo s32a done
