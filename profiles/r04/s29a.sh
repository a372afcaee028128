#!/bin/bash
# Round 4 final pass (after the sweep-boundary and libFM host-sum changes), part A: the whole GPU suite on the final kernels, then the default bench.py
# line (f64 + f32 + CPU baselines + time-to-RMSE + load / prepare).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=30 \
  > $O/r04g_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04g_pytest.log; exit 1; }
tail -1 $O/r04g_pytest.log
bash profiles/collect.sh r04g bench || { echo "bench failed"; tail -20 $O/r04g_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/r04g_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['config']['ms_user_half'], d['config']['ms_item_half'])"
echo s29a done
