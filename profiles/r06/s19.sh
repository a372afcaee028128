#!/bin/bash
# r06 step 19: online VB (config 5) with its dominant kernels timed: the factor passes (every
# mini-batch's 2K k_user_v / k_item_vp launches) with HIP events (sbmf_timing.ms_vb_factor), and
# their HBM traffic from FETCH_SIZE / WRITE_SIZE passes (profiles/pmc_vb.py).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_vbo.py tests/test_gpu_resources.py -x -q --timeout 400 \
  --timeout-method thread > "$O/r06s19_vb_tests.log" 2>&1 || { tail -30 "$O/r06s19_vb_tests.log"; exit 1; }
tail -1 "$O/r06s19_vb_tests.log"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 900 python3 "$R/bench.py" --method vb > "$O/r06s19_vb_bench.json" 2> "$O/r06s19_vb_bench.err"
python3 -c "
import json; d=json.load(open('$O/r06s19_vb_bench.json')); r=d['roofline']
print('vb', round(d['ms_per_step'],1), 'ms/epoch', d['value'], 'factor ms', round(r['ms_per_epoch'],1), 'frac', r['frac'], 'aggregate', r['epoch_aggregate']['frac'])"
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$O/r06s19_vb_pmc_fetch" -o r06s19 -- \
  python3 "$R/bench.py" --method vb --steps 1 --warmup 1 --no-cpu > "$O/r06s19_vb_pmc_fetch.log" 2>&1
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$O/r06s19_vb_pmc_write" -o r06s19 -- \
  python3 "$R/bench.py" --method vb --steps 1 --warmup 1 --no-cpu > "$O/r06s19_vb_pmc_write.log" 2>&1
python3 "$R/profiles/pmc_vb.py" "$O/r06s19_vb_pmc_fetch/r06s19_counter_collection.csv" \
  "$O/r06s19_vb_pmc_write/r06s19_counter_collection.csv" "$O/r06s19_pmc_vb_traffic.json" "r06s19"
