#!/bin/bash
# r06 step 2: per-XCD k_gres task queues.  (1) where workgroups land (HW_REG_XCC_ID probe);
# (2) the whole GPU suite on the new default; (3) A/B against the single queue (tune bit 16),
# 3 interleaved rounds of the default bench line (no CPU / f32 / time-to-RMSE legs).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 60 tests/hip/xcc_probe | tee "$O/r06s2_xcc_probe.txt"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
    > "$O/r06s2_suite.log" 2>&1 || { tail -40 "$O/r06s2_suite.log"; exit 1; }
tail -2 "$O/r06s2_suite.log"
for i in 1 2 3; do
  for t in 0 65536; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t \
      > "$O/r06s2_ab_t${t}_$i.json" 2> "$O/r06s2_ab_t${t}_$i.err"
    python3 -c "
import json; d=json.load(open('$O/r06s2_ab_t${t}_$i.json')); c=d['config']
print('t=$t round $i', round(d['ms_per_step'],3), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'stage', round(d['roofline']['ms_per_launch'],3), d['roofline']['frac'])"
  done
done
# the full default bench line (CPU baselines, f32, time-to-RMSE, loads, standalone bins)
bash profiles/collect.sh r06s2 bench
python3 -c "
import json; d=json.load(open('$O/r06s2_bench.json')); c=d['config']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), d['roofline']['frac'], d['cpu_baseline']['value'], d['f32_ms_per_step'])"
