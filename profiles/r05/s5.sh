#!/bin/bash
# r05 step 5: tune bit 25 (Gram-block kinds on two side streams) -- parity of the variants,
# A/B of the single-GPU bench (3 interleaved rounds), and per-rank compute of the 8-way split
# with and without it (virtual ranks).  Also the sincos Box-Muller (parity via the Philox tests).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py > "$O/r05s5_parity.log" 2>&1 \
    || { tail -30 "$O/r05s5_parity.log"; exit 1; }
tail -1 "$O/r05s5_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2 3; do for t in 0 33554432; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s5_ab_t${t}_$i.json" 2> "$O/r05s5_ab_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s5_ab_t${t}_$i.json')); c=d['config']; print('ab t=$t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_hyper'],3), round(c['ms_eval'],3))"
done; done
cd /tmp && export TMPDIR=/tmp
for K in 100 200; do for t in 0 33554432; do
  SBMF_STAGES=4 timeout -k 10 300 python3 "$R/profiles/r05/rank_stages.py" --K $K --tune $t > "$O/r05s5_rank_k${K}_t${t}.json" 2> "$O/r05s5_rank_k${K}_t${t}.txt"
  python3 -c "
import json; d=json.load(open('$O/r05s5_rank_k${K}_t${t}.json')); print('K=$K tune=$t 4 stages: max user %.3f item %.3f max sweep %.3f' % (d['max_over_ranks']['user'], d['max_over_ranks']['item'], max(x['ms_sweep'] for x in d['per_rank'])))"
done; done
