#!/bin/bash
# r06 step 3: the whole GPU suite (per-XCD queues, RCCL by path, sweep graph), then 3 interleaved
# rounds of the default bench line: per-XCD queues vs one queue (tune bit 16), eager vs graph
# (SBMF_GRAPH=0), and config 2 (ML-1M K=50) eager vs graph; then the full default bench line.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
    > "$O/r06s3_suite.log" 2>&1 || { tail -40 "$O/r06s3_suite.log"; exit 1; }
tail -2 "$O/r06s3_suite.log"
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],3), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'stage', round(d['roofline']['ms_per_launch'],3), round(d['roofline']['frac'],4))"; }
for i in 1 2 3; do
  for v in "0 1" "65536 1" "0 0"; do
    set -- $v
    SBMF_GRAPH=$2 timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $1 \
      > "$O/r06s3_ab_t$1_g$2_$i.json" 2> "$O/r06s3_ab_t$1_g$2_$i.err"
    show "$O/r06s3_ab_t$1_g$2_$i.json" "ml20m t=$1 graph=$2 round $i"
  done
  for g in 1 0; do
    SBMF_GRAPH=$g timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s3_ml1m_g${g}_$i.json" 2> "$O/r06s3_ml1m_g${g}_$i.err"
    show "$O/r06s3_ml1m_g${g}_$i.json" "ml1m graph=$g round $i"
  done
done
bash profiles/collect.sh r06s3 bench
show "$O/r06s3_bench.json" "default line"
