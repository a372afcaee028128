#!/bin/bash
# r05 step 42: rocprofv3 kernel trace of config 2 (ML-1M K=50) -- how much of the 0.45 ms sweep is
# device time and how much is launch / host gap.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/r05s42_ml1m" -o r05s42 -- \
  python3 "$R/bench.py" --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr --no-load --no-f32 > "$O/r05s42_ml1m_bench.json" 2> "$O/r05s42_ml1m.err"
ls "$O/r05s42_ml1m"
