#!/bin/bash
# r06 step 10: ML-1M K=50 (config 2) per-sweep timeline on the event-merged build: kernels, memory
# copies and the HIP API calls of 20 timed sweeps (no counters), for the sweep-boundary gap.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d "$O/r06s10_ml1m_trace" -o r06s10 -- python3 "$R/bench.py" --shape ml-1m --K 50 --steps 20 --warmup 3 \
  --no-cpu --no-ttr --no-f32 --no-load > "$O/r06s10_ml1m_trace.log" 2>&1
find "$O/r06s10_ml1m_trace" -name "*.csv" | head -20
tail -3 "$O/r06s10_ml1m_trace.log"
