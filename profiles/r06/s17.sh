#!/bin/bash
# r06 step 17: sweeps queued a whole sweep ahead (sbmf_config.pipeline, unbiased sampler): each
# sweep starts with k_hyper_wait, which holds the stream until the host has published the sweep's
# draws in a pinned slot, and the row kernels read tau from the device; the timing events in two
# sets.  (1) the GPU suite; (2) A/B: this build with and without --no-pipeline against build_prev
# (the r06s14 build), ML-1M K=50 and ML-20M, 3 interleaved rounds; (3) the ML-1M timeline.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > "$O/r06s17_suite.log" 2>&1 || { tail -30 "$O/r06s17_suite.log"; exit 1; }
tail -2 "$O/r06s17_suite.log"
P=$R/scalable-bayesian-matrix-factorization_amd/build_prev/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'hyper', round(c['ms_hyper'],3), 'eval', round(c['ms_eval'],3))"; }
for i in 1 2 3; do
  for v in pipe nopipe prev; do
    L=$N; X=""; [ $v = prev ] && L=$P; [ $v = nopipe ] && X="--no-pipeline"
    SBMF_LIB=$L timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr \
      --no-f32 --no-load $X > "$O/r06s17_ml1m_${v}_$i.json" 2> "$O/r06s17_ml1m_${v}_$i.err"
    show "$O/r06s17_ml1m_${v}_$i.json" "ml1m $v round $i"
    SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load $X \
      > "$O/r06s17_ml20m_${v}_$i.json" 2> "$O/r06s17_ml20m_${v}_$i.err"
    show "$O/r06s17_ml20m_${v}_$i.json" "ml20m $v round $i"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d "$O/r06s17_ml1m_trace" -o r06s17 -- python3 "$R/bench.py" --shape ml-1m --K 50 --steps 20 --warmup 3 \
  --no-cpu --no-ttr --no-f32 --no-load > "$O/r06s17_ml1m_trace.log" 2>&1
python3 "$R/profiles/r06/timeline.py" "$O/r06s17_ml1m_trace" 3 > "$O/r06s17_ml1m_timeline.txt"
tail -1 "$O/r06s17_ml1m_timeline.txt"
