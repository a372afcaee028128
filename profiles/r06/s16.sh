#!/bin/bash
# r06 step 16: the sweep's three small host transfers (prologue sums and results to pinned memory,
# hyperparameters from it) as a one-block kernel with system-scope accesses instead of
# hipMemcpyAsync, whose calls blocked the host ~57 us each in the r06s13 API trace.  (1) parity
# subset (sampler parity, pipelined chains, multi-rank, production ML-20M); (2) A/B against
# build_prev (the r06s14 build), ML-1M K=50 and ML-20M, 3 interleaved rounds; (3) the ML-1M timeline.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_production.py \
  tests/test_gpu_bias.py tests/test_gpu_cli.py -x -q --timeout 600 --timeout-method thread \
  > "$O/r06s16_suite.log" 2>&1 || { tail -30 "$O/r06s16_suite.log"; exit 1; }
tail -1 "$O/r06s16_suite.log"
P=$R/scalable-bayesian-matrix-factorization_amd/build_prev/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
show() { python3 -c "
import json; d=json.load(open('$1')); c=d['config']
print('$2', round(d['ms_per_step'],4), 'user', round(c['ms_user_half'],3), 'item', round(c['ms_item_half'],3), 'hyper', round(c['ms_hyper'],3), 'eval', round(c['ms_eval'],3))"; }
for i in 1 2 3; do
  for v in new prev; do
    L=$N; [ $v = prev ] && L=$P
    SBMF_LIB=$L timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr \
      --no-f32 --no-load > "$O/r06s16_ml1m_${v}_$i.json" 2> "$O/r06s16_ml1m_${v}_$i.err"
    show "$O/r06s16_ml1m_${v}_$i.json" "ml1m $v round $i"
    SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load \
      > "$O/r06s16_ml20m_${v}_$i.json" 2> "$O/r06s16_ml20m_${v}_$i.err"
    show "$O/r06s16_ml20m_${v}_$i.json" "ml20m $v round $i"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d "$O/r06s16_ml1m_trace" -o r06s16 -- python3 "$R/bench.py" --shape ml-1m --K 50 --steps 20 --warmup 3 \
  --no-cpu --no-ttr --no-f32 --no-load > "$O/r06s16_ml1m_trace.log" 2>&1
python3 "$R/profiles/r06/timeline.py" "$O/r06s16_ml1m_trace" 3 > "$O/r06s16_ml1m_timeline.txt"
tail -1 "$O/r06s16_ml1m_timeline.txt"
