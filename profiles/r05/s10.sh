#!/bin/bash
# r05 step 10: narrow tail block in k_gres (K % 16 in 1..4: the last 16-column block
# gathers and multiplies 4 columns): parity subset, then bench A/B against the
# previous build (build_base, SBMF_LIB), 2 interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_cli.py > "$O/r05s10_parity.log" 2>&1 \
    || { tail -30 "$O/r05s10_parity.log"; exit 1; }
tail -1 "$O/r05s10_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
B=$R/scalable-bayesian-matrix-factorization_amd/build_base/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2; do for v in base tail; do
  L=$N; [ $v = base ] && L=$B
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > "$O/r05s10_ab_${v}_$i.json" 2> "$O/r05s10_ab_${v}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s10_ab_${v}_$i.json')); c=d['config']; print('$v round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_hyper'],3), round(c['ms_eval'],3))"
done; done
for v in base tail; do
  L=$N; [ $v = base ] && L=$B
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --shape ml-1m --K 50 --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > "$O/r05s10_k50_${v}.json" 2> "$O/r05s10_k50_${v}.err"
  python3 -c "
import json; d=json.load(open('$O/r05s10_k50_${v}.json')); c=d['config']; print('K50 $v', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))"
done
