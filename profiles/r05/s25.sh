#!/bin/bash
# r05 step 25: k_gres claims its next ticket as a task's epilogue starts (blocks done: no peer waits on
# it) and its task-boundary barriers are LDS-only, so the scattered residual stores drain in the background: parity subset (+production, multirank), bench A/B against HEAD (build_prev), 3 rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_cli.py tests/test_gpu_production.py tests/test_gpu_multirank.py > "$O/r05s25_parity.log" 2>&1 \
    || { tail -30 "$O/r05s25_parity.log"; exit 1; }
tail -1 "$O/r05s25_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
B=$R/scalable-bayesian-matrix-factorization_amd/build_prev/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2 3; do for t in prev new; do
  L=$N; [ $t = prev ] && L=$B
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > "$O/r05s25_ab_${t}_$i.json" 2> "$O/r05s25_ab_${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s25_ab_${t}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('$t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'ustream', b['user_gres_stage']['ms'], 'istream', b['item_gres_stage']['ms'])"
done; done
