#!/bin/bash
# r05 step 36: eighth size classes (20 and 28 vectors per wave) for the 16-wave item set, against
# HEAD (build_prev, quarters only):
# parity subset, 3 interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "variants or split" > "$O/r05s36_parity.log" 2>&1 \
    || { tail -30 "$O/r05s36_parity.log"; exit 1; }
tail -1 "$O/r05s36_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
B=$R/scalable-bayesian-matrix-factorization_amd/build_prev/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2 3; do for t in prev 0; do
  L=$N; tn=$t; [ $t = prev ] && { L=$B; tn=0; }
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $tn > "$O/r05s36_ab_t${t}_$i.json" 2> "$O/r05s36_ab_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s36_ab_t${t}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('$t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'istream', b['item_gres_stage']['ms'])"
done; done
