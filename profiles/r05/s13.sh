#!/bin/bash
# r05 step 13: k_grow for the 9..256-rating f64 bins by default (its task loop in the form that
# compiles to 1-2 spilled VGPRs; the r05s11/s12 builds had 50-70): GPU parity subset, then bench
# A/B against the Gram-block kinds (tune 1792) and an SBMF_ALLW=1 build (every wave of a
# multi-wave k_gres / k_grow workgroup draws the block itself: no D hand-off), 2 rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_cli.py > "$O/r05s13_parity.log" 2>&1 \
    || { tail -30 "$O/r05s13_parity.log"; exit 1; }
tail -1 "$O/r05s13_parity.log"
SBMF_LIB=$R/scalable-bayesian-matrix-factorization_amd/build_allw/libsbmf.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py -k "variants or golden" > "$O/r05s13_parity_allw.log" 2>&1 \
    || { tail -30 "$O/r05s13_parity_allw.log"; exit 1; }
tail -1 "$O/r05s13_parity_allw.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
A=$R/scalable-bayesian-matrix-factorization_amd/build_allw/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2; do for t in 0 1792 allw; do
  L=$N; tag=$t; tn=$t; [ $t = allw ] && { L=$A; tn=0; }
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $tn > "$O/r05s13_ab_t${tag}_$i.json" 2> "$O/r05s13_ab_t${tag}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s13_ab_t${tag}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('$tag round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'ustream', b['user_gres_stage']['ms'], 'istream', b['item_gres_stage']['ms'], 'b4', b['user_gblock_b4']['ms'], 'b8', b['user_gblock_b8']['ms'], 'w16', b['user_gblock_w16']['ms'])"
done; done
