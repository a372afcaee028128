#!/bin/bash
# r05 step 12: k_grow default for the 65..256-rating f64 bins (bits 8 / 9 opt out); bit 10 puts
# the 9..64 bin on one-wave k_grow too: variant parity, GPU parity + CLI subset, bench A/B
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_cli.py tests/test_gpu_bias.py > "$O/r05s12_parity.log" 2>&1 \
    || { tail -30 "$O/r05s12_parity.log"; exit 1; }
tail -1 "$O/r05s12_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
B=$R/scalable-bayesian-matrix-factorization_amd/build_base/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2; do for t in 0 768 1024; do
  L=$N; [ $t = base ] && { L=$B; t=0; tag=base; } || tag=$t
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s12_ab_t${tag}_$i.json" 2> "$O/r05s12_ab_t${tag}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s12_ab_t${tag}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('tune $tag round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'b4', b['user_gblock_b4']['ms'], 'b8', b['user_gblock_b8']['ms'], 'w16', b['user_gblock_w16']['ms'], 'ib4', b['item_gblock_b4']['ms'], 'ib8', b['item_gblock_b8']['ms'])"
done; done
