#!/bin/bash
# r05 step 11: k_grow -- the 65..128 / 129..256-rating f64 Gram-block bins as whole rows on
# the streaming kernel's code with one / two waves per row (tune bits 8 / 9): kernel-variant
# parity against the oracle, then bench A/B (tune 0 / 256 / 512 / 768, and HEAD's build through SBMF_LIB), 2 interleaved rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "variants" > "$O/r05s11_parity.log" 2>&1 \
    || { tail -30 "$O/r05s11_parity.log"; exit 1; }
tail -1 "$O/r05s11_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
B=$R/scalable-bayesian-matrix-factorization_amd/build_base/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2; do for t in base 0 256 512 768; do
  L=$N; [ $t = base ] && { L=$B; t=0; tag=base; } || tag=$t
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s11_ab_t${tag}_$i.json" 2> "$O/r05s11_ab_t${tag}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s11_ab_t${tag}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('tune $tag round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'b4', b['user_gblock_b4']['ms'], 'b8', b['user_gblock_b8']['ms'])"
done; done
