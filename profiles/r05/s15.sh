#!/bin/bash
# r05 step 15: beside two item streaming sets every Gram-block kind on the second side stream
# (not queued behind streaming set 0); also tune bit 23 (user streaming rows on 8-wave k_gres
# workgroups, 1024-rating tasks) on top of k_grow: variant parity, bench A/B against HEAD's
# build (SBMF_LIB), 2 rounds.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "variants or golden" tests/test_gpu_rccl.py > "$O/r05s15_parity.log" 2>&1 \
    || { tail -30 "$O/r05s15_parity.log"; exit 1; }
tail -1 "$O/r05s15_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
B=$R/scalable-bayesian-matrix-factorization_amd/build_base/libsbmf.so
N=$R/scalable-bayesian-matrix-factorization_amd/build/libsbmf.so
for i in 1 2; do for t in base 0 8388608; do
  L=$N; tag=$t; tn=$t; [ $t = base ] && { L=$B; tn=0; }
  SBMF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $tn > "$O/r05s15_ab_t${tag}_$i.json" 2> "$O/r05s15_ab_t${tag}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s15_ab_t${tag}_$i.json')); c=d['config']; b=d['roofline']['bins']; print('$tag round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), 'ustream', b['user_gres_stage']['ms'], 'istream', b['item_gres_stage']['ms'])"
done; done
