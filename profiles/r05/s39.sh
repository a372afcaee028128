#!/bin/bash
# r05 step 39: repeatability on the final kernels -- smoke(), then the default bench line twice more
# (box-to-box range of 6.77 ms, r05s37) and config 4 (ML-20M K=200) twice more (12.25 ms, r05s38).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/r05s39_smoke.log" 2>&1 || { tail -20 "$O/r05s39_smoke.log"; exit 1; }
tail -1 "$O/r05s39_smoke.log"
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2; do
  timeout -k 10 400 python3 "$R/bench.py" --no-ttr --no-load --no-cpu > "$O/r05s39_bench_$i.json" 2> "$O/r05s39_bench_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s39_bench_$i.json')); c=d['config']; print('default $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(d['roofline']['frac'],3), d.get('f32_ms_per_step'))"
  timeout -k 10 400 python3 "$R/bench.py" --shape ml-20m --K 200 --no-ttr --no-load --no-cpu > "$O/r05s39_bench_k200_$i.json" 2> "$O/r05s39_bench_k200_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s39_bench_k200_$i.json')); print('K200 $i', round(d['ms_per_step'],3), round(d['roofline']['frac'],3), d.get('f32_ms_per_step'))"
done
