#!/bin/bash
# r05 step 7: 256-row column statistics with 16 rows in flight per wave, and the k_test
# variant (tune bit 9: 4 ratings x 4 k-blocks per round): parity subset, bench A/B
# (2 interleaved rounds), and a per-dispatch trace of the default.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_bias.py tests/test_gpu_cli.py > "$O/r05s7_parity.log" 2>&1 \
    || { tail -30 "$O/r05s7_parity.log"; exit 1; }
tail -1 "$O/r05s7_parity.log"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2; do for t in 0 512; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load --tune $t > "$O/r05s7_ab_t${t}_$i.json" 2> "$O/r05s7_ab_t${t}_$i.err"
  python3 -c "
import json; d=json.load(open('$O/r05s7_ab_t${t}_$i.json')); c=d['config']; print('ab t=$t round $i', round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_hyper'],3), round(c['ms_eval'],3))"
done; done
bash profiles/collect.sh r05s7 trace
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/r05s7_trace/*kernel_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = rows[-16:]
b = int(sel[0]["Start_Timestamp"])
for r in sel:
    print("%8.1f %7.1f %s" % ((int(r["Start_Timestamp"]) - b) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:60]))
PY
