#!/bin/bash
# r06 step 14: evidence on the final round-6 build -- the whole GPU suite, smoke(), the default bench
# line (f64 + f32 + CPU baselines + time-to-RMSE + load), the default and serial (tune bit 29)
# rocprofv3 kernel traces, the PMC FETCH / WRITE / LDS passes, configs 2-4 and the biased line, and
# the per-rank compute of the 8-way split (virtual ranks, K=100 and K=200).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > "$O/r06s14_suite.log" 2>&1 || { tail -30 "$O/r06s14_suite.log"; exit 1; }
tail -1 "$O/r06s14_suite.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/r06s14_smoke.txt" 2>&1
tail -1 "$O/r06s14_smoke.txt"
bash profiles/collect.sh r06s14 bench
python3 -c "
import json; d=json.load(open('$O/r06s14_bench.json')); c=d['config']; print('bench', round(d['ms_per_step'],3), d['value'], round(c['ms_user_half'],3), round(c['ms_item_half'],3), d['roofline']['frac'], d['cpu_baseline']['value'], d['f32_ms_per_step'])"
bash profiles/collect.sh r06s14 trace
BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r06s14_serial trace
bash profiles/collect.sh r06s14 fetch && bash profiles/collect.sh r06s14 write && bash profiles/collect.sh r06s14 lds
echo pmc done
cd /tmp && export TMPDIR=/tmp
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for cfg in "ml-1m 50" "ml-10m 100" "ml-20m 200"; do
  set -- $cfg
  timeout -k 10 400 python3 "$R/bench.py" --shape $1 --K $2 --no-ttr --no-load > "$O/r06s14_bench_$1_k$2.json" 2> "$O/r06s14_bench_$1_k$2.err"
  python3 -c "
import json; d=json.load(open('$O/r06s14_bench_$1_k$2.json')); print('$1 K$2', round(d['ms_per_step'],3), d['value'], d['f32_ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 400 python3 "$R/bench.py" --quirks bias2 > "$O/r06s14_bench_bias2.json" 2> "$O/r06s14_bias2.err"
python3 -c "
import json; d=json.load(open('$O/r06s14_bench_bias2.json')); print('bias2', round(d['ms_per_step'],3), d.get('cpu_baseline',{}).get('value'))"
for K in 100 200; do
  timeout -k 10 300 python3 "$R/profiles/r05/rank_stages.py" --K $K > "$O/r06s14_rank_k${K}.json" 2> "$O/r06s14_rank_k${K}.txt"
  python3 -c "
import json; d=json.load(open('$O/r06s14_rank_k${K}.json')); print('rank K=$K: max user %.3f item %.3f max sweep %.3f' % (d['max_over_ranks']['user'], d['max_over_ranks']['item'], max(x['ms_sweep'] for x in d['per_rank'])))"
done
echo s14 done
