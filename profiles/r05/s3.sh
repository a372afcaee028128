#!/bin/bash
# r05 step 3: the secondary lines with their CPU baselines: libFM MCMC
# and ALS (ML-20M K=100), online VB (Netflix-shaped 100M, K=200), the biased sampler (bias2).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 "$R/bench.py" --method libfm --steps 10 --warmup 2 > "$O/r05s3_bench_libfm_mcmc.json" 2> "$O/r05s3_libfm_mcmc.err"
timeout -k 10 400 python3 "$R/bench.py" --method als --steps 10 --warmup 2 > "$O/r05s3_bench_libfm_als.json" 2> "$O/r05s3_libfm_als.err"
timeout -k 10 400 python3 "$R/bench.py" --quirks bias2 > "$O/r05s3_bench_bias2.json" 2> "$O/r05s3_bias2.err"
timeout -k 10 600 python3 "$R/bench.py" --method vb --steps 3 --warmup 1 > "$O/r05s3_vb_bench.json" 2> "$O/r05s3_vb.err"
for f in libfm_mcmc libfm_als bias2; do python3 -c "
import json; d=json.load(open('$O/r05s3_bench_$f.json')); print('$f', d['ms_per_step'], d.get('cpu_baseline',{}).get('value'))"; done
python3 -c "
import json; d=json.load(open('$O/r05s3_vb_bench.json')); print('vb', d['ms_per_step'], d.get('cpu_baseline',{}).get('value'))"
