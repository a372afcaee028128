#!/bin/bash
# Round 4 final pass (after the sweep-boundary and libFM host-sum changes), part B: rocprofv3 kernel trace (per-dispatch CSV kept) + FETCH_SIZE /
# WRITE_SIZE / LDS passes of the default line; BASELINE configs 2-4 lines; the biased sampler,
# online VB (config 5) and libFM MCMC / ALS lines.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for p in trace fetch write lds; do
  bash profiles/collect.sh r04g_ml20m $p || { echo "collect $p failed"; exit 1; }
done
for c in "ml-1m 50" "ml-10m 100" "ml-20m 200"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --shape $1 --K $2 --no-ttr --no-load --no-f32 > $O/r04g_bench_$1_k$2.json 2> $O/r04g_bench_$1_k$2.err \
    || { echo "bench $1 $2 rc $?"; tail -5 $O/r04g_bench_$1_k$2.err; exit 1; }
  echo "bench $1 K=$2 ok"
done
timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-ttr --no-load --no-f32 --no-cpu > $O/r04g_bench_bias2.json 2> $O/r04g_bench_bias2.err || { echo "bias2 rc $?"; exit 1; }
timeout -k 10 400 python3 bench.py --method vb --steps 2 --warmup 1 --no-cpu > $O/r04g_vb_bench.json 2> $O/r04g_vb_bench.err || { echo "vb rc $?"; tail -5 $O/r04g_vb_bench.err; exit 1; }
for m in libfm als; do
  timeout -k 10 300 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu > $O/r04g_bench_libfm_$m.json 2> $O/r04g_bench_libfm_$m.err || { echo "$m rc $?"; exit 1; }
done
export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04g_libfm_trace -o libfm -- \
  python3 $R/bench.py --method libfm --steps 2 --warmup 1 --no-cpu > $O/r04g_libfm_trace.log 2>&1 || { echo "libfm trace rc $?"; exit 1; }
echo s29b done
