#!/bin/bash
# Round 3 VB profile (Netflix shape): kernel stats of one K=200 epoch, then FETCH_SIZE and WRITE_SIZE
# passes (each counter pass on its own) over one K=16 epoch restricted to the update kernels (the
# per-factor passes do the same per-launch work at any K; K=16 keeps the serialised counter run short),
# then the sampler's kernel stats under rocprofv3 (exit status after the quick-exit change).
# Outputs gpurun_out/r03l_*.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
cd /tmp && export TMPDIR=/tmp
VB="python3 $R/bench.py --method vb --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03l_vbtrace -o vb -- \
  $VB --steps 1 --warmup 0 > $O/r03l_vbtrace.log 2>&1 || { echo "vbtrace rc $?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $c --kernel-include-regex 'k_update' \
    -d $O/r03l_vb_$c -o vb -- $VB --K 16 --steps 1 --warmup 0 > $O/r03l_vb_$c.log 2>&1 || { echo "$c rc $?"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03l_trace -o sb -- \
  python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 > $O/r03l_trace.log 2>&1 || { echo "trace rc $?"; exit 1; }
echo vbprof done
