#!/bin/bash
# Round 3 VB profile (Netflix shape, K=200, one epoch after one warm-up epoch): kernel stats, then
# FETCH_SIZE and WRITE_SIZE passes (each counter pass on its own), plus the sampler under rocprofv3
# once more (exit status after the quick-exit change).  Outputs gpurun_out/r03h_*.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 -c "import sys; sys.path.insert(0,'scalable-bayesian-matrix-factorization_amd'); from sbmf import synth; synth.generate('netflix'); synth.generate('ml-20m')" > $O/r03h_gen.log 2>&1 || { echo gen failed; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03h_vbtrace -o vb -- \
  python3 $R/bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/r03h_vbtrace.log 2>&1
echo "rc $?" >> $O/r03h_vbtrace.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/r03h_vbfetch -o vb -- \
  python3 $R/bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/r03h_vbfetch.log 2>&1
echo "rc $?" >> $O/r03h_vbfetch.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/r03h_vbwrite -o vb -- \
  python3 $R/bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/r03h_vbwrite.log 2>&1
echo "rc $?" >> $O/r03h_vbwrite.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03h_trace -o sb -- \
  python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 > $O/r03h_trace.log 2>&1
echo "rc $?" >> $O/r03h_trace.log
echo vbprof done
