#!/bin/bash
# Round 4 step 4: rocprofv3 passes of bench.py with a normal process exit (RCCL no longer linked):
# kernel trace (per-dispatch CSV kept) + stats, FETCH_SIZE, WRITE_SIZE and LDS passes of the
# default ML-20M K=100 line, and config 3's (ML-10M K=100) trace / FETCH / WRITE.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for p in trace fetch write lds; do
  bash profiles/collect.sh r04s4_ml20m $p || { echo "collect ml20m $p failed rc $?"; tail -3 $O/r04s4_ml20m_*$p*.log; exit 1; }
done
for p in trace fetch write; do
  BENCH_ARGS="--shape ml-10m --K 100" bash profiles/collect.sh r04s4_ml10m $p || { echo "collect ml10m $p failed"; exit 1; }
done
ls $O | grep r04s4
echo s4 done
