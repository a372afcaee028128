#!/bin/bash
# Round 4 step 16: per-dispatch kernel trace of the serial launch schedule (tune bit 29: a half's
# Gram-block launches after its streaming launch, the item sets one after the other), so every
# launch's device time is its own (no sharing), against the overlapped default's trace (r04f).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
# the serial schedule keeps the cooperative launch, whose process faults at exit under rocprofv3
# (first try: SIGSEGV in exit after the bench line, r04s16_coop_exit_fault.txt); with the opt-in guard
# the process exits 0 but rocprofv3 writes no trace (its own exit handler is skipped too), so the
# serial schedule's per-dispatch times stay unmeasured; its bench line: 7.86 ms against 7.71 overlapped
SBMF_EXIT=guard BENCH_ARGS="--tune 536870912" bash profiles/collect.sh r04s16_serial trace || { echo "trace failed"; exit 1; }
echo s16 done
