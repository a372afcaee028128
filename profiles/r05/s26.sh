#!/bin/bash
# r05 step 26: wave-0 phase profile (KPROF build, SBMF_KPROF=1) of the final kernels' streaming
# sets: the item 16-wave set (SBMF_KPROF_SET=1) and the item 8-wave / user 4-wave sets (set 0).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
K=$R/scalable-bayesian-matrix-factorization_amd/build_kprof/libsbmf.so
SBMF_LIB=$K SBMF_KPROF=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 --no-load \
    > "$O/r05s26_kprof0.json" 2> "$O/r05s26_kprof0.txt"
SBMF_LIB=$K SBMF_KPROF=1 SBMF_KPROF_SET=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 --no-load \
    > "$O/r05s26_kprof1.json" 2> "$O/r05s26_kprof1.txt"
grep "sweep 2" -A 3 "$O/r05s26_kprof0.txt" | head -12
grep "sweep 2" -A 3 "$O/r05s26_kprof1.txt" | head -12
