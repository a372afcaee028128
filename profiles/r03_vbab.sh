#!/bin/bash
# VB variants on the Netflix K=200 epoch (GPU ms per epoch): default (8 XCD slices, partner re-read,
# 6 waves/SIMD), no slices, partner values kept in registers at 5 waves/SIMD, 8 waves/SIMD; then
# counter passes over a K=16 epoch of the update kernels: L2 requests/hits/misses and SQ wave states.
# Outputs gpurun_out/r03o_*.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
B=$R/scalable-bayesian-matrix-factorization_amd
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
VB="python3 $R/bench.py --method vb --no-cpu --steps 1 --warmup 1"
run() { # tag, env...
  local t=$1; shift
  env "$@" timeout -k 10 300 $VB > $O/r03o_$t.json 2> $O/r03o_$t.err || { echo "$t rc $?"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/r03o_$t.json').read().strip().splitlines()[-1]); print('$t', round(d['config']['gpu_ms_per_epoch'],1), 'ms/epoch')" | tee -a $O/r03o_summary.txt
}
: > $O/r03o_summary.txt
run default SBMF_X=1
run slices1 SBMF_VB_SLICES=1
run keep5 SBMF_LIB=$B/build_vbk/libsbmf.so
run occ8 SBMF_LIB=$B/build_vbo8/libsbmf.so
cd /tmp && export TMPDIR=/tmp
K16="python3 $R/bench.py --method vb --no-cpu --K 16 --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex 'k_user|k_item' \
  -d $O/r03o_tcc -o vb -- $K16 > $O/r03o_tcc.log 2>&1 || { echo "tcc rc $?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-include-regex 'k_user|k_item' \
  -d $O/r03o_sq -o vb -- $K16 > $O/r03o_sq.log 2>&1 || { echo "sq rc $?"; exit 1; }
echo vbab done
