#!/bin/bash
# r05 step 31: the CHECK=1 build (every global index of the row kernels checked against its
# array's extent; a violation is printed and redirected) over the final kernels: the default line
# (K=100 f64), K=200, f32, the biased sampler, and a small-K line (KL=128 k_grow at K=20).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
export SBMF_LIB=$R/scalable-bayesian-matrix-factorization_amd/build_check/libsbmf.so
for a in "--K 100" "--K 200" "--K 100 --precision f32" "--K 100 --quirks bias2" "--shape ml-1m --K 20"; do
  tag=$(echo $a | tr -d ' -')
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 --no-load $a > "$O/r05s31_check_$tag.json" 2> "$O/r05s31_check_$tag.err"
  echo "$a: $(grep -c 'sbmf check' "$O/r05s31_check_$tag.err" || true) index violations"
done
