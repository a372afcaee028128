#!/bin/bash
# Round 4 step 17: libFM MCMC / ALS passes (1) with each length bin's rows longest-first (one
# block per row, results unchanged) and (2) with the long-row bin's rows (> 4096 cases) cut into
# 4096-case chunks (chunk sums, a per-row draw, a per-chunk residual update); the libFM GPU tests
# (incl. the chunked rows against the oracle); A/B against HEAD (build_base), 2 rounds:
# base / LPT only (SBMF_FMM_CHUNK=0) / LPT + chunks.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_libfm.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread > $O/r04s17_pytest.log 2>&1 || { echo "pytest rc $?"; tail -20 $O/r04s17_pytest.log; exit 1; }
tail -1 $O/r04s17_pytest.log
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for v in "base:build_base:4096" "lpt:build:0" "chunk:build:4096"; do
    IFS=: read -r lab d ch <<< "$v"
    for m in libfm als; do
      SBMF_FMM_CHUNK=$ch SBMF_LIB=$R/$B/$d/libsbmf.so timeout -k 10 200 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu \
        > $O/r04s17_${lab}_${m}_$i.json 2> $O/r04s17_${lab}_${m}_$i.err || { echo "$lab $m rc $?"; tail -5 $O/r04s17_${lab}_${m}_$i.err; exit 1; }
    done
  done
done
for f in $O/r04s17_*_[12].json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('test_rmse_after'))")"; done
echo s17 done
