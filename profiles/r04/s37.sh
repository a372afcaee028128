#!/bin/bash
# Round 4 step 37: k_fmm_hsums with the next 32 values' LDS reads issued before the current adds, against HEAD.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_libfm.py tests/test_gpu_cli.py -x -q --timeout 400 --timeout-method thread > $O/r04s37_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s37_pytest.log; exit 1; }
tail -1 $O/r04s37_pytest.log
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for d in build_base build; do
    for m in libfm; do
      SBMF_LIB=$R/$B/$d/libsbmf.so timeout -k 10 200 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu > $O/r04s37_${d}_${m}_$i.json 2> $O/r04s37_${d}_${m}_$i.err || { echo "$d $m rc $?"; exit 1; }
    done
  done
done
for f in $O/r04s37_build*_[12].json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('test_rmse_after'))")"; done
echo s37 done
