#!/bin/bash
# Round 4 step 19: libFM's prediction kernels read the factor rows four factors at a time (same
# terms, same order); online VB's prediction kernel loads the next case's partner id while it
# reads the current case's rows.  GPU tests of both learners, then A/B against HEAD (build_base).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_libfm.py tests/test_gpu_cli.py tests/test_gpu_vbo.py -x -q --timeout 400 --timeout-method thread > $O/r04s19_pytest.log 2>&1 || { echo "pytest rc $?"; tail -20 $O/r04s19_pytest.log; exit 1; }
tail -1 $O/r04s19_pytest.log
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for d in build_base build; do
    SBMF_LIB=$R/$B/$d/libsbmf.so timeout -k 10 200 python3 bench.py --method libfm --steps 3 --warmup 1 --no-cpu > $O/r04s19_${d}_libfm_$i.json 2> $O/r04s19_${d}_libfm_$i.err || { echo "$d libfm rc $?"; exit 1; }
    SBMF_LIB=$R/$B/$d/libsbmf.so timeout -k 10 300 python3 bench.py --method vb --steps 2 --warmup 1 --no-cpu > $O/r04s19_${d}_vb_$i.json 2> $O/r04s19_${d}_vb_$i.err || { echo "$d vb rc $?"; exit 1; }
  done
done
for f in $O/r04s19_*_[12].json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('test_rmse_after'))")"; done
echo s19 done
