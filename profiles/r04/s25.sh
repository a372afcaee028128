#!/bin/bash
# Round 4 step 25: libFM MCMC / ALS with a pass's three length bins on three streams
# (SBMF_FMM_STREAMS=3) against one stream: the libFM GPU tests under 3 streams, then A/B.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
SBMF_FMM_STREAMS=3 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_libfm.py -x -q --timeout 400 --timeout-method thread > $O/r04s25_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s25_pytest.log; exit 1; }
tail -1 $O/r04s25_pytest.log
for i in 1 2; do
  for ns in 1 3; do
    for m in libfm als; do
      SBMF_FMM_STREAMS=$ns timeout -k 10 200 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu > $O/r04s25_s${ns}_${m}_$i.json 2> $O/r04s25_s${ns}_${m}_$i.err || { echo "s$ns $m rc $?"; exit 1; }
    done
  done
done
for f in $O/r04s25_s*_[12].json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('test_rmse_after'))")"; done
echo s25 done
