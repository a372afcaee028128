#!/bin/bash
# Round 4 step 7: one-wave Gram-block rows split by length -- rows of 9-32 ratings on 8-vector
# waves, 33-64 on 16-vector waves (round 3's "wide" kind put every row of 9-64 ratings on 16
# vectors: tune bit 31 here, temporary) -- parity subset, then A/B, 3 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q \
  --timeout 300 --timeout-method thread > $O/r04s7_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s7_pytest.log; exit 1; }
tail -1 $O/r04s7_pytest.log
bash profiles/ab_args.sh r04s7 3 "split=build: merged=build:--tune,2147483648" || { echo "ab failed"; exit 1; }
for f in $O/r04s7_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items()})")"; done
echo s7 done
