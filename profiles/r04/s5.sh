#!/bin/bash
# Round 4 step 5: the split-row counters cleared by one memset per half (was three fill kernels per
# stream set, the last of which waited behind the other set's persistent launch) and same-shape
# Gram-block sub-launches merged; parity subset, then A/B against the previous HEAD (build_base):
# stream-set order (tune bit 31 = set 0 first, temporary) and the stream threshold (128 / 192).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q \
  --timeout 300 --timeout-method thread > $O/r04s5_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s5_pytest.log; exit 1; }
tail -1 $O/r04s5_pytest.log
bash profiles/ab_args.sh r04s5 2 "base=build_base: new=build: set0first=build:--tune,2147483648 thr192=build:--stream-threshold,192 thr128=build:--stream-threshold,128" \
  || { echo "ab failed"; exit 1; }
for f in $O/r04s5_*_[12].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3))")"; done
echo s5 done
