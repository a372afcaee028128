#!/bin/bash
# Round 4 step 8: Gram-block kernels skip the gathers, MFMAs and c terms of a wave's vectors
# past the row's end (wave-uniform; SBMF_GB_SKIP=0 build keeps them): parity subset, A/B 3
# rounds; SQ counter passes (instruction mix, waits) of the default line.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -x -q \
  --timeout 300 --timeout-method thread > $O/r04s8_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s8_pytest.log; exit 1; }
tail -1 $O/r04s8_pytest.log
bash profiles/ab_args.sh r04s8 3 "skip=build: noskip=build_noskip:" || { echo "ab failed"; exit 1; }
for f in $O/r04s8_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items()})")"; done
for p in sq sq2; do bash profiles/collect.sh r04s8 $p || { echo "collect $p failed"; exit 1; }; done
echo s8 done
