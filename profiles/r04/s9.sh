#!/bin/bash
# Round 4 step 9: the block solve broadcasts d_j with one 64-bit DPP row_newbcast move instead of
# a readlane pair (k_gblock and k_gres); parity subset; A/B against HEAD (build_base), plus user
# rows above 1024 / 2048 ratings on 16-wave k_gres workgroups (SBMF_X_USER16, experiment), 3 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py tests/test_gpu_bias.py -x -q \
  --timeout 400 --timeout-method thread > $O/r04s9_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/r04s9_pytest.log; exit 1; }
tail -1 $O/r04s9_pytest.log
bash profiles/ab_args.sh r04s9 3 "base=build_base: dpp=build: u1024=build:env:SBMF_X_USER16=1024 u2048=build:env:SBMF_X_USER16=2048" || { echo "ab failed"; exit 1; }
for f in $O/r04s9_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items()})")"; done
echo s9 done
