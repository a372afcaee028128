#!/bin/bash
# Round 4 step 6: what bounds the user half's launches.  ABLATE=1 build (timing only, wrong
# results), launches serial (tune bit 29) so every bin's HIP-event time is its own: Gram-block
# ablations (0x100 every gather on one cached row, 0x200 no recurrence, 0x800 the block loop
# twice, 0x1000 no MFMA) and k_gres ones (0x4000 no split-row hand-off, 0x8000 no recurrence,
# 0x40000 no residual update, 0x80000 no MFMA); then stream threshold 192 against 256, 3 rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
S=536870912
bash profiles/ab_args.sh r04s6 1 "abl=build_ablate:--tune,$S gat=build_ablate:--tune,$((S+0x100)) sol=build_ablate:--tune,$((S+0x200)) twice=build_ablate:--tune,$((S+0x800)) mfma=build_ablate:--tune,$((S+0x1000)) gxchg=build_ablate:--tune,$((S+0x4000)) gsol=build_ablate:--tune,$((S+0x8000)) gres=build_ablate:--tune,$((S+0x40000)) gmfma=build_ablate:--tune,$((S+0x80000))" \
  || { echo "ab1 failed"; exit 1; }
bash profiles/ab_args.sh r04s6 3 "new=build: thr192=build:--stream-threshold,192" || { echo "ab2 failed"; exit 1; }
for f in $O/r04s6_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), {k: round(v,3) for k,v in c['kernel_ms'].items()})")"; done
echo s6 done
