#!/bin/bash
# Round 4 step 33: bench.py reads each sweep's launch-kind times through a preallocated struct
# view (the callback's Python cost sits between two sweeps); the default line as the driver runs
# it, then two short lines.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 500 python3 bench.py > $O/r04s33_default.json 2> $O/r04s33_default.err || { echo "default bench rc $?"; tail -20 $O/r04s33_default.err; exit 1; }
for i in 1 2; do
  timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > $O/r04s33_short_$i.json 2> $O/r04s33_short_$i.err || { echo "short rc $?"; exit 1; }
done
for f in $O/r04s33_default.json $O/r04s33_short_[12].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), round(d['roofline']['ms_per_launch'],3), round(d['roofline']['frac'],3), c['test_rmse_after'])")"; done
echo s33 done
