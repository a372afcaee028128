#!/bin/bash
# Round 4 step 34: A/B on one box of bench.py's per-sweep timing read: the committed version
# (bench_prev.py, a temporary copy: one L.timing() + list comprehension per sweep) against the
# preallocated struct view, 3 interleaved rounds each.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for i in 1 2 3; do
  for b in bench_prev bench; do
    timeout -k 10 150 python3 $b.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > $O/r04s34_${b}_$i.json 2> $O/r04s34_${b}_$i.err || { echo "$b rc $?"; exit 1; }
  done
done
for f in $O/r04s34_*_[123].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3))")"; done
echo s34 done
