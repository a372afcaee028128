#!/bin/bash
# Round 4 step 26: kernel trace of one libFM MCMC and one ALS bench run (launch gaps per pass).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
cd /tmp && export TMPDIR=/tmp
for m in libfm als; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04s26_${m}_trace -o r04s26 -- \
    python3 $R/bench.py --method $m --steps 2 --warmup 1 --no-cpu > $O/r04s26_${m}_trace.log 2>&1 || { echo "$m trace rc $?"; exit 1; }
done
echo s26 done
