#!/bin/bash
# Round 4 step 18: rocprofv3 kernel statistics of the libFM MCMC line (after the long-row work)
# and of the online VB line (config 5).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04s18_libfm -o libfm -- \
  python3 $R/bench.py --method libfm --steps 2 --warmup 1 --no-cpu > $O/r04s18_libfm.log 2>&1 || { echo "libfm rc $?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04s18_vb -o vb -- \
  python3 $R/bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/r04s18_vb.log 2>&1 || { echo "vb rc $?"; exit 1; }
echo s18 done
