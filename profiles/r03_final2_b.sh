#!/bin/bash
# Round-3 (session 2) final pass B: kernel stats under rocprofv3, FETCH_SIZE / WRITE_SIZE and LDS
# passes (each counter pass on its own run), the VB bench line and the biased-sampler line.
set -uo pipefail
TAG=${TAG:-r03v}
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for p in trace fetch write lds; do
  bash profiles/collect.sh ${TAG} $p || { echo "collect $p failed"; exit 1; }
done
timeout -k 10 400 python3 bench.py --method vb > $O/${TAG}_vb.json 2> $O/${TAG}_vb.err || { echo "vb rc $?"; exit 1; }
timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-cpu > $O/${TAG}_bias2.json 2> $O/${TAG}_bias2.err || { echo "bias2 rc $?"; exit 1; }
echo final-b done
