#!/bin/bash
# Round-3 (session 2) final measurement pass at the final HEAD, one call: the whole GPU test suite, the
# default bench line (the driver's command), kernel stats under rocprofv3, FETCH_SIZE / WRITE_SIZE and
# LDS passes (each counter pass on its own run), and the VB, biased-sampler and libFM / ALS lines.
set -uo pipefail
TAG=${TAG:-r03w}
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/${TAG}_pytest.log; exit 1; }
grep -E "passed|failed" $O/${TAG}_pytest.log | tail -1
timeout -k 10 500 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench rc $?"; exit 1; }
for p in trace fetch write lds; do
  bash profiles/collect.sh ${TAG} $p || { echo "collect $p failed"; exit 1; }
done
timeout -k 10 400 python3 bench.py --method vb > $O/${TAG}_vb.json 2> $O/${TAG}_vb.err || { echo "vb rc $?"; exit 1; }
timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-cpu > $O/${TAG}_bias2.json 2> $O/${TAG}_bias2.err || { echo "bias2 rc $?"; exit 1; }
for m in libfm als; do
  timeout -k 10 300 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu > $O/${TAG}_$m.json 2> $O/${TAG}_$m.err || { echo "$m rc $?"; exit 1; }
done
echo final done
