#!/bin/bash
# Round-3 (session 2) final pass A on a 1-GPU MI355X: the whole GPU test suite and the default
# bench line (the driver's command).  Outputs gpurun_out/${TAG}_*.
set -uo pipefail
TAG=${TAG:-r03v}
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/${TAG}_pytest.log; exit 1; }
grep -E "passed|failed" $O/${TAG}_pytest.log | tail -1
timeout -k 10 500 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench rc $?"; exit 1; }
echo final-a done
