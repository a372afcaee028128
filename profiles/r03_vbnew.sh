#!/bin/bash
# Online VB with one in-place {e,t} copy (user passes in place, item passes read-only + per-item deltas):
# parity (VB tests incl. several ranks), then the Netflix K=200 bench old (build_vbold: scatter design)
# vs new, the new kernels' stats, and FETCH/WRITE passes over a K=16 epoch.  Outputs gpurun_out/${TAG}_*.
set -uo pipefail
TAG=${TAG:-r03m}
R=$PWD; O=$R/gpurun_out; mkdir -p $O
B=$R/scalable-bayesian-matrix-factorization_amd
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_vbo.py tests/test_gpu_multirank.py -k "vb" -x -v --timeout 600 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { echo "pytest rc $?"; tail -30 $O/${TAG}_pytest.log; exit 1; }
timeout -k 10 300 python3 bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/${TAG}_vb_new.json 2> $O/${TAG}_vb_new.err || { echo "new rc $?"; exit 1; }
if [ -n "${OLD:-}" ]; then
  SBMF_LIB=$B/build_vbold/libsbmf.so timeout -k 10 300 python3 bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/${TAG}_vb_old.json 2> $O/${TAG}_vb_old.err || { echo "old rc $?"; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp
VB="python3 $R/bench.py --method vb --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_vbtrace -o vb -- \
  $VB --steps 1 --warmup 0 > $O/${TAG}_vbtrace.log 2>&1 || { echo "vbtrace rc $?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $c --kernel-include-regex 'k_user|k_item' \
    -d $O/${TAG}_vb_$c -o vb -- $VB --K 16 --steps 1 --warmup 0 > $O/${TAG}_vb_$c.log 2>&1 || { echo "$c rc $?"; exit 1; }
done
cat $O/${TAG}_vb_new.json $O/${TAG}_vb_old.json 2>/dev/null | grep -h "value" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['gpu_ms_per_epoch'], d['value'], d['roofline']['frac'])"
echo vbnew done
