#!/bin/bash
# Round 3 probe 2: (1) the load-time-linked CLI under rocprofv3 (does the exit-time SIGSEGV follow the
# Python dlopen teardown or the library?); (2) the biased-sampler throughput line (quirks bias2, ML-20M
# K=100 f64); (3) a round-3 online-VB line (Netflix shape, K=200) and its rocprofv3 kernel stats.
# Outputs gpurun_out/r03f_*.  Every rocprofv3 pass is the last step that may crash; each runs under timeout.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
python3 - <<'PY'
import gzip
for nm in ("train", "test"):
    with gzip.open("tests/golden/ml100k_%s.tsv.gz" % nm, "rt") as f, open("/tmp/ml100k_%s.tsv" % nm, "w") as g:
        g.write(f.read())
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03f_cli -o cli -- \
  $R/scalable-bayesian-matrix-factorization_amd/build/sbmf -task r -train /tmp/ml100k_train.tsv -test /tmp/ml100k_test.tsv \
  -dim 0,0,20 -iter 5 > $O/r03f_cli.log 2>&1
echo "cli under rocprofv3 exit code: $?" >> $O/r03f_cli.log
cd $R
timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-cpu > $O/r03f_bias2.json 2> $O/r03f_bias2.err || echo "bias2 bench rc $?" >> $O/r03f_bias2.err
timeout -k 10 600 python3 bench.py --method vb --steps 2 --warmup 1 > $O/r03f_vb.json 2> $O/r03f_vb.err || { echo "vb bench rc $?" >> $O/r03f_vb.err; exit 1; }
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03f_vbtrace -o vb -- \
  python3 $R/bench.py --method vb --steps 1 --warmup 1 --no-cpu > $O/r03f_vbtrace.log 2>&1
echo "vb trace rc $?" >> $O/r03f_vbtrace.log
echo probe2 done
