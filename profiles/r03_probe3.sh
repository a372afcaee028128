#!/bin/bash
# Round 3 probe 3: VB (several cases per lane) and the staged multi-rank pipeline -- parity first;
# then the VB and biased-sampler bench lines; then the CLI under rocprofv3 (exit-time SIGSEGV probe).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_vbo.py tests/test_gpu_multirank.py -x -v --timeout 600 --timeout-method thread > $O/r03g_pytest.log 2>&1 || { echo "pytest rc $?"; exit 1; }
timeout -k 10 600 python3 bench.py --method vb --steps 2 --warmup 1 > $O/r03g_vb.json 2> $O/r03g_vb.err || { echo "vb bench rc $?"; exit 1; }
timeout -k 10 300 python3 bench.py --quirks bias2 --steps 10 --warmup 2 --no-cpu > $O/r03g_bias2.json 2> $O/r03g_bias2.err || { echo "bias2 rc $?"; exit 1; }
python3 - <<'PY'
import gzip
for nm in ("train", "test"):
    with gzip.open("tests/golden/ml100k_%s.tsv.gz" % nm, "rt") as f, open("/tmp/ml100k_%s.tsv" % nm, "w") as g:
        g.write(f.read())
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03g_cli -o cli -- \
  $R/scalable-bayesian-matrix-factorization_amd/build/sbmf -task r -train /tmp/ml100k_train.tsv -test /tmp/ml100k_test.tsv \
  -dim 0,0,20 -iter 5 > $O/r03g_cli.log 2>&1
echo "cli under rocprofv3 exit code: $?" >> $O/r03g_cli.log
echo probe3 done
