#!/bin/bash
# After the exit guard (sbmf_exit_guard): the CLI and bench.py under rocprofv3 --kernel-trace --stats,
# default exit path -- exit code and the files rocprofv3 wrote.  Outputs gpurun_out/r03k_*.
set -u
R=$PWD; O=$R/gpurun_out; mkdir -p $O
python3 - <<'PY'
import gzip
for nm in ("train", "test"):
    with gzip.open("tests/golden/ml100k_%s.tsv.gz" % nm, "rt") as f, open("/tmp/ml100k_%s.tsv" % nm, "w") as g:
        g.write(f.read())
PY
cd /tmp && export TMPDIR=/tmp
S=$O/r03k_summary.txt; : > $S
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03k_cli -o cli -- \
  $R/scalable-bayesian-matrix-factorization_amd/build/sbmf -task r -train /tmp/ml100k_train.tsv -test /tmp/ml100k_test.tsv \
  -dim 0,0,20 -iter 5 -out /tmp/pred.txt > $O/r03k_cli.log 2>&1
rc=$?; echo "cli rc=$rc files: $(ls $O/r03k_cli 2>/dev/null | tr '\n' ' ') pred lines: $(wc -l < /tmp/pred.txt)" >> $S
[ $rc -eq 124 ] || [ $rc -eq 137 ] && { cat $S; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03k_bench -o b -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 > $O/r03k_bench.log 2>&1
rc=$?; echo "bench rc=$rc files: $(ls $O/r03k_bench 2>/dev/null | tr '\n' ' ')" >> $S
cat $S
