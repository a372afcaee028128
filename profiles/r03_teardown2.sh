#!/bin/bash
# rocprofv3 exit-time fault: which exit path keeps the profiler's output AND exits 0?
# CLI (load-time linked libsbmf) on ML-100k, SBMF_EXIT = normal | quick (_Exit after flush) |
# early (atexit handler registered at main's start that _Exits) | reset (hipDeviceReset before return);
# bench.py normal vs quick.  Per run: exit code + the files rocprofv3 wrote.  Outputs gpurun_out/r03j_*.
set -u
R=$PWD; O=$R/gpurun_out; mkdir -p $O
python3 - <<'PY'
import gzip
for nm in ("train", "test"):
    with gzip.open("tests/golden/ml100k_%s.tsv.gz" % nm, "rt") as f, open("/tmp/ml100k_%s.tsv" % nm, "w") as g:
        g.write(f.read())
PY
cd /tmp && export TMPDIR=/tmp
S=$O/r03j_summary.txt; : > $S
for m in normal quick early reset; do
  SBMF_EXIT=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03j_cli_$m -o cli -- \
    $R/scalable-bayesian-matrix-factorization_amd/build/sbmf -task r -train /tmp/ml100k_train.tsv -test /tmp/ml100k_test.tsv \
    -dim 0,0,20 -iter 5 > $O/r03j_cli_$m.log 2>&1
  rc=$?
  echo "cli SBMF_EXIT=$m rc=$rc files: $(ls $O/r03j_cli_$m 2>/dev/null | tr '\n' ' ')" >> $S
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && break
done
for m in normal quick; do
  SBMF_EXIT=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03j_bench_$m -o b -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 > $O/r03j_bench_$m.log 2>&1
  rc=$?
  echo "bench SBMF_EXIT=$m rc=$rc files: $(ls $O/r03j_bench_$m 2>/dev/null | tr '\n' ' ')" >> $S
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && break
done
cat $S
