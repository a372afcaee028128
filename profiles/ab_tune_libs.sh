# A/B of built libraries x tune bits on one box (bench.py f64 only):
#   ab_tune_libs.sh TAG "DIR:TUNE DIR:TUNE ..." ; DIR is a build directory under the package.
# Two rounds over the list; outputs gpurun_out/<tag>_<dir>_t<tune>_<round>.json (+ .err).
# A run that exits with an ordinary error is recorded and the list goes on; an abort, a
# segfault or a time limit ends the script (nothing more runs on the GPU in that call).
set -e
TAG=$1
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for dt in $2; do
    d=${dt%%:*}; t=${dt##*:}
    rc=0
    SBMF_LIB=$PWD/$B/$d/libsbmf.so timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 \
      --tune $t > gpurun_out/${TAG}_${d}_t${t}_$i.json 2> gpurun_out/${TAG}_${d}_t${t}_$i.err || rc=$?
    if [ $rc -ne 0 ]; then
      echo "ab: $d tune $t round $i exited $rc"
      case $rc in 124|134|137|139) exit $rc ;; esac
    fi
  done
done
