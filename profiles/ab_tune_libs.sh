# A/B of built libraries x tune bits on one box (bench.py f64 only):
#   ab_tune_libs.sh TAG "DIR:TUNE DIR:TUNE ..." ; DIR is a build directory under the package.
# Two rounds over the list; outputs gpurun_out/<tag>_<dir>_t<tune>_<round>.json
set -e
TAG=$1
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for dt in $2; do
    d=${dt%%:*}; t=${dt##*:}
    SBMF_LIB=$PWD/$B/$d/libsbmf.so timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 \
      --tune $t > gpurun_out/${TAG}_${d}_t${t}_$i.json 2>/dev/null
  done
done
