# A/B of built libraries on one box (bench.py f64 only, default tune): ab_libs.sh TAG DIR... ;
# DIR is a build directory under the package (build, build_base, ...); outputs gpurun_out/<tag>_<dir>_<i>.json
set -e
TAG=$1
shift
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for d in "$@"; do
    SBMF_LIB=$PWD/$B/$d/libsbmf.so timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 \
      > gpurun_out/${TAG}_${d}_$i.json 2>/dev/null
  done
done
