# A/B of built libraries on the libFM MCMC bench (ML-20M shape, K=100): ab_libfm.sh TAG DIR...
set -e
TAG=$1
shift
B=scalable-bayesian-matrix-factorization_amd
for d in "$@"; do
  SBMF_LIB=$PWD/$B/$d/libsbmf.so timeout -k 10 300 python3 bench.py --method libfm --steps 3 --warmup 1 \
    > gpurun_out/${TAG}_${d}.json 2>/dev/null
done
