# A/B of k_gres scheduling variants on one box (bench.py, f64 only); outputs gpurun_out/<tag>_<name>.json
set -e
TAG=${1:-ab}
B=scalable-bayesian-matrix-factorization_amd
run() { name=$1; lib=$2; shift 2; SBMF_LIB=$PWD/$B/$lib/libsbmf.so timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 "$@" > gpurun_out/${TAG}_$name.json 2>/dev/null; }
run t0 build --tune 0
run rounds build --tune 65536
run kp build_kprof --tune 0
run kp_noxchg build_kprof --tune 16384
run kp_noxchg_nosolve build_kprof --tune 49152
run t0b build --tune 0
