# A/B of k_gres scheduling variants and KPROF-build ablations on one box (bench.py, f64 only);
# outputs gpurun_out/<tag>_<name>.json.  Ablation bits (KPROF build only, wrong results, timing only):
# 0x4000 no split-row hand-off, 0x8000 no 16-step recurrence, 0x40000 no residual update, 0x80000 no MFMA
set -e
TAG=${1:-ab}
B=scalable-bayesian-matrix-factorization_amd
run() { name=$1; lib=$2; shift 2; SBMF_LIB=$PWD/$B/$lib/libsbmf.so timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 "$@" > gpurun_out/${TAG}_$name.json 2>/dev/null; }
run t0 build --tune 0
run abl build_abl --tune 0
run kp_noxchg build_abl --tune 16384
run kp_nosolve build_abl --tune 32768
run kp_noapply build_abl --tune 262144
run kp_nomfma build_abl --tune 524288
run kp_noxchg_nosolve_noapply build_abl --tune 311296
run kp_all build_abl --tune 835584
