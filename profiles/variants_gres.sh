# k_gres workgroup-shape variants on one box (bench.py f64 only); outputs gpurun_out/<tag>_t<tune>.json
set -e
TAG=${1:-var}
shift
for t in "$@"; do
  timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 --tune $t > gpurun_out/${TAG}_t$t.json 2>/dev/null
done
