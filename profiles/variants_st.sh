# stream-threshold variants (bench.py f64 only): variants_st.sh TAG THRESHOLD...
set -e
TAG=$1
shift
for t in "$@"; do
  timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 --stream-threshold $t > gpurun_out/${TAG}_st$t.json 2>/dev/null
done
