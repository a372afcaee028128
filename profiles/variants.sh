# Kernel-variant comparison on one GPU (ML-20M-shaped synthetic, K=100, f64).
# Each line: ENV=value bench-arguments...
set -e
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
run() {
  echo "== $*"
  local e="$1"; shift
  env "$e" timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu --no-ttr --no-f32 "$@" | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('%.3f G/s %.2f ms user %.2f item %.2f' % (d['value']/1e9, d['ms_per_step'], c['ms_user_half'], c['ms_item_half'])); print({k: v for k, v in c['kernel_ms'].items() if v > 0.1})"
}
run X=0 --tune 0
run X=0 --tune 0 --precision f32
