# Gram-block ablations (KPROF=1 diagnostic build; tune bits 0x100 one cached partner row,
# 0x200 no recurrence, 0x400 no residual row sums, 0x800 block loop run twice, 0x1000 no MFMA -- timings only, results are wrong).
set -e
make -C scalable-bayesian-matrix-factorization_amd/csrc KPROF=1 -B -j16 > gpurun_out/mk.log 2>&1
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
for t in 0 4096 6144 1792 5888; do
  echo "== tune $t"
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --no-ttr --no-f32 --tune $t | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('%.2f ms user %.2f item %.2f' % (d['ms_per_step'], c['ms_user_half'], c['ms_item_half'])); print({k: v for k, v in c['kernel_ms'].items() if v > 0.1 and 'gblock' in k})"
done
