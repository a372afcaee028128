#!/bin/bash
# Round 4 step 22: the whole GPU suite on the final code (libFM long rows, prediction loads and
# 16-byte attribute records, the default-off launch-order experiments); libFM MCMC / ALS A/B of
# the 16-byte records against HEAD (build_base); the launch-order A/B of step 21 (2 rounds).
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $O/r04s22_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s22_pytest.log; exit 1; }
tail -1 $O/r04s22_pytest.log
B=scalable-bayesian-matrix-factorization_amd
for i in 1 2; do
  for d in build_base build; do
    for m in libfm als; do
      SBMF_LIB=$R/$B/$d/libsbmf.so timeout -k 10 200 python3 bench.py --method $m --steps 3 --warmup 1 --no-cpu > $O/r04s22_${d}_${m}_$i.json 2> $O/r04s22_${d}_${m}_$i.err || { echo "$d $m rc $?"; exit 1; }
    done
  done
done
for f in $O/r04s22_build*_[12].json; do echo "$(basename $f) $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), d['config'].get('test_rmse_after'))")"; done
bash profiles/ab_args.sh r04s22 2 "def=build: gfirst=build:--tune,2147483648 pareval=build:--tune,268435456 both=build:--tune,2415919104" || { echo "ab failed"; exit 1; }
for f in $O/r04s22_{def,gfirst,pareval,both}_[12].json; do echo "$(basename $f) $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(round(d['ms_per_step'],3), round(c['ms_user_half'],3), round(c['ms_item_half'],3), round(c['ms_eval'],3), round(c['ms_hyper'],3), c['test_rmse_after'])")"; done
echo s22 done
