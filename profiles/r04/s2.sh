#!/bin/bash
# Round 4 step 2: config 4 (ML-20M K=200) at 2 / 4 / 8 ranks on one GPU (host comm backend) and the
# degree-sorted 8-rank edge cases; the biased-chain stall; wave-0 phase profiles (KPROF build) of
# k_gres with and without the LDS-DMA prefetch; last, the CLI under rocprofv3 with a normal exit
# (RCCL no longer linked) -- last because a fault at exit ends the call.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_collapse.py -x -v --timeout 900 \
  --timeout-method thread --durations=20 -k "config4 or stall" > $O/r04s2_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s2_pytest.log; exit 1; }
grep -E "passed|failed" $O/r04s2_pytest.log | tail -1
for t in 0 33554432; do
  SBMF_LIB=$R/scalable-bayesian-matrix-factorization_amd/build_kprof/libsbmf.so SBMF_KPROF=1 timeout -k 10 200 \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 --no-load --tune $t > $O/r04s2_kprof_t$t.json 2> $O/r04s2_kprof_t$t.log || { echo "kprof $t rc $?"; exit 1; }
  SBMF_LIB=$R/scalable-bayesian-matrix-factorization_amd/build_kprof/libsbmf.so SBMF_KPROF=1 SBMF_KPROF_SET=1 timeout -k 10 200 \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-ttr --no-f32 --no-load --tune $t > $O/r04s2_kprof1_t$t.json 2> $O/r04s2_kprof1_t$t.log || { echo "kprof1 $t rc $?"; exit 1; }
done
echo kprof ok
# CHECK=1 builds (every row-kernel index checked; a violation is printed and redirected, not
# faulted): the default kernels, then round 3's two-step solve (SBMF_SOLVE2) that faulted in r03s3
for b in build_check build_check_v2; do
  SBMF_LIB=$R/scalable-bayesian-matrix-factorization_amd/$b/libsbmf.so timeout -k 10 200 \
    python3 bench.py --steps 5 --warmup 2 --no-cpu --no-ttr --no-f32 --no-load > $O/r04s2_$b.json 2> $O/r04s2_$b.err \
    || { echo "$b rc $?"; tail -20 $O/r04s2_$b.err; exit 1; }
  echo "$b: $(grep -c 'sbmf check' $O/r04s2_$b.err || true) index violations"
done
zcat tests/golden/ml100k_train.tsv.gz > /tmp/ml100k_train.tsv && zcat tests/golden/ml100k_test.tsv.gz > /tmp/ml100k_test.tsv
cd /tmp && export TMPDIR=/tmp
rc=0
SBMF_EXIT=normal timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04s2_cli_prof -o cli -- \
  $R/scalable-bayesian-matrix-factorization_amd/build/sbmf -task r -train /tmp/ml100k_train.tsv -test /tmp/ml100k_test.tsv \
  -dim 1,1,8 -iter 5 -method mcmc > $O/r04s2_cli_prof.log 2>&1 || rc=$?
echo "cli under rocprofv3 with a normal exit: rc=$rc"
tail -3 $O/r04s2_cli_prof.log
