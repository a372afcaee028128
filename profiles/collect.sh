#!/bin/bash
# One measurement pass on a 1-GPU MI355X box (run from the repo root via gpurun):
#   bash profiles/collect.sh <tag> bench   default bench line (f64 + f32 + CPU baseline + time-to-RMSE)
#   bash profiles/collect.sh <tag> trace   rocprofv3 --kernel-trace --stats of a bench run
#   bash profiles/collect.sh <tag> fetch   --pmc FETCH_SIZE      (each counter pass on its own,
#   bash profiles/collect.sh <tag> write   --pmc WRITE_SIZE       never combined with other
#   bash profiles/collect.sh <tag> l2      --pmc TCC_HIT/MISS     tracing domains)
#   bash profiles/collect.sh <tag> lds     --pmc SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (bank-conflict share)
#   bash profiles/collect.sh <tag> gather  --pmc FETCH_SIZE over tests/hip/gather_bench (known bytes: calibration)
# Outputs land in gpurun_out/<tag>_<pass>*.  Since round 4 libsbmf loads RCCL only for a
# multi-GPU communicator (dlopen), and a single-GPU process exits normally under
# rocprofv3 (profiles/r04/r04s2_cli_rocprof_kernel_stats.csv): a plain exit, the profiler's
# own exit handler writes the files (SBMF_EXIT=guard would restore round 3's _Exit guard).
set -euo pipefail
TAG=${1:-r01}
PASS=${2:-bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py"
SHORT="--no-cpu --no-f32 --no-ttr --no-load ${BENCH_ARGS:-}"  # BENCH_ARGS: e.g. "--shape ml-10m --K 100"
case "$PASS" in
  bench) timeout -k 10 500 python3 "$BENCH" ${BENCH_ARGS:-} > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" ;;
  trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_trace" -o "$TAG" -- \
           python3 "$BENCH" --steps 10 --warmup 2 $SHORT > "$O/${TAG}_trace.log" 2>&1 ;;
  fetch) timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$O/${TAG}_pmc_fetch" -o "$TAG" -- \
           python3 "$BENCH" --steps 2 --warmup 1 $SHORT > "$O/${TAG}_pmc_fetch.log" 2>&1 ;;
  write) timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$O/${TAG}_pmc_write" -o "$TAG" -- \
           python3 "$BENCH" --steps 2 --warmup 1 $SHORT > "$O/${TAG}_pmc_write.log" 2>&1 ;;
  l2)    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum -d "$O/${TAG}_pmc_l2" -o "$TAG" -- \
           python3 "$BENCH" --steps 2 --warmup 1 $SHORT > "$O/${TAG}_pmc_l2.log" 2>&1 ;;
  sq)    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$O/${TAG}_pmc_sq" -o "$TAG" -- \
           python3 "$BENCH" --steps 2 --warmup 1 $SHORT > "$O/${TAG}_pmc_sq.log" 2>&1 ;;
  lds)   timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES -d "$O/${TAG}_pmc_lds" -o "$TAG" -- \
           python3 "$BENCH" --steps 2 --warmup 1 $SHORT > "$O/${TAG}_pmc_lds.log" 2>&1 ;;
  gather) timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$O/${TAG}_pmc_gather" -o "$TAG" -- \
           "$R/tests/hip/gather_bench" > "$O/${TAG}_pmc_gather.log" 2>&1 ;;
  sq2)   timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM -d "$O/${TAG}_pmc_sq2" -o "$TAG" -- \
           python3 "$BENCH" --steps 2 --warmup 1 $SHORT > "$O/${TAG}_pmc_sq2.log" 2>&1 ;;
  *) echo "unknown pass $PASS" >&2; exit 2 ;;
esac
echo "collect.sh $TAG $PASS done"
