# A/B of built libraries x bench arguments on one box (bench.py f64 only, no CPU / f32 / ttr / load legs):
#   ab_args.sh TAG ROUNDS "label=DIR:arg,arg ..." ; DIR is a build directory under the package,
#   the args (comma-separated) go to bench.py, e.g. "thr128=build:--stream-threshold,128";
#   an arg of the form env:NAME=VALUE sets that environment variable for the run instead.
# ROUNDS passes over the list, interleaved; outputs gpurun_out/<tag>_<label>_<round>.json (+ .err).
# A run that exits with an ordinary error is recorded and the list goes on; an abort, a
# segfault or a time limit ends the script (nothing more runs on the GPU in that call).
set -e
TAG=$1
ROUNDS=$2
B=scalable-bayesian-matrix-factorization_amd
for i in $(seq 1 $ROUNDS); do
  for e in $3; do
    label=${e%%=*}; rest=${e#*=}
    d=${rest%%:*}; args=${rest#*:}
    [ "$args" = "$rest" ] && args=""
    envs=(); bargs=()
    for x in ${args//,/ }; do
      case $x in env:*) envs+=("${x#env:}") ;; *) bargs+=("$x") ;; esac
    done
    rc=0
    env "${envs[@]}" SBMF_LIB=$PWD/$B/$d/libsbmf.so timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 \
      --no-load "${bargs[@]}" > gpurun_out/${TAG}_${label}_$i.json 2> gpurun_out/${TAG}_${label}_$i.err || rc=$?
    if [ $rc -ne 0 ]; then
      echo "ab: $label round $i exited $rc"
      case $rc in 124|134|137|139) exit $rc ;; esac
    fi
  done
done
