#!/bin/bash
# Round 3 (session 2): streaming-threshold A/B after the k_gres solve and issue-order changes
# (rows above the threshold leave the Gram-block bins for k_gres; default 256 f64), two rounds.
set -uo pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for st in 0 96 128 192; do
    timeout -k 10 150 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-ttr --no-f32 --stream-threshold $st \
      > gpurun_out/r03st_${st}_$i.json 2> gpurun_out/r03st_${st}_$i.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "st $st round $i exited $rc"; case $rc in 124|134|137|139) exit $rc ;; esac; fi
  done
done
echo st done
