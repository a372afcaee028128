#!/bin/bash
# Round 3 (session 2) step 13: Gram-block launches enqueued before the streaming launch (tune bit 31) against after it (default); the two lines' test RMSE must agree
set -euo pipefail
mkdir -p gpurun_out
bash profiles/ab_tune_libs.sh r03s13 "build:0 build:2147483648"
echo s13 done
