#!/bin/bash
# Round 3 (session 2) step 12: the item half's two streaming sets side by side (default) against one after the other
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03s12_pytest.log 2>&1
echo pytest ok
bash profiles/ab_tune_libs.sh r03s12 "build:0 build:1073741824 build:536870912"
echo s12 done
