#!/bin/bash
# r06 step 21: the whole GPU suite on the final tree (after the online-VB timing events).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > "$O/r06s21_suite.log" 2>&1 || { tail -30 "$O/r06s21_suite.log"; exit 1; }
tail -1 "$O/r06s21_suite.log"
