#!/bin/bash
# r06 step 9: steps 6 and 8 in one call (the pool had no box free for step 6 alone).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash profiles/r06/s8.sh
bash profiles/r06/s6.sh
