#!/bin/bash
# Round 4 step 38: the whole GPU suite and smoke() on the round's last HEAD, then one short bench line.
set -uo pipefail
R=$PWD; O=$R/gpurun_out; mkdir -p $O
export SBMF_SYNTH_CACHE=/tmp/sbmf_synth
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/r04s38_pytest.log 2>&1 || { echo "pytest rc $?"; tail -40 $O/r04s38_pytest.log; exit 1; }
tail -1 $O/r04s38_pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r04s38_smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 $O/r04s38_smoke.log; exit 1; }
tail -1 $O/r04s38_smoke.log
timeout -k 10 150 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-ttr --no-f32 --no-load > $O/r04s38_bench.json 2> $O/r04s38_bench.err || { echo "bench rc $?"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/r04s38_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"
echo s38 done
