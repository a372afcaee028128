# Does rocprofv3 (ROCm 7.2) crash at the exit of ANY Python process, or only of ones that load libsbmf?
#   bash profiles/teardown_probe.sh <tag> plain|hip|sbmf|sweep|sweep_unload   -> gpurun_out/<tag>_<mode>.rc
# (sweep: 2 Gibbs sweeps on the ML-100k fixture, context destroyed; sweep_unload: the same, then
# libsbmf.so dlclose()d as bench.py does)
set -u
TAG=$1; MODE=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
case "$MODE" in
  plain) PY='import numpy; print("plain python")' ;;
  hip)   PY='import ctypes; n = ctypes.c_int(); h = ctypes.CDLL("libamdhip64.so.7"); print("hipGetDeviceCount", h.hipGetDeviceCount(ctypes.byref(n)), n.value)' ;;
  sbmf)  PY='import sys; sys.path.insert(0, "'$R'/scalable-bayesian-matrix-factorization_amd"); import sbmf; L = sbmf.FMLearnSBPMF(num_factor=8); L.init(); L.close(); print("libsbmf context created and destroyed")' ;;
  sweep|sweep_unload)
         PY='import sys; sys.path.insert(0, "'$R'/scalable-bayesian-matrix-factorization_amd"); sys.path.insert(0, "'$R'/tests")
import numpy as np, sbmf
from sbmf import _lib
from conftest import read_triples_text
g = "'$R'/tests/golden/"
tr, te = read_triples_text(g + "ml100k_train.tsv.gz"), read_triples_text(g + "ml100k_test.tsv.gz")
L = sbmf.FMLearnSBPMF(num_factor=20, seed=1); L.set_data(sbmf.Data(*tr), sbmf.Data(*te)); L.learn(sweeps=2); L.close()
print("2 sweeps", L.rmse_trajectory)
if "'$MODE'" == "sweep_unload": _lib.unload(); print("unloaded")
for ln in open("/proc/self/maps"):
    if "r-xp" in ln and ".so" in ln: print("MAP", ln.strip())' ;;
esac
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_$MODE" -o "$MODE" -- python3 -c "$PY" > "$O/${TAG}_$MODE.log" 2>&1
echo "rc=$?" > "$O/${TAG}_$MODE.rc"
cat "$O/${TAG}_$MODE.rc"
