"""Worker for tests/test_gpu_rccl.py: the RCCL self-test in a fresh process (RCCL's
communicator set-up then sees only this process's own device state).  Prints one JSON line."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "scalable-bayesian-matrix-factorization_amd"))
from sbmf import Data, FMLearnSBPMF, lib, synth  # noqa: E402
from sbmf import _lib  # noqa: E402


def main():
    nbytes, reps = int(sys.argv[1]), int(sys.argv[2])
    tr, te, _ = synth.generate("ml-1m")
    L = FMLearnSBPMF(num_factor=50, seed=3, rng="philox", recompute_every=0)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=1)
    t = L.timing()
    out = _lib.RcclSelftest()
    rc = lib.sbmf_test_rccl_selftest(L.ctx, nbytes, reps, 60.0, C.byref(out))
    res = {f: getattr(out, f) for f, _ in _lib.RcclSelftest._fields_}
    res.update(rc=rc, err=lib.sbmf_last_error(L.ctx).decode() if rc else "", item_stream_rows=t.kern_rows[1][5])
    L.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
