"""The multi-GPU transport's RCCL calls on one GPU, and one rank's stage compute.

RCCL refuses two ranks on one device, so the exchange (comm.cpp) cannot run
between peers here.  What one GPU can show:

* sbmf_test_rccl_selftest: a one-rank RCCL communicator created through the
  library's own dlopen/dlsym table issues the exchange's exact calls -- grouped
  in-place ncclBroadcast over adjacent blocks (bcast_stage), grouped
  ncclSend/ncclRecv (alltoallv, here to the rank itself), ncclAllGather -- on the
  multi-GPU comm stream while the item half's persistent k_gres grids run on the
  compute streams, as in the pipelined half (stage p's exchange beside stage
  p+1's compute; reference halves gibbs_sbpmf_final.cpp:453-535).  Every byte is
  checked and the comm stream must finish within a deadline.
* sbmf_test_virtual_rank: rank r of an N-rank run on this GPU with the exchange
  skipped runs exactly its own blocks, stages, bins and tasks (timing only)."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

from sbmf import Data, FMLearnSBPMF, lib, synth
from sbmf import _lib

pytestmark = pytest.mark.gpu
WORKER = os.path.join(REPO, "tests", "workers", "rccl_selftest.py")


def _learner(shape="ml-1m", K=50, **kw):
    tr, te, _ = synth.generate(shape)
    L = FMLearnSBPMF(num_factor=K, seed=3, rng="philox", recompute_every=0, **kw)
    return L, Data(*tr), Data(*te)


def test_rccl_calls_beside_persistent_kgres_grids():
    """In a fresh process (tests/workers/rccl_selftest.py), without torch: the same self-test
    as test_gpu_resources.py's in-process one, from a clean start.  (Round 5 moved it here
    after ncclCommInitRank failed inside the suite process; the cause was torch's bundled
    librccl.so answering dlopen("librccl.so.1"), fixed in comm.cpp in round 6.)"""
    env = dict(os.environ, NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"))
    p = subprocess.run([sys.executable, WORKER, str(16 << 20), "8"], capture_output=True, text=True, timeout=180,
                       env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["rc"] == 0, out["err"] + "\n" + p.stderr[-3000:]
    print("rccl self-test: half %.3f ms x8, rccl %.3f ms, rccl end %.3f ms, overlapped %d, calls %d"
          % (out["ms_half"], out["ms_rccl"], out["ms_rccl_end"], out["overlapped"], out["n_calls"]))
    assert out["item_stream_rows"] > 0  # the item half has streaming (k_gres) rows
    assert out["n_calls"] == 8 * 6
    assert out["bad_bcast"] == 0 and out["bad_p2p"] == 0 and out["bad_allgather"] == 0
    assert out["ms_half"] > 0 and out["ms_rccl"] > 0


def test_rccl_selftest_argument_checks():
    L, tr, te = _learner("ml-100k", K=8)
    out = _lib.RcclSelftest()
    L.init()
    assert lib.sbmf_test_rccl_selftest(L.ctx, 1 << 20, 1, 10.0, C.byref(out)) != 0  # not prepared
    L.set_data(tr, te)
    assert lib.sbmf_test_rccl_selftest(L.ctx, 100, 1, 10.0, C.byref(out)) != 0  # not a multiple of 64
    L.close()


def test_virtual_rank_runs_its_stages():
    """Config-4-like partitioning (8 ranks, the default 2 stages per half) of the ML-1M-shaped
    set: every virtual rank runs; its stage times are positive and the stages add up to about
    the half."""
    tr, te, _ = synth.generate("ml-1m")
    for r in (0, 7):
        L = FMLearnSBPMF(num_factor=50, seed=3, rng="philox", recompute_every=0)
        L.init()
        assert lib.sbmf_test_virtual_rank(L.ctx, 8, r) == 0
        L.set_data(Data(*tr), Data(*te))
        L.learn(sweeps=2)
        ns = C.c_uint32()
        assert lib.sbmf_test_stage_ms(L.ctx, None, 0, C.byref(ns)) == 0
        assert ns.value == 2  # sbmf.cpp: two stages per half for several ranks
        n = ns.value
        ms = np.zeros(2 * n)
        assert lib.sbmf_test_stage_ms(L.ctx, ms.ctypes.data_as(C.POINTER(C.c_double)), 2 * n, C.byref(ns)) == 0
        assert np.all(ms > 0) and np.all(np.isfinite(ms)), ms
        t = L.timing()
        assert ms[:n].sum() <= t.ms_user_half * 1.05 + 0.05 and ms[n:].sum() <= t.ms_item_half * 1.05 + 0.05
        L.close()
