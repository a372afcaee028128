"""Every learner gives back what it takes, and RCCL then initialises in the
same long-lived process.

Round 5's whole-suite process failed ncclCommInitRank ("unhandled cuda error")
(profiles/r05/r05s1_suite_summary.txt).  The cause (round 6, r06s2): pytest had
imported torch.distributed while collecting test_multirank_cpu.py, which maps
torch's bundled librccl.so (soname librccl.so.1) bound to torch's own copy of the
HIP / HSA runtime; comm.cpp's dlopen("librccl.so.1") returned that copy.  RCCL is
now opened by path from the directory of the HIP runtime libsbmf is bound to.  This
test imports torch.distributed itself, so it reproduces the round-5 process.
sbmf_test_device_usage counts what the library holds -- device and pinned
buffers, streams, events, contexts, RCCL communicators -- where each is created
and released, next to hipMemGetInfo.  Here 150 learners of every kind (the SBPMF
sampler f64 / f32 / biased, online VB, libFM's MCMC and ALS), half closed
explicitly and half only dropped, must leave those counts where they were;
then the RCCL self-test (a one-rank communicator, the exchange's calls beside
the persistent k_gres grids; reference halves gibbs_sbpmf_final.cpp:453-535)
runs in this process.  A failing ncclCommInitRank reports the same audit in
its message (comm.cpp init_fail)."""
import ctypes as C
import gc

import pytest

from sbmf import Data, FMLearnSBPMF, FMLearnVBOnline, SBMFError, device_usage, lib, synth
from sbmf import _lib

pytestmark = pytest.mark.gpu

COUNTS = ("dev_bytes", "dev_allocs", "pinned_bytes", "pinned_allocs", "streams", "events", "contexts", "comms")


def _kinds():
    return [
        lambda: FMLearnSBPMF(num_factor=8, seed=1),
        lambda: FMLearnSBPMF(num_factor=20, seed=2, rng="philox", precision="f32", recompute_every=0),
        lambda: FMLearnSBPMF(num_factor=8, seed=3, quirks="bias2"),
        lambda: FMLearnVBOnline(num_factor=8, seed=4),
        lambda: FMLearnSBPMF(num_factor=8, seed=5, order="libfm"),
        lambda: FMLearnSBPMF(num_factor=8, seed=6, method="als", regular=(0.0, 0.0, 10.0)),
    ]


def _held(u):
    return {k: u[k] for k in COUNTS}


def _mapped(sub):
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if sub in l})


def test_learners_give_everything_back_then_rccl_initialises_in_process():
    import torch.distributed  # noqa: F401  (maps torch's own librccl.so, as the round-5 suite process had)
    tr, te, _ = synth.generate("ml-100k")
    gc.collect()
    base = device_usage()
    kinds = _kinds()
    for n in range(150):
        L = kinds[n % len(kinds)]()
        L.set_data(Data(*tr), Data(*te))
        L.learn(sweeps=2)
        if n == 5:  # every kind is live at once here: the audit sees them
            held = device_usage()
            assert held["contexts"] >= base["contexts"] + 1 and held["dev_bytes"] > base["dev_bytes"]
        if n % 2 == 0:
            L.close()
        del L  # the other half: released by the learner's __del__ / the collector
        if n % 25 == 24:
            gc.collect()
            assert _held(device_usage()) == _held(base), n
    gc.collect()
    after = device_usage()
    print("device usage before / after 150 learners:", _held(base), _held(after),
          "free %.2f -> %.2f GiB" % (base["device_free"] / 2**30, after["device_free"] / 2**30))
    assert _held(after) == _held(base)
    # the allocator may keep a little; 150 learners must not have eaten the device
    assert after["device_free"] >= base["device_free"] - (256 << 20)

    # the RCCL self-test in this process (a fresh worker in test_gpu_rccl.py)
    t1, t2, _ = synth.generate("ml-1m")
    L = FMLearnSBPMF(num_factor=50, seed=3, rng="philox", recompute_every=0)
    L.set_data(Data(*t1), Data(*t2))
    L.learn(sweeps=1)
    out = _lib.RcclSelftest()
    rc = lib.sbmf_test_rccl_selftest(L.ctx, 16 << 20, 8, 60.0, C.byref(out))
    assert rc == 0, lib.sbmf_last_error(L.ctx).decode()
    assert out.n_calls == 48 and out.bad_bcast == 0 and out.bad_p2p == 0 and out.bad_allgather == 0
    assert device_usage()["comms"] == base["comms"]  # the loopback communicator is gone again
    # the RCCL the library opened sits beside the HIP runtime libsbmf is bound to, not torch's
    hip_dirs = {p.rsplit("/", 1)[0] for p in _mapped("libamdhip64") if "torch" not in p}
    rccl = [p for p in _mapped("librccl") if "torch" not in p]
    assert rccl and all(p.rsplit("/", 1)[0] in hip_dirs for p in rccl), (rccl, hip_dirs)
    # the self-test ran extra item halves on this chain: the context refuses further sweeps
    with pytest.raises(SBMFError, match="rccl_selftest ran extra item halves"):
        L.learn(sweeps=1)
    L.close()
    gc.collect()
    assert _held(device_usage()) == _held(base)
