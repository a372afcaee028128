"""Several ranks on one GPU (host comm backend instead of RCCL, which refuses
two ranks on one device): the row-block partition, the per-half block
exchange, the point-to-point residual exchange and the fixed-order partial
sums must reproduce a single-rank run bit for bit.  tune=2 runs every rank
(and the single-rank reference) with residuals recomputed from r - own.partner
instead of exchanged.  The biased sampler (quirks bias2) also exchanges the
fresh user / item bias blocks and sums the sweep-start residuals per row."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
from conftest import golden_rmse
from sbmf import Data, FMLearnSBPMF, FMLearnVBOnline, comm_unique_id

pytestmark = pytest.mark.gpu
WORKER = os.path.join(REPO, "tests", "workers", "multirank_worker.py")


def _run_ranks(tmp_path, nranks, args, env=None, timeout=240):
    """Spawn the ranks (host comm backend) and return their output files."""
    old = os.environ.get("SBMF_COMM")
    os.environ["SBMF_COMM"] = "host"
    try:
        uid = comm_unique_id()
    finally:
        if old is None:
            del os.environ["SBMF_COMM"]
        else:
            os.environ["SBMF_COMM"] = old
    outs = [str(tmp_path / ("r%d.npz" % r)) for r in range(nranks)]
    penv = dict(os.environ, **(env or {}))
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), str(nranks), uid.hex(), outs[r]] + args,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=penv)
             for r in range(nranks)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-2000:]
    return outs


@pytest.mark.parametrize("nranks,rng,tune,quirks", [(2, "ref", 0, "final"), (3, "philox", 0, "final"),
                                                   (2, "philox", 2, "final"), (2, "ref", 0, "bias2"),
                                                   (3, "philox", 0, "bias22")])
def test_ranks_on_one_gpu_match_single_rank(ml100k, tmp_path, nranks, rng, tune, quirks):
    K, sweeps, seed = 30, 3, 6
    tr, te = ml100k
    # single rank, same residual form as every rank of the multi-rank run
    L = FMLearnSBPMF(num_factor=K, seed=seed, rng=rng, tune=tune, quirks=quirks)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=sweeps)
    U1, V1 = L.factors()
    rmse1 = L.rmse_trajectory
    biased = quirks in ("bias2", "bias22")
    if biased:
        bu1, bv1, b01 = L.biases()
    L.close()

    outs = _run_ranks(tmp_path, nranks, [str(K), str(sweeps), str(seed), rng, str(tune), quirks])
    for r in range(nranks):
        z = np.load(outs[r])
        # every rank ends with the full, identical factor tables
        assert np.array_equal(z["U"], U1) and np.array_equal(z["V"], V1), \
            (r, np.abs(z["U"] - U1).max(), np.abs(z["V"] - V1).max())
        assert np.array_equal(z["rmse"], rmse1)
        if biased:
            assert np.array_equal(z["bu"], bu1) and np.array_equal(z["bv"], bv1) and z["b0"][0] == b01


@pytest.mark.parametrize("nranks,quirks", [(3, "final"), (2, "bias2")])
def test_pipelined_ranks_match_single_rank(ml100k, tmp_path, nranks, quirks):
    """sbmf_config.pipeline on every rank (bench.py's setting at N > 1): each rank queues sweep
    s+1's start -- its user half and that half's block broadcasts and residual exchange --
    before reporting sweep s.  The ranks still end with the single-rank chain bit for bit."""
    K, sweeps, seed = 30, 4, 6
    tr, te = ml100k
    L = FMLearnSBPMF(num_factor=K, seed=seed, rng="philox", quirks=quirks)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=sweeps)
    U1, V1 = L.factors()
    rmse1 = L.rmse_trajectory
    L.close()
    outs = _run_ranks(tmp_path, nranks, [str(K), str(sweeps), str(seed), "philox", "0", quirks],
                      env={"SBMF_WORKER_PIPELINE": "1"})
    for r in range(nranks):
        z = np.load(outs[r])
        assert np.array_equal(z["U"], U1) and np.array_equal(z["V"], V1), r
        assert np.array_equal(z["rmse"], rmse1)


@pytest.mark.parametrize("nranks,data,K,seed,epochs,rng", [(2, "ml100k", 8, 1, 10, "ref"), (3, "ml100k", 20, 7, 5, "ref"),
                                                           (3, "ragged", 8, 2, 20, "ref"), (2, "ml100k", 8, 5, 4, "philox")])
def test_vb_ranks_on_one_gpu(ml100k, ragged, tmp_path, nranks, data, K, seed, epochs, rng):
    """Online VB over several ranks (users split into ranges, the item rows'
    sums all-gathered and added in rank order): every rank ends with the same
    means, the per-epoch test RMSE tracks the reference learner (golden, 1e-9,
    as one rank does) and one rank's run to rounding (item sums added rank by
    rank instead of in one group reduction)."""
    tr, te = ml100k if data == "ml100k" else ragged
    L = FMLearnVBOnline(num_factor=K, seed=seed, rng=rng)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=epochs)
    U1, V1 = L.factors()
    bu1, bv1, b01 = L.biases()
    rmse1, pred1 = L.rmse_trajectory, L.predict()
    L.close()
    outs = _run_ranks(tmp_path, nranks, [str(K), str(epochs), str(seed), rng, "0", "final", "vb"],
                      env={"SBMF_WORKER_DATA": data})
    z0 = np.load(outs[0])
    for r in range(1, nranks):  # identical on every rank
        z = np.load(outs[r])
        for k in ("U", "V", "bu", "bv", "b0", "rmse", "pred"):
            assert np.array_equal(z[k], z0[k]), (r, k)
    print("vb %d ranks %s K=%d: max|dRMSE| %.2e max|dU| %.2e max|dV| %.2e" % (
        nranks, data, K, np.abs(z0["rmse"] - rmse1).max(), np.abs(z0["U"] - U1).max(), np.abs(z0["V"] - V1).max()))
    assert np.abs(z0["rmse"] - rmse1).max() < 1e-11
    assert np.abs(z0["U"] - U1).max() < 1e-9 and np.abs(z0["V"] - V1).max() < 1e-9
    assert np.abs(z0["bu"] - bu1).max() < 1e-9 and np.abs(z0["bv"] - bv1).max() < 1e-9
    assert abs(z0["b0"][0] - b01) < 1e-11
    assert np.abs(z0["pred"] - pred1).max() < 1e-9
    if rng == "ref":
        gold = golden_rmse("ref_vbo_%s_k%d_s%d_e%d.txt" % (data, K, seed, epochs))
        assert np.abs(z0["rmse"] - gold).max() < 1e-9


@pytest.mark.parametrize("nranks,run", [(2, 0), (3, 1), (2, 2), (3, 3), (2, 4)])
def test_libfm_ranks_on_one_gpu(ml100k, ragged, tmp_path, nranks, run):
    """libFM's own MCMC / ALS chain over several ranks (users split into
    ranges, item rows' sums all-gathered and added in rank order, the owned
    users' w and v broadcast after each sweep): identical on every rank, one
    rank's run to rounding, and bin/libFM's printed digits (tests/golden)."""
    from test_gpu_libfm import _within_printed
    from test_oracle_libfm import RUNS, golden_name
    method, dname, dim, seed, iters, reg = RUNS[run]
    tr, te = ml100k if dname == "ml100k" else ragged
    k0, k1, K = (int(x) for x in dim.split(","))
    regular = reg or "0,0,0"
    L = FMLearnSBPMF(num_factor=K, seed=seed, order="libfm", method="als" if method == "als" else "mcmc", k0=k0,
                     k1=k1, regular=tuple(float(x) for x in regular.split(",")), init_stdev=0.1)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=iters)
    U1, V1 = L.factors()
    test1 = L.rmse_trajectory
    train1 = np.array([h["rmse_train"] for h in L.history])
    pred1 = L.predict()
    L.close()
    outs = _run_ranks(tmp_path, nranks, [str(K), str(iters), str(seed), "ref", "0", "%d,%d;%s" % (k0, k1, regular),
                                         "als" if method == "als" else "libfm"], env={"SBMF_WORKER_DATA": dname})
    z0 = np.load(outs[0])
    for r in range(1, nranks):
        z = np.load(outs[r])
        for k in ("U", "V", "bu", "bv", "b0", "rmse", "rmse_train", "pred"):
            assert np.array_equal(z[k], z0[k]), (r, k)
    print("libfm %s %d ranks: max|dTest| %.2e max|dTrain| %.2e max|dU| %.2e max|dV| %.2e" % (
        golden_name(method, dname, dim, seed, iters), nranks, np.abs(z0["rmse"] - test1).max(),
        np.abs(z0["rmse_train"] - train1).max(), np.abs(z0["U"] - U1).max(), np.abs(z0["V"] - V1).max()))
    np.testing.assert_allclose(z0["rmse"], test1, rtol=1e-9, atol=0)
    np.testing.assert_allclose(z0["rmse_train"], train1, rtol=1e-9, atol=0)
    assert np.abs(z0["U"] - U1).max() < 1e-8 and np.abs(z0["V"] - V1).max() < 1e-8
    assert np.abs(z0["pred"] - pred1).max() < 1e-9
    with open(os.path.join(REPO, "tests", "golden", golden_name(method, dname, dim, seed, iters) + ".txt")) as f:
        lines = f.read().splitlines()
    assert _within_printed(z0["rmse_train"], [float(l.split("Train=")[1].split()[0]) for l in lines])
    assert _within_printed(z0["rmse"], [float(l.split("Test=")[1]) for l in lines])


_C4 = {}  # (relabel) -> (cache dir, data, single-rank digests): one single-rank run per id order


def _config4(tmp_path_factory, relabel):
    """ML-20M K=200 synthetic (ids shuffled, or renumbered heaviest-first) and the
    single-rank chain's U / V digests, RMSE and tau after one reference-stream sweep."""
    import hashlib
    from sbmf import synth
    if relabel in _C4:
        return _C4[relabel]
    cache = os.environ.get("SBMF_SYNTH_CACHE") or str(tmp_path_factory.mktemp("synth"))
    old = os.environ.get("SBMF_SYNTH_CACHE")
    os.environ["SBMF_SYNTH_CACHE"] = cache  # generated once here, read back by the ranks
    try:
        tr, te, dims = synth.generate("ml-20m")
    finally:
        if old is None:
            del os.environ["SBMF_SYNTH_CACHE"]
        else:
            os.environ["SBMF_SYNTH_CACHE"] = old
    if relabel == "degree":
        tr, te, dims = synth.relabel_by_degree(tr, te, dims)
    L = FMLearnSBPMF(num_factor=200, seed=1, rng="ref")
    L.set_data(Data(*tr), Data(*te), num_users=dims[0], num_items=dims[1])
    L.learn(sweeps=1)
    U1, V1 = L.factors()
    ref = {"rmse": L.rmse_trajectory, "tau": np.array([h["tau"] for h in L.history]),
           "U": np.frombuffer(hashlib.sha256(np.ascontiguousarray(U1).tobytes()).digest(), np.uint8),
           "V": np.frombuffer(hashlib.sha256(np.ascontiguousarray(V1).tobytes()).digest(), np.uint8)}
    L.close()
    del U1, V1
    _C4[relabel] = (cache, tr, dims, ref)
    return _C4[relabel]


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("nranks,relabel", [(2, "none"), (4, "none"), (8, "none"), (8, "degree")])
def test_config4_ml20m_k200_ranks_match_single_rank(tmp_path, tmp_path_factory, nranks, relabel):
    """BASELINE config 4's split (ML-20M K=200, user and item row blocks over ranks,
    /root/reference/src/libfm/gibbs_sbpmf_final.cpp:453-535 sharded) at its own shape
    and at 2, 4 and its own 8 ranks, reference stream, one sweep, default 2 stages per
    half: every rank (host comm backend, all on one GPU) ends with the single-rank U, V,
    tau and RMSE bit for bit.  The single-rank run is pinned to the oracle by
    test_gpu_production.py::test_ml20m_k200_reference_stream_one_sweep.  With shuffled
    ids every rank owns split item rows (over 2048 ratings: co-resident chunks) and
    residuals of over a million ratings cross the cuts.  With ids renumbered
    heaviest-first (relabel "degree") the 8-way cut has the edge cases a shuffled order
    never produces: an empty item block (rank 0), item blocks of only split rows and
    of no split row, a user block of only Gram-block rows (every row <= 256 ratings)."""
    from sbmf import partition_rows
    cache, tr, dims, ref = _config4(tmp_path_factory, relabel)
    I, J = dims
    iptr = np.concatenate([[0], np.cumsum(np.bincount(tr[1], minlength=J))]).astype(np.uint64)
    uptr = np.concatenate([[0], np.cumsum(np.bincount(tr[0], minlength=I))]).astype(np.uint64)
    ib, ub = partition_rows(iptr, nranks), partition_rows(uptr, nranks)
    ideg, udeg = np.diff(iptr), np.diff(uptr)
    imax = [int(ideg[ib[r]:ib[r + 1]].max()) if ib[r + 1] > ib[r] else 0 for r in range(nranks)]
    umax = [int(udeg[ub[r]:ub[r + 1]].max()) if ub[r + 1] > ub[r] else 0 for r in range(nranks)]
    user_rank = np.searchsorted(np.asarray(ub[1:-1], np.int64), tr[0].astype(np.int64), side="right")
    item_rank = np.searchsorted(np.asarray(ib[1:-1], np.int64), tr[1].astype(np.int64), side="right")
    cross = int((user_rank != item_rank).sum())
    if relabel == "none":
        assert min(imax) > 2048, imax  # every rank owns split item rows
        assert cross > 1_000_000
    else:
        assert nranks == 8
        assert ib[1] == ib[0], list(ib)  # rank 0 owns no item row
        assert any(m <= 2048 for m in imax[1:]), imax  # an item block without a split row
        assert udeg[ub[-2]:ub[-1]].max() <= 256, umax  # a user block of Gram-block rows only
        assert ideg[ib[1]:ib[2]].min() > 2048, imax  # an item block of split rows only
    env = {"SBMF_WORKER_DATA": "synth:ml-20m", "SBMF_WORKER_DIGEST": "1", "SBMF_SYNTH_CACHE": cache}
    if relabel == "degree":
        env["SBMF_WORKER_RELABEL"] = "degree"
    outs = _run_ranks(tmp_path, nranks, ["200", "1", "1", "ref", "0", "final"], env=env, timeout=900)
    for r in range(nranks):
        z = np.load(outs[r])
        assert np.array_equal(z["U"], ref["U"]) and np.array_equal(z["V"], ref["V"]), r
        assert np.array_equal(z["rmse"], ref["rmse"]) and np.array_equal(z["tau"], ref["tau"]), r
    print("config 4 split, %d ranks (%s ids): item blocks %s (max degree %s), user blocks %s (max degree %s), "
          "%d ratings cross the cuts, rmse %s" % (nranks, relabel, list(ib), imax, list(ub), umax, cross, ref["rmse"]))


@pytest.mark.parametrize("stages", [2, 3])
def test_stages_do_not_change_the_chain(ml100k, stages):
    """One rank with its half-sweeps cut into stages (the multi-GPU pipeline's unit:
    each stage's launches, then its exchange while the next stage computes) gives the
    single-stage chain bit for bit: a row's draws do not depend on which launch runs it."""
    tr, te = ml100k
    out = []
    for st in (1, stages):
        old = os.environ.get("SBMF_STAGES")
        os.environ["SBMF_STAGES"] = str(st)
        try:
            L = FMLearnSBPMF(num_factor=30, seed=6, rng="philox", quirks="bias2", stream_threshold=40, split_chunk=64)
            L.set_data(Data(*tr), Data(*te))
        finally:
            if old is None:
                del os.environ["SBMF_STAGES"]
            else:
                os.environ["SBMF_STAGES"] = old
        L.learn(sweeps=3)
        out.append((L.factors(), L.biases(), L.rmse_trajectory, L.timing().kern_rows[1][5]))
        L.close()
    (U1, V1), b1, r1, n1 = out[0]
    (U2, V2), b2, r2, n2 = out[1]
    assert np.array_equal(U1, U2) and np.array_equal(V1, V2) and np.array_equal(r1, r2)
    assert np.array_equal(b1[0], b2[0]) and np.array_equal(b1[1], b2[1]) and b1[2] == b2[2]
    assert n1 == n2 > 0  # the streaming rows are counted over the stages


@pytest.mark.parametrize("stages", [1, 3])
def test_ranks_with_stage_count(ml100k, tmp_path, stages):
    """2 ranks (host comm backend) with the exchange unpipelined (1 stage) and cut into 3
    stages: both equal the single-rank chain bit for bit."""
    K, sweeps, seed = 30, 3, 6
    tr, te = ml100k
    L = FMLearnSBPMF(num_factor=K, seed=seed, rng="philox")
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=sweeps)
    U1, V1 = L.factors()
    rmse1 = L.rmse_trajectory
    L.close()
    outs = _run_ranks(tmp_path, 2, [str(K), str(sweeps), str(seed), "philox", "0", "final"],
                      env={"SBMF_STAGES": str(stages)})
    for r in range(2):
        z = np.load(outs[r])
        assert np.array_equal(z["U"], U1) and np.array_equal(z["V"], V1) and np.array_equal(z["rmse"], rmse1)
