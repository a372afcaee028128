"""libFM-order MCMC and ALS on the GPU (sbmf_config.method LIBFM_MCMC / ALS,
csrc/fmm.hip + fmm.cpp) against the reference: libFM compiled unmodified
(tests/golden/ref_libfm_*: its "#Iter=" lines and -out predictions, 6
significant digits) and the oracle restatement (oracle/fmm_oracle.c, pinned to
those files by tests/test_oracle_libfm.py) at full precision."""
import gzip
import os

import numpy as np
import pytest

import oracle
from conftest import GOLD, gpu_available
from sbmf import Data, FMLearnSBPMF
from test_oracle_libfm import RUNS, golden_name

pytestmark = pytest.mark.gpu


def _gpu(tr, te, K, iters, seed, method, k0, k1, regular, rng="ref"):
    L = FMLearnSBPMF(num_factor=K, seed=seed, rng=rng, method="als" if method == "als" else "mcmc", order="libfm",
                     k0=k0, k1=k1, regular=regular, init_stdev=0.1)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=iters)
    return L


def _within_printed(x, printed):
    """|x - printed| within half a unit of printed's 6th significant digit."""
    p = np.asarray(printed, float)
    ulp6 = 10.0 ** (np.floor(np.log10(np.abs(p))) - 5)
    return np.all(np.abs(np.asarray(x) - p) <= 0.5 * ulp6 + 1e-12)


@pytest.mark.parametrize("run", RUNS, ids=[golden_name(*r[:5]) for r in RUNS])
def test_libfm_chain_matches_reference(run, ml100k, ragged):
    assert gpu_available()
    method, dname, dim, seed, iters, reg = run
    tr, te = ml100k if dname == "ml100k" else ragged
    k0, k1, K = (int(x) for x in dim.split(","))
    regular = tuple(float(x) for x in reg.split(",")) if reg else (0.0, 0.0, 0.0)
    L = _gpu(tr, te, K, iters, seed, method, k0, k1, regular)
    o = oracle.run_fmm(tr, te, K=K, iters=iters, seed=seed, method=method, k0=k0, k1=k1, regular=regular)
    h = L.history
    train = np.array([x["rmse_train"] for x in h])
    test = np.array([x["rmse_avg"] for x in h])
    # full precision against the oracle (same RNG stream; only reduction order differs)
    np.testing.assert_allclose(train, o["rmse_train"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(test, o["rmse_test"], rtol=1e-9, atol=0)
    U, V = L.factors()
    I = U.shape[0]
    np.testing.assert_allclose(U, o["v"][:, :I].T, rtol=0, atol=1e-8)
    np.testing.assert_allclose(V, o["v"][:, I:I + V.shape[0]].T, rtol=0, atol=1e-8)
    pred = L.predict()
    np.testing.assert_allclose(pred, o["pred"], rtol=0, atol=1e-9)
    # against libFM's own output (6 significant digits)
    with open(os.path.join(GOLD, golden_name(method, dname, dim, seed, iters) + ".txt")) as f:
        lines = f.read().splitlines()
    ref_train = [float(l.split("Train=")[1].split()[0]) for l in lines]
    ref_test = [float(l.split("Test=")[1]) for l in lines]
    assert _within_printed(train, ref_train) and _within_printed(test, ref_test)
    with gzip.open(os.path.join(GOLD, golden_name(method, dname, dim, seed, iters) + "_pred.txt.gz"), "rt") as f:
        ref_pred = np.array([float(x) for x in f.read().split()])
    assert _within_printed(pred, ref_pred)


@pytest.mark.parametrize("method", ["mcmc", "als"])
def test_libfm_long_rows_in_chunks_match_oracle(method, ml100k, monkeypatch):
    """One rank cuts the long-row bin's rows into chunks (sums per chunk, the draw per row
    from the chunk sums in chunk order, then each chunk's residual update).  ML-100k has no
    row over the default 4096-case bound: SBMF_FMM_LONG=256 / SBMF_FMM_CHUNK=64 put its
    users and items of more than 256 ratings into 5-12 chunks each, on both sides (the user
    side's chunks replay the item pass's pending update from the record the draw replaced)."""
    assert gpu_available()
    tr, te = ml100k
    regular = (0.0, 0.0, 10.0) if method == "als" else (0.0, 0.0, 0.0)
    monkeypatch.setenv("SBMF_FMM_LONG", "256")
    monkeypatch.setenv("SBMF_FMM_CHUNK", "64")
    L = _gpu(tr, te, 8, 5, 1, method, 1, 1, regular)
    monkeypatch.delenv("SBMF_FMM_LONG")
    monkeypatch.delenv("SBMF_FMM_CHUNK")
    o = oracle.run_fmm(tr, te, K=8, iters=5, seed=1, method=method, k0=1, k1=1, regular=regular)
    h = L.history
    np.testing.assert_allclose([x["rmse_train"] for x in h], o["rmse_train"], rtol=1e-9, atol=0)
    np.testing.assert_allclose([x["rmse_avg"] for x in h], o["rmse_test"], rtol=1e-9, atol=0)
    U, V = L.factors()
    I = U.shape[0]
    np.testing.assert_allclose(U, o["v"][:, :I].T, rtol=0, atol=1e-8)
    np.testing.assert_allclose(V, o["v"][:, I:I + V.shape[0]].T, rtol=0, atol=1e-8)
    np.testing.assert_allclose(L.predict(), o["pred"], rtol=0, atol=1e-9)


def test_libfm_als_is_deterministic_and_biases_exposed(ml100k):
    tr, te = ml100k
    a = _gpu(tr, te, 8, 4, 3, "als", 1, 1, (0.0, 0.0, 10.0))
    b = _gpu(tr, te, 8, 4, 3, "als", 1, 1, (0.0, 0.0, 10.0))
    assert [h["rmse_avg"] for h in a.history] == [h["rmse_avg"] for h in b.history]
    o = oracle.run_fmm(tr, te, K=8, iters=4, seed=3, method="als", regular=(0.0, 0.0, 10.0))
    bu, bv, b0 = a.biases()
    np.testing.assert_allclose(np.concatenate([bu, bv]), o["w"][:len(bu) + len(bv)], rtol=0, atol=1e-9)
    assert abs(b0 - o["w0"]) < 1e-9
    assert a.history[-1]["tau"] == 1.0  # ALS: alpha stays alpha_0


def test_libfm_philox_mode_deterministic_and_learns(ml100k):
    tr, te = ml100k
    a = _gpu(tr, te, 8, 12, 5, "mcmc", 1, 1, (0.0, 0.0, 0.0), rng="philox")
    b = _gpu(tr, te, 8, 12, 5, "mcmc", 1, 1, (0.0, 0.0, 0.0), rng="philox")
    ra = np.array([h["rmse_avg"] for h in a.history])
    assert np.array_equal(ra, np.array([h["rmse_avg"] for h in b.history]))
    # the running mean of the reference chain on ML-100k K=8 settles near 0.93-0.95 within 10 iterations
    assert ra[-1] < 0.97 and ra[-1] < ra[0]


def test_libfm_trailing_unrated_items_read_zero(ml100k):
    """sbmf_set_dims with more items than libFM's attribute count (ids past every
    rated one): those items have no attribute, so factors and biases read 0 and
    the rated items are unchanged (no read past the attribute table)."""
    tr, te = ml100k
    I = int(max(tr[0].max(), te[0].max())) + 1
    J = int(max(tr[1].max(), te[1].max())) + 1
    extra = 37
    runs = []
    for nj in (0, J + extra):
        L = FMLearnSBPMF(num_factor=4, seed=2, method="mcmc", order="libfm", init_stdev=0.1)
        L.set_data(Data(*tr), Data(*te), num_users=I, num_items=nj)
        L.learn(sweeps=2)
        runs.append((L.factors(), L.biases()))
    (U0, V0), (bu0, bv0, _) = runs[0]
    (U1, V1), (bu1, bv1, _) = runs[1]
    assert V1.shape[0] == J + extra and bv1.shape[0] == J + extra
    assert np.array_equal(U0, U1) and np.array_equal(bu0, bu1)
    assert np.array_equal(V0, V1[:V0.shape[0]]) and np.array_equal(bv0, bv1[:bv0.shape[0]])
    # item J is libFM's phantom attribute (num_all_attribute = max feature id + 1 + 1,
    # libfm.cpp:328): it exists, is drawn from its prior and keeps its value; past it, nothing
    assert V1[J].any()
    assert not V1[J + 1:].any() and not bv1[J + 1:].any()
