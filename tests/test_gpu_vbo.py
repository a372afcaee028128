"""GPU parity of the online variational-Bayes learner (-method vb: the
reference's fm_learn_vb_online, src/libfm/src/fm_learn_vb_online.h) against
the oracle (oracle/vbo_oracle.c, itself bit-identical to the compiled
reference learner on these inputs, tests/test_oracle_golden.py).

The learner is deterministic given the shuffle, which the reference-RNG mode
replays draw for draw.  The GPU sums natural parameters in a different order
and uses the collapsed one-hot forms of the reference's cached sums, so the
per-epoch test RMSE must agree within 1e-9 and the posterior means within
1e-8 (absolute) after the last epoch."""
import numpy as np
import pytest

import oracle
from conftest import golden_rmse
from sbmf import Data, FMLearnVBOnline

pytestmark = pytest.mark.gpu


def _run(train, test, epochs, **kw):
    L = FMLearnVBOnline(**kw)
    L.set_data(Data(*train), Data(*test))
    L.learn(sweeps=epochs)
    return L


@pytest.mark.parametrize("data,K,seed,epochs", [("ml100k", 8, 1, 10), ("ml100k", 20, 7, 5), ("ragged", 8, 2, 20)])
def test_vbo_tracks_reference_trajectory(ml100k, ragged, data, K, seed, epochs):
    tr, te = ml100k if data == "ml100k" else ragged
    gold = golden_rmse("ref_vbo_%s_k%d_s%d_e%d.txt" % (data, K, seed, epochs))
    L = _run(tr, te, epochs, num_factor=K, seed=seed)
    err = np.abs(L.rmse_trajectory - gold)
    print("vbo %s K=%d: max |dRMSE| = %.3e" % (data, K, err.max()))
    assert err.max() < 1e-9
    L.close()


def test_vbo_means_match_oracle(ml100k):
    tr, te = ml100k
    K, epochs = 16, 3
    o = oracle.run_vbo(tr, te, K=K, epochs=epochs, seed=3)
    L = _run(tr, te, epochs, num_factor=K, seed=3)
    U, V = L.factors()
    bu, bv, b0 = L.biases()
    I = U.shape[0]
    assert np.abs(U - o["mu_v"][:I]).max() < 1e-8
    assert np.abs(V - o["mu_v"][I:]).max() < 1e-8
    assert np.abs(bu - o["mu_w"][:I]).max() < 1e-8
    assert np.abs(bv - o["mu_w"][I:]).max() < 1e-8
    assert abs(b0 - o["mu0"]) < 1e-10
    assert abs(L.hyper()["tau"] - o["alpha"]) < 1e-9 * o["alpha"]
    np.testing.assert_allclose(L.predict(), o["pred"], rtol=0, atol=1e-9)
    L.close()


def test_vbo_philox_deterministic_and_converges(ml100k):
    """Throughput mode (Philox shuffle and start state): bitwise repeatable,
    and it reaches the reference-stream run's RMSE level."""
    tr, te = ml100k
    a = _run(tr, te, 8, num_factor=8, seed=5, rng="philox")
    b = _run(tr, te, 8, num_factor=8, seed=5, rng="philox")
    assert np.array_equal(a.rmse_trajectory, b.rmse_trajectory)
    gold = golden_rmse("ref_vbo_ml100k_k8_s1_e10.txt")
    assert abs(a.rmse_trajectory[-1] - gold[7]) < 0.01
    a.close()
    b.close()


def test_vbo_continues_across_learn_calls(ml100k):
    tr, te = ml100k
    a = _run(tr, te, 4, num_factor=8, seed=1)
    b = FMLearnVBOnline(num_factor=8, seed=1)
    b.set_data(Data(*tr), Data(*te))
    b.learn(sweeps=2)
    b.learn(sweeps=2)
    assert np.array_equal(a.rmse_trajectory, b.rmse_trajectory)
    a.close()
    b.close()


@pytest.mark.timeout(900)
def test_vbo_ml1m_k200_matches_oracle():
    """BASELINE config 5's factor count (K=200) on the ML-1M shape (sbmf/synth.py), two
    epochs, reference RNG: per-epoch test RMSE within 1e-9 and the posterior means
    within 1e-8 of the oracle (fm_learn_vb_online.h:712-800 update_v, :391-583
    update_all; fm_learn_vb_online_simultaneous.h:148-299 the epoch loop)."""
    from sbmf import synth
    tr, te, dims = synth.generate("ml-1m")
    K, epochs, seed = 200, 2, 3
    o = oracle.run_vbo(tr, te, K=K, epochs=epochs, seed=seed, num_users=dims[0], num_items=dims[1])
    L = FMLearnVBOnline(num_factor=K, seed=seed)
    L.set_data(Data(*tr), Data(*te), num_users=dims[0], num_items=dims[1])
    L.learn(sweeps=epochs)
    err = np.abs(L.rmse_trajectory - o["rmse"])
    U, V = L.factors()
    bu, bv, b0 = L.biases()
    I = U.shape[0]
    print("vbo ml-1m K=200: rmse %s, max|dRMSE| %.2e max|dU| %.2e max|dV| %.2e" % (
        L.rmse_trajectory, err.max(), np.abs(U - o["mu_v"][:I]).max(), np.abs(V - o["mu_v"][I:]).max()))
    assert err.max() < 1e-9
    assert np.abs(U - o["mu_v"][:I]).max() < 1e-8
    assert np.abs(V - o["mu_v"][I:]).max() < 1e-8
    assert np.abs(bu - o["mu_w"][:I]).max() < 1e-8 and np.abs(bv - o["mu_w"][I:]).max() < 1e-8
    assert abs(b0 - o["mu0"]) < 1e-10
    L.close()


@pytest.mark.timeout(900)
def test_vbo_netflix_k200_full_size():
    """BASELINE config 5 at its own size: the Netflix-shaped synthetic set (90.4 M
    train ratings, 480,189 x 17,770), K=200, throughput mode (bench.py --method vb).
    Two epochs: finite test RMSE that falls from epoch 1 to 2, and a second run's
    first epoch bitwise equal to the first run's (the Philox shuffle, the batch
    layout and every reduction are fixed-order)."""
    from sbmf import synth
    tr, te, dims = synth.generate("netflix")
    runs = []
    for epochs in (2, 1):
        L = FMLearnVBOnline(num_factor=200, seed=2015, rng="philox")
        L.set_data(Data(*tr), Data(*te), num_users=dims[0], num_items=dims[1])
        L.learn(sweeps=epochs)
        runs.append(L.rmse_trajectory.copy())
        L.close()
    a, b = runs
    print("vbo netflix K=200: rmse %s / %s" % (a, b))
    assert np.all(np.isfinite(a)) and a[1] < a[0] < 1.5
    assert np.array_equal(a[:1], b)
