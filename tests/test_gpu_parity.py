"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's own golden trajectories.

Tolerances (north_star: test RMSE within 1e-3 of the reference at fixed
seed after equal sweeps):
  * f64, reference RNG stream: per-sweep running-mean test RMSE within 1e-6
    of the compiled reference over all 100 sweeps (ML-100k, K=20), factors
    within 1e-7 of the oracle after 5 sweeps.  The only differences are
    floating-point summation order (wave reductions, carried residuals).
  * f32, reference RNG stream: RMSE within 1e-3 (the north-star bar).
"""
import numpy as np
import pytest

import oracle
from conftest import golden_rmse
from sbmf import Data, FMLearnSBPMF

pytestmark = pytest.mark.gpu


def _run(train, test, sweeps, **kw):
    L = FMLearnSBPMF(**kw)
    L.set_data(Data(*train), Data(*test))
    L.learn(sweeps=sweeps)
    return L


@pytest.mark.parametrize("seed", [1, 7])
def test_f64_ref_stream_tracks_reference_100_sweeps(ml100k, seed):
    tr, te = ml100k
    gold = golden_rmse("ref_final_ml100k_k20_s%d.txt" % seed)
    L = _run(tr, te, 100, num_factor=20, seed=seed)
    traj = L.rmse_trajectory
    assert traj.shape == gold.shape
    err = np.abs(traj - gold)
    print("max |dRMSE| over 100 sweeps = %.3e" % err.max())
    assert err.max() < 1e-6


def test_f64_factors_match_oracle_after_5_sweeps(ml100k):
    """The MFMA Gram-block kernels (every row of ML-100k at K=20 is in a Gram-block bin or k_gres)."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=20, iters=5, seed=1)
    L = _run(tr, te, 5, num_factor=20, seed=1)
    U, V = L.factors()
    h = L.hyper()
    assert np.abs(U - o["U"]).max() < 1e-7
    assert np.abs(V - o["V"]).max() < 1e-7
    assert abs(h["tau"] - o["tau"][-1]) < 1e-9 * o["tau"][-1]
    np.testing.assert_allclose(L.rmse_trajectory, o["rmse"], rtol=0, atol=1e-9)


def test_sbpmf2_quirks_track_reference(ml100k):
    tr, te = ml100k
    gold = golden_rmse("ref_sbpmf2_ml100k_k20_s1.txt")
    L = _run(tr, te, 100, num_factor=20, seed=1, quirks="sbpmf2")
    assert np.abs(L.rmse_trajectory - gold).max() < 1e-6


@pytest.mark.parametrize("name,quirks,seed", [("ref_final_ragged_k20_s1.txt", "final", 1),
                                              ("ref_sbpmf2_ragged_k20_s5.txt", "sbpmf2", 5)])
def test_ragged_edge_cases_track_reference(ragged, name, quirks, seed):
    """Empty user/item rows, a test-only user id beyond the train range,
    single-rating rows, half-star ratings."""
    tr, te = ragged
    gold = golden_rmse(name)
    L = _run(tr, te, 100, num_factor=20, seed=seed, quirks=quirks)
    assert np.abs(L.rmse_trajectory - gold).max() < 1e-6


@pytest.mark.parametrize("tune", [0, 2048])
def test_f32_ref_stream_within_north_star_tolerance(ml100k, tune):
    """f32 against the reference trajectory; tune bit 11 runs the f32 rows of 17..512 ratings
    on the Gram-block kinds instead of k_grow workgroups."""
    tr, te = ml100k
    gold = golden_rmse("ref_final_ml100k_k20_s1.txt")
    L = _run(tr, te, 100, num_factor=20, seed=1, precision="f32", tune=tune)
    err = np.abs(L.rmse_trajectory - gold)
    print("f32 max |dRMSE| = %.3e" % err.max())
    assert err.max() < 1e-3


@pytest.mark.parametrize("K", [130, 200])
def test_f32_wide_factor_counts_within_north_star(ml100k, K):
    """f32 at K above 128: k_grow's KL = 256 register form (sigma and mu read from
    memory) for the 17..512-rating rows, 9..13 k-blocks in the f32 Gram-block and
    streaming kinds.  RMSE within 1e-3 of the f64 oracle over 3 sweeps, same RNG stream."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=K, iters=3, seed=3)
    L = _run(tr, te, 3, num_factor=K, seed=3, precision="f32")
    err = np.abs(L.rmse_trajectory - o["rmse"])
    print("f32 K=%d max |dRMSE| = %.3e" % (K, err.max()))
    assert err.max() < 1e-3
    U, V = L.factors()
    assert np.abs(U - o["U"]).max() < 5e-2 and np.abs(V - o["V"]).max() < 5e-2


@pytest.mark.parametrize("thr", [1, 40, 200])
@pytest.mark.parametrize("K", [20, 100, 200])
def test_streaming_kernel_matches_oracle(ml100k, thr, K):
    """Rows above `thr` ratings through the streaming Gram-block kernel."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=K, iters=3, seed=5)
    L = _run(tr, te, 3, num_factor=K, seed=5, stream_threshold=thr)
    U, V = L.factors()
    assert np.abs(U - o["U"]).max() < 1e-7
    assert np.abs(V - o["V"]).max() < 1e-7
    np.testing.assert_allclose(L.rmse_trajectory, o["rmse"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("chunk", [16, 64, 150])
@pytest.mark.parametrize("K", [20, 100])
def test_split_rows_match_oracle(ml100k, chunk, K):
    """Long rows split over several workgroups (k_gres tasks claimed from the task
    queue) that exchange their per-block (G, c) partials through global memory."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=K, iters=3, seed=9)
    L = _run(tr, te, 3, num_factor=K, seed=9, stream_threshold=40, split_chunk=chunk)
    U, V = L.factors()
    assert np.abs(U - o["U"]).max() < 1e-7
    assert np.abs(V - o["V"]).max() < 1e-7
    np.testing.assert_allclose(L.rmse_trajectory, o["rmse"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("tune", [0, 4, 8, 12, 128, 131072, 1 << 23, 1 << 24, 1 << 25, 1 << 27, 1 << 29, 1 << 30,
                                  (1 << 30) | (1 << 27), (1 << 29) | 128, (1 << 30) | 131072, (1 << 25) | 128, 256, 512,
                                  768, 1024, 1792, 4096, 8192, 16384])
def test_kernel_variants_match_oracle(ml100k, tune):
    """Kernel variants (sbmf_config.tune, include/sbmf.h): bit 2 power-of-two
    waves per Gram-block row, bit 3 two 8-vector waves for 33..64-rating f64
    rows; k_gres workgroup shapes (bit 7: 4-wave everywhere, 17: 16-wave
    everywhere, 23: 8-wave user rows, 27: 8-wave item rows); bit 24: k_gres as an
    cooperative launch; bit 25: the Gram-block kinds on one side stream; bit 29:
    no launch overlap (Gram-block launches after the streaming one); bit 30: the item half's two
    streaming sets one after the other instead of side by side; bits 8 / 9 / 10:
    the 65..128 / 129..256 / 9..64-rating f64 bins as Gram-block rows instead of
    one- / two- / one-wave k_grow workgroups; bit 12: k_grow's KL = 256 form (sigma
    and mu read from memory) at a K whose default is the KL = 128 one; bit 13: one 4-wave
    user streaming set (default: rows above 512 ratings on a second, 8-wave set); bit 14:
    that set on 16-wave workgroups.  Under the
    default overlap the two item streaming sets run concurrently on two streams
    beside the Gram-block launches, their split rows handing partials over while
    the other launches hold CUs: split_chunk 16 splits the longest rows into
    more than 30 chunks (co-residency of both sets under load), 64 into fewer."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=50, iters=3, seed=4)
    for kw in ({}, {"stream_threshold": 40, "split_chunk": 64}, {"stream_threshold": 40, "split_chunk": 16}):
        L = _run(tr, te, 3, num_factor=50, seed=4, tune=tune, **kw)
        U, V = L.factors()
        assert np.abs(U - o["U"]).max() < 1e-7
        assert np.abs(V - o["V"]).max() < 1e-7


def test_evaluation_order_changes_nothing(ml100k):
    """One rank evaluates the test RMSE on the second stream beside the next
    sweep's prologue kernels; tune bit 28 puts it back after them on the compute
    stream.  Both read U and V only and write different slots: the chain, the
    printed RMSEs and the factors are the same bit for bit."""
    tr, te = ml100k
    kw = dict(num_factor=30, seed=8, rng="philox", eval_train=True)  # the overlapped schedule (device RNG)
    a = _run(tr, te, 4, **kw)
    b = _run(tr, te, 4, tune=1 << 28, **kw)
    assert np.array_equal(a.rmse_trajectory, b.rmse_trajectory)
    # the train RMSE's sum runs beside the prologue's (separate scratch areas)
    assert np.array_equal([h["rmse_train"] for h in a.history], [h["rmse_train"] for h in b.history])
    for x, y in zip(a.factors(), b.factors()):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("quirks", ["final", "bias2"])
def test_pipelined_sweeps_change_nothing(ml100k, quirks):
    """sbmf_config.pipeline: sweep s+1's start (hyperparameter upload, user half) is queued
    before sweep s is reported.  The chain, every per-sweep report and the factors are the
    same bit for bit; a stop asked for at sweep s takes effect after sweep s+1."""
    tr, te = ml100k
    kw = dict(num_factor=30, seed=8, rng="philox", eval_train=True, quirks=quirks)
    a = _run(tr, te, 6, **kw)
    b = _run(tr, te, 6, pipeline=1, **kw)
    for f in ("sweep", "rmse_avg", "rmse_this", "rmse_train", "tau", "collected"):
        assert np.array_equal([h[f] for h in a.history], [h[f] for h in b.history]), f
    for x, y in zip(a.factors(), b.factors()):
        assert np.array_equal(x, y)
    # two runs in a row on one learner (the second starts from the staged sweep 6)
    b.learn(sweeps=3)
    a.learn(sweeps=3)
    assert np.array_equal(a.rmse_trajectory, b.rmse_trajectory)
    # a stop at sweep 2: sweep 3 is already queued, so the run ends after it
    L = FMLearnSBPMF(pipeline=1, **kw)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=6, callback=lambda h: h["sweep"] == 2)
    assert [h["sweep"] for h in L.history] == [0, 1, 2, 3]
    assert np.array_equal(L.rmse_trajectory, a.rmse_trajectory[:4])


@pytest.mark.parametrize("kw", [{}, {"stream_threshold": 40, "split_chunk": 64}, {"stream_threshold": 16}])
def test_multigpu_residual_mode_matches_oracle(ml100k, kw):
    """The residual form every rank uses with several GPUs (e0 = r - own.partner
    recomputed per row instead of carried), forced on one GPU (tune bit 1)."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=30, iters=3, seed=6)
    L = _run(tr, te, 3, num_factor=30, seed=6, tune=2, **kw)
    U, V = L.factors()
    assert np.abs(U - o["U"]).max() < 1e-7
    assert np.abs(V - o["V"]).max() < 1e-7
    np.testing.assert_allclose(L.rmse_trajectory, o["rmse"], rtol=0, atol=1e-9)


def test_split_rows_deterministic(ml100k):
    tr, te = ml100k
    a = _run(tr, te, 3, num_factor=32, seed=2, rng="philox", stream_threshold=40, split_chunk=50)
    b = _run(tr, te, 3, num_factor=32, seed=2, rng="philox", stream_threshold=40, split_chunk=50)
    for x, y in zip(a.factors(), b.factors()):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("K", [8, 50, 100, 130, 200, 256])
def test_factor_counts_match_oracle(ml100k, K):
    """K spanning 1..4 register slots of 64, partial 16-wide k-blocks and padded tails."""
    tr, te = ml100k
    o = oracle.run(tr, te, K=K, iters=3, seed=3)
    L = _run(tr, te, 3, num_factor=K, seed=3)
    U, V = L.factors()
    assert np.abs(U - o["U"]).max() < 1e-7
    assert np.abs(V - o["V"]).max() < 1e-7


def test_philox_deterministic_and_init_matches_host(ml100k):
    from sbmf import philox_normals
    tr, te = ml100k
    a = FMLearnSBPMF(num_factor=20, seed=11, rng="philox")
    a.set_data(Data(*tr), Data(*te))
    U0, V0 = a.factors()
    for row in (0, 5, 942):  # init: U[r][k] = 1.0 * z(seed, sweep=0xffffffff, tag 3, r, k)
        np.testing.assert_allclose(U0[row], philox_normals(11, 0xffffffff, 3, row, 20), rtol=1e-13, atol=1e-13)
    a.learn(sweeps=4)
    b = _run(tr, te, 4, num_factor=20, seed=11, rng="philox")
    Ua, Va = a.factors()
    Ub, Vb = b.factors()
    assert np.array_equal(Ua, Ub) and np.array_equal(Va, Vb)
    assert np.array_equal(a.rmse_trajectory, b.rmse_trajectory)
