"""The reference sampler's long-chain collapse, pinned on one set (VERDICT r2
"next round" item 4).

gibbs_sbpmf_final passes the posterior variance as the stdev of ran_gaussian
(:393,413,485,529).  On the ML-1M-shaped synthetic set (sbmf/synth.py) at
K=20, seed 1, its chain reaches its best running-mean test RMSE at sweep 36;
then tau falls to 0 within six sweeps, the hyperparameters turn NaN and every
prediction clamps.  tests/golden/ref_final_ml1msynth_k20_s1.txt is the
compiled reference's own 100-sweep trajectory on that set
(oracle/make_golden.py collapse); the oracle reproduces it bit for bit
(tests/test_oracle_golden.py) and gives tau per sweep.  The GPU chain, same
stream, must follow it: RMSE within 1e-6 up to the collapse, tau below 1e-3
at the same sweep +-2 and NaN by the same sweep +-2, the RMSE minimum at the
same sweep +-2.  bench.py's time-to-RMSE note (burn-in 50 on the ML-20M
shape) relies on this being the reference's behaviour, not a GPU defect."""
import numpy as np
import pytest

import oracle
from conftest import golden_rmse
from sbmf import Data, FMLearnSBPMF, synth

pytestmark = pytest.mark.gpu


def _first(mask):
    idx = np.flatnonzero(mask)
    return int(idx[0]) if len(idx) else -1


@pytest.mark.timeout(900)
@pytest.mark.parametrize("recompute_every", [1, 0])
def test_gpu_chain_collapses_with_the_reference(recompute_every):
    tr, te, dims = synth.generate("ml-1m")
    gold = golden_rmse("ref_final_ml1msynth_k20_s1.txt")
    o = oracle.run(tr, te, K=20, iters=50, seed=1, want_factors=False)
    assert np.array_equal(o["rmse"], gold[:50])  # the oracle is the reference here
    L = FMLearnSBPMF(num_factor=20, seed=1, rng="ref", recompute_every=recompute_every)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=100)
    rmse = L.rmse_trajectory
    tau = np.array([h["tau"] for h in L.history])
    L.close()
    c_ref = _first(~(o["tau"] >= 1e-3))     # first sweep with tau < 1e-3 (or NaN)
    n_ref = _first(np.isnan(o["tau"]))
    c_gpu, n_gpu = _first(~(tau >= 1e-3)), _first(np.isnan(tau))
    print("collapse: oracle tau<1e-3 at %d, NaN at %d; GPU %d, %d; RMSE min at %d (ref %d); "
          "max|dRMSE| to sweep 30 %.2e, final %.6f vs %.6f" % (
              c_ref, n_ref, c_gpu, n_gpu, int(np.argmin(rmse)), int(np.argmin(gold)),
              np.abs(rmse[:31] - gold[:31]).max(), rmse[-1], gold[-1]))
    assert c_ref == 37 and n_ref == 43 and int(np.argmin(gold)) == 36
    assert np.abs(rmse[:31] - gold[:31]).max() < 1e-6
    assert abs(c_gpu - c_ref) <= 2 and abs(n_gpu - n_ref) <= 2
    assert abs(int(np.argmin(rmse)) - int(np.argmin(gold))) <= 2
    assert np.all(np.isnan(tau[n_ref + 2:]))
    # after the collapse every prediction is the clamp bound: the running mean drifts the same way
    assert abs(rmse[-1] - gold[-1]) < 1e-3


@pytest.mark.timeout(600)
def test_gpu_biased_chain_stalls_with_the_reference():
    """The biased sampler (quirks bias2: top-level gibbs_sbpmf2.cpp:335-637) on the
    ML-1M-shaped set, K=20, seed 1, reference stream: the compiled reference's 100
    running-mean test RMSEs (tests/golden/ref_bias2_ml1msynth_k20_s1.txt, pinned to
    the oracle by test_oracle_golden.py) stay at the bias-only fit (> 1.05, never
    0.85); the GPU chain follows them to 1e-6 with the same shrunk factors."""
    tr, te, dims = synth.generate("ml-1m")
    gold = golden_rmse("ref_bias2_ml1msynth_k20_s1.txt")
    L = FMLearnSBPMF(num_factor=20, seed=1, rng="ref", quirks="bias2")
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=100)
    rmse = L.rmse_trajectory
    U, V = L.factors()
    L.close()
    print("bias2 stall: max|dRMSE| %.2e, final %.6f (ref %.6f), mean|U| %.2e" % (
        np.abs(rmse - gold).max(), rmse[-1], gold[-1], np.abs(U).mean()))
    assert np.abs(rmse - gold).max() < 1e-6
    assert rmse.min() > 1.05 and np.abs(U).mean() < 0.01 and np.abs(V).mean() < 0.01
