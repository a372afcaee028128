"""The oracle (CPU restatement, oracle/sbpmf_oracle.c) against the reference's
own outputs: per-sweep test RMSE trajectories produced by the compiled,
unmodified reference samplers (tests/golden/, oracle/make_golden.py).  Bit-exact:
every one of the 100 "%.17g" values must be identical."""
import numpy as np
import pytest

import oracle
from conftest import golden_rmse


@pytest.mark.parametrize("variant,data,seed,K", [("final", "ml100k", 1, 20), ("final", "ml100k", 7, 20),
                                                 ("sbpmf2", "ml100k", 1, 20), ("final", "ragged", 1, 20),
                                                 ("sbpmf2", "ragged", 5, 20), ("bias2", "ml100k", 1, 20),
                                                 ("bias2", "ragged", 3, 20), ("bias22", "ml100k", 1, 100)])
def test_oracle_bitwise_equals_reference(variant, data, seed, K, ml100k, ragged):
    """bias2 = the biased sampler at the top level of the reference
    (gibbs_sbpmf2.cpp, D=20), bias22 = src/libfm/gibbs_sbpmf22.cpp (D=100)."""
    tr, te = ml100k if data == "ml100k" else ragged
    gold = golden_rmse("ref_%s_%s_k%d_s%d.txt" % (variant, data, K, seed))
    o = oracle.run(tr, te, K=K, iters=100, seed=seed, quirks=variant, want_factors=False)
    assert np.array_equal(o["rmse"], gold), np.abs(o["rmse"] - gold).max()


def test_oracle_bitwise_equals_reference_on_its_own_m1m100k_files(m1m100k):
    """gibbs_sbpmf_final (K=20, seed 1) on the reference's converted data/m1m/m100k/{train,test}_sbpmf:
    raw item ids 943..2624 kept by create_file_scalable_bpmf.py, so items 0..942 are empty rows
    drawn from the prior every sweep."""
    tr, te = m1m100k
    gold = golden_rmse("ref_final_m1m100k_k20_s1.txt")
    o = oracle.run(tr, te, K=20, iters=100, seed=1, want_factors=False)
    assert np.array_equal(o["rmse"], gold), np.abs(o["rmse"] - gold).max()
    assert o["num_items"] == 2625


def test_oracle_dims_follow_reference_rule(ragged):
    """num_users/items = max id + 1 over train AND test (gibbs_sbpmf_final.cpp:146-148)."""
    tr, te = ragged
    o = oracle.run(tr, te, K=4, iters=1, seed=1, want_factors=False)
    assert o["num_users"] == max(tr[0].max(), te[0].max()) + 1
    assert o["num_items"] == max(tr[1].max(), te[1].max()) + 1


@pytest.mark.parametrize("data,K,seed,epochs", [("ml100k", 8, 1, 10), ("ml100k", 20, 7, 5), ("ragged", 8, 2, 20)])
def test_vbo_oracle_bitwise_equals_reference(data, K, seed, epochs, ml100k, ragged):
    """Online VB (-method vb_online): the oracle (vbo_oracle.c) against the
    reference learner itself (fm_learn_vb_online*.h compiled unmodified, driven
    by oracle/ref_vbo_harness.cpp): every per-epoch test RMSE identical."""
    tr, te = ml100k if data == "ml100k" else ragged
    gold = golden_rmse("ref_vbo_%s_k%d_s%d_e%d.txt" % (data, K, seed, epochs))
    o = oracle.run_vbo(tr, te, K=K, epochs=epochs, seed=seed, want_params=False)
    assert np.array_equal(o["rmse"], gold), np.abs(o["rmse"] - gold).max()


def test_oracle_follows_reference_through_collapse():
    """gibbs_sbpmf_final on the ML-1M-shaped synthetic set (K=20, seed 1): the
    reference's 100-sweep trajectory bottoms at sweep 36 and rises as tau falls
    to 0 and turns NaN; the oracle reproduces all 100 lines bit for bit."""
    from sbmf import synth
    tr, te, _ = synth.generate("ml-1m")
    gold = golden_rmse("ref_final_ml1msynth_k20_s1.txt")
    o = oracle.run(tr, te, K=20, iters=100, seed=1, want_factors=False)
    assert np.array_equal(o["rmse"], gold)
    assert int(np.argmin(gold)) == 36 and np.isnan(o["tau"][43:]).all()


def test_oracle_follows_biased_reference_stall():
    """The top-level biased sampler (gibbs_sbpmf2.cpp, the paper's SBMF-P model,
    D=20) on the same ML-1M-shaped set: the compiled reference never leaves the
    bias-only fit -- test RMSE 1.0632 -> 1.0587, about the spread of the test
    ratings (1.056) -- because the factor precisions drawn with shape alpha0 + I
    (no 1/2, :386) and the posterior variance passed as the stdev shrink every
    factor to ~1e-3.  The oracle reproduces the first 40 of its 100 lines bit for
    bit and shows the shrunk factors; bench.py's biased time-to-RMSE legs, which
    never reach 0.85, rest on this being the reference's behaviour."""
    from sbmf import synth
    tr, te, _ = synth.generate("ml-1m")
    gold = golden_rmse("ref_bias2_ml1msynth_k20_s1.txt")
    o = oracle.run(tr, te, K=20, iters=40, seed=1, quirks="bias2", want_factors=True)
    assert np.array_equal(o["rmse"], gold[:40])
    assert gold.min() > 1.05 and abs(gold[-1] - te[2].std()) < 0.01
    assert np.abs(o["U"]).mean() < 0.01 and np.abs(o["V"]).mean() < 0.01


def _seeds_golden(name):
    import os
    from conftest import GOLD
    with open(os.path.join(GOLD, name)) as f:
        return np.array([[float(x) for x in line.split()] for line in f if line.strip()])


def test_seed_sweep_golden_is_the_reference_chain(ml100k):
    """tests/golden/ref_final_ml100k_k20_seeds64.txt (the compiled gibbs_sbpmf_final over
    seeds 1..64, first 20 sweeps) is the reference-stream chain: the oracle reproduces
    sampled rows bit for bit."""
    ref = _seeds_golden("ref_final_ml100k_k20_seeds64.txt")
    assert ref.shape == (64, 20)
    for seed in (1, 33, 64):
        o = oracle.run(*ml100k, K=20, iters=20, seed=seed, want_factors=False)
        assert np.array_equal(o["rmse"], ref[seed - 1])


def test_oracle_philox_chain_matches_reference_chain_in_distribution(ml100k):
    """The throughput stream's restatement (the oracle's Philox mode, which the GPU
    follows to ~1e-9) against the 64 reference chains: seed means at sweeps 10 and 20
    within two standard errors (the criterion of tests/test_gpu_statistical.py)."""
    ref = _seeds_golden("ref_final_ml100k_k20_seeds64.txt")
    ph = np.array([oracle.run(*ml100k, K=20, iters=20, seed=s, rng="philox", want_factors=False)["rmse"]
                   for s in range(1, 65)])
    for k in (9, 19):
        d = ph[:, k].mean() - ref[:, k].mean()
        se = np.sqrt(ph[:, k].var(ddof=1) / 64 + ref[:, k].var(ddof=1) / 64)
        assert abs(d) <= 2 * se, (k, d, se)
