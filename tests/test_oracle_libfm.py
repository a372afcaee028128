"""The libFM MCMC / ALS oracle (oracle/fmm_oracle.c) against libFM itself:
tests/golden/ref_libfm_* hold the stdout "#Iter=" lines and -out predictions
of src/libfm/libfm.cpp compiled unmodified (time() pinned to the seed,
oracle/ref_pin_time.c; oracle/make_golden.py libfm).  libFM prints 6
significant digits, so the lines must be equal as text and the predictions
within the rounding of their last digit."""
import gzip
import os

import numpy as np
import pytest

import oracle
from conftest import GOLD, read_libfm_text

# (method, data, dim, seed, iterations, -regular) -- as oracle/make_golden.py LIBFM_RUNS
RUNS = [("mcmc", "ml100k", "1,1,8", 1, 10, None), ("als", "ml100k", "1,1,8", 1, 10, "0,0,10"),
        ("mcmc", "ml100k", "0,0,20", 7, 20, None), ("mcmc", "ragged", "1,1,8", 3, 20, None),
        ("als", "ragged", "1,1,4", 2, 10, "1,2,5")]


def golden_name(method, dname, dim, seed, iters):
    return "ref_libfm_%s_%s_d%s_s%d_i%d" % (method, dname, dim.replace(",", ""), seed, iters)


def iter_lines(res):
    return ["#Iter=%3d\tTrain=%s\tTest=%s" % (i, "%g" % a, "%g" % b)
            for i, (a, b) in enumerate(zip(res["rmse_train"], res["rmse_test"]))]


@pytest.mark.parametrize("run", RUNS, ids=[golden_name(*r[:5]) for r in RUNS])
def test_oracle_matches_compiled_libfm(run, ml100k, ragged):
    method, dname, dim, seed, iters, reg = run
    tr, te = ml100k if dname == "ml100k" else ragged
    k0, k1, K = (int(x) for x in dim.split(","))
    regular = tuple(float(x) for x in reg.split(",")) if reg else (0.0, 0.0, 0.0)
    o = oracle.run_fmm(tr, te, K=K, iters=iters, seed=seed, method=method, k0=k0, k1=k1, regular=regular)
    name = golden_name(method, dname, dim, seed, iters)
    with open(os.path.join(GOLD, name + ".txt")) as f:
        ref_lines = f.read().splitlines()
    assert iter_lines(o) == ref_lines
    with gzip.open(os.path.join(GOLD, name + "_pred.txt.gz"), "rt") as f:
        ref_pred = np.array([float(x) for x in f.read().split()])
    assert ref_pred.shape == o["pred"].shape
    # libFM writes 6 significant digits: |err| <= half a unit of the last digit
    ulp6 = 10.0 ** (np.floor(np.log10(np.abs(ref_pred))) - 5)
    assert np.all(np.abs(o["pred"] - ref_pred) <= 0.5 * ulp6 * (1 + 1e-9))


def test_oracle_als_is_deterministic_and_seed_only_moves_the_init(ml100k):
    tr, te = ml100k
    a = oracle.run_fmm(tr, te, K=4, iters=3, seed=5, method="als", regular=(0.0, 0.0, 10.0))
    b = oracle.run_fmm(tr, te, K=4, iters=3, seed=5, method="als", regular=(0.0, 0.0, 10.0))
    assert np.array_equal(a["rmse_test"], b["rmse_test"]) and np.array_equal(a["v"], b["v"])


@pytest.mark.parametrize("method,reg", [("mcmc", None), ("als", "0,0,10")])
def test_oracle_matches_libfm_on_the_reference_files(method, reg, m1m100k):
    """bin/libFM -task r -dim '1,1,8' -iter 10 -method mcmc|als on the reference's own
    data/m1m/m100k/{train,test}_libfm, argv unchanged (tests/golden/ref_libfm_*_m1m100k_*).
    libFM's attributes are the file's feature ids: num_user = max first feature + 1
    (libfm.cpp:375) = 943, items rebased onto it."""
    (tu, ti, tr_), (su, si, sr) = m1m100k
    I = int(max(tu.max(), su.max())) + 1
    assert I == 943 and min(ti.min(), si.min()) >= I
    regular = tuple(float(x) for x in reg.split(",")) if reg else (0.0, 0.0, 0.0)
    o = oracle.run_fmm((tu, ti - I, tr_), (su, si - I, sr), K=8, iters=10, seed=1, method=method,
                       regular=regular)
    assert o["v"].shape[1] == int(max(ti.max(), si.max())) + 1 + 1  # libFM's p (+1: libfm.cpp:328)
    name = golden_name(method, "m1m100k", "1,1,8", 1, 10)
    with open(os.path.join(GOLD, name + ".txt")) as f:
        assert iter_lines(o) == f.read().splitlines()
    with gzip.open(os.path.join(GOLD, name + "_pred.txt.gz"), "rt") as f:
        ref_pred = np.array([float(x) for x in f.read().split()])
    ulp6 = 10.0 ** (np.floor(np.log10(np.abs(ref_pred))) - 5)
    assert np.all(np.abs(o["pred"] - ref_pred) <= 0.5 * ulp6 * (1 + 1e-9))
