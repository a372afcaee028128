"""Reference RNG stream: the product's host generator (rng.h, reached through
sbmf_ref_stream) and the oracle against the reference's own random.h output
(tests/golden/ref_rng_s*.txt from oracle/_ref/ref_rng_dump).  Bit-exact."""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLD
from sbmf import philox_normals, ref_stream


def _golden(seed):
    rand, gauss, gamma = [], [], {}
    with open(os.path.join(GOLD, "ref_rng_s%d.txt" % seed)) as f:
        for line in f:
            p = line.split()
            if p[0] == "rand":
                rand.append(float(p[1]))
            elif p[0] == "gauss":
                gauss.append(float(p[1]))
            else:
                gamma.setdefault(float(p[1]), []).append(float(p[2]))
    return np.array(rand), np.array(gauss), {k: np.array(v) for k, v in gamma.items()}


@pytest.mark.parametrize("seed", [1, 7])
def test_host_stream_bitwise_equals_reference_random_h(seed):
    rand, gauss, gamma = _golden(seed)
    assert np.array_equal(ref_stream(seed, 0, len(rand)), rand)
    assert np.array_equal(ref_stream(seed, 1, len(gauss)), gauss)
    for shape, vals in gamma.items():
        assert np.array_equal(ref_stream(seed, 2, len(vals), shape), vals), shape


@pytest.mark.parametrize("seed", [1, 7])
def test_oracle_stream_bitwise_equals_reference_random_h(seed):
    rand, gauss, gamma = _golden(seed)
    assert np.array_equal(oracle.stream(seed, 0, 500), rand[:500])
    assert np.array_equal(oracle.stream(seed, 1, 500), gauss[:500])


def test_glibc_seed_zero_is_seed_one():
    assert np.array_equal(ref_stream(0, 0, 100), ref_stream(1, 0, 100))


def test_philox_normals_deterministic_and_standard():
    a = philox_normals(2015, 3, 1, 77, 256)
    assert np.array_equal(a, philox_normals(2015, 3, 1, 77, 256))
    assert not np.array_equal(a, philox_normals(2015, 4, 1, 77, 256))  # sweep in the counter
    assert not np.array_equal(a[:128], a[128:])
    z = np.concatenate([philox_normals(9, s, 0, r, 200) for s in range(4) for r in range(100)])
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02


def test_oracle_philox_mode_restates_the_device_stream(ml100k):
    """oracle rng='philox' (test infrastructure) draws the GPU build's Philox
    normals: its initial factors equal sbmf_philox_normals (host C ABI) for
    (seed, sweep 0xffffffff, TAG_INIT_U / TAG_INIT_V, row)."""
    import oracle
    from sbmf import philox_normals
    tr, te = ml100k
    o = oracle.run(tr, te, K=20, iters=0, seed=2015, rng="philox")
    for row in (0, 17, 942):
        assert np.array_equal(o["U"][row], philox_normals(2015, 0xffffffff, 3, row, 20))
    for row in (0, 1681):
        assert np.array_equal(o["V"][row], philox_normals(2015, 0xffffffff, 4, row, 20))
    with pytest.raises(ValueError):
        oracle.run(tr, te, K=8, iters=1, rng="philox", quirks="bias2")
