"""The all-core CPU baseline: the oracle's Philox mode
with the rows of each half-sweep spread over OpenMP threads follows the same
chain as the serial Philox run (only tau's residual sum changes order)."""
import numpy as np

import oracle


def test_parallel_oracle_matches_serial_philox(ml100k):
    tr, te = ml100k
    a = oracle.run(tr, te, K=20, iters=3, seed=4, rng="philox", threads=1)
    b = oracle.run(tr, te, K=20, iters=3, seed=4, rng="philox", threads=4)
    np.testing.assert_allclose(b["rmse"], a["rmse"], rtol=1e-9)
    np.testing.assert_allclose(b["U"], a["U"], rtol=0, atol=1e-8)
    np.testing.assert_allclose(b["V"], a["V"], rtol=0, atol=1e-8)


def test_parallel_oracle_needs_philox(ml100k):
    import pytest
    tr, te = ml100k
    with pytest.raises(ValueError):
        oracle.run(tr, te, K=4, iters=1, threads=2)
