import numpy as np

from sbmf import synth


def test_synthetic_shape_deterministic():
    a = synth.generate("ml-100k", seed=1)
    b = synth.generate("ml-100k", seed=1)
    for x, y in zip(a[0] + a[1], b[0] + b[1]):
        assert np.array_equal(x, y)
    train, test, dims = a
    assert dims == (943, 1682)
    assert len(train[0]) + len(test[0]) == 100_000
    assert set(np.unique(train[2])) <= {1.0, 2.0, 3.0, 4.0, 5.0}
    key = train[0].astype(np.int64) * dims[1] + train[1]
    assert len(np.unique(key)) == len(key)  # no duplicate pairs
