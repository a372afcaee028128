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


def test_relabel_by_degree_is_a_degree_sorted_renumbering():
    """synth.relabel_by_degree (the 8-rank partition edge cases of test_gpu_multirank):
    the same ratings under a bijective renumbering of users and items, heaviest first,
    ties in old-id order, test ratings renumbered with the same maps."""
    train, test, dims = synth.generate("ml-100k", seed=3)
    tr2, te2, dims2 = synth.relabel_by_degree(train, test, dims)
    assert dims2 == dims
    np.testing.assert_array_equal(tr2[2], train[2])
    np.testing.assert_array_equal(te2[2], test[2])
    for a, n in ((0, dims[0]), (1, dims[1])):
        old = np.bincount(train[a], minlength=n)
        new = np.bincount(tr2[a], minlength=n)
        assert np.all(np.diff(new) <= 0)                     # heaviest first
        np.testing.assert_array_equal(np.sort(old)[::-1], new)  # a permutation of the degrees
        # the map old id -> new id is one bijection, applied to train and test alike
        m = np.full(n, -1, np.int64)
        m[train[a]] = tr2[a]
        assert np.all(m[train[a]] == tr2[a])
        seen = m[m >= 0]
        assert len(np.unique(seen)) == len(seen)
        # ties keep the old id order (stable)
        order = np.argsort(-old, kind="stable")
        np.testing.assert_array_equal(m[order[old[order] > 0]], np.arange(n)[old[order] > 0])
        both = np.isin(test[a], train[a])
        np.testing.assert_array_equal(te2[a][both], m[test[a][both]])
