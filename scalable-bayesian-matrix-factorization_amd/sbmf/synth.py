"""Deterministic synthetic rating sets shaped like the BASELINE configs.

MovieLens files are not available offline, so benchmarks run on planted
low-rank data with MovieLens-like degree distributions:
user degrees Pareto (alpha 1.2) with a floor of 20 ratings, item degrees
log-normal (heavy head, long tail), duplicates removed, ratings
clip(round(3.5 + u.v + N(0, 0.5)), 1, 5) from a rank-10 model (signal std 1;
noise floor with rounding ~0.58, below the metric's 0.85 RMSE target, as
SURVEY.md §7.3(6) asks), and a random 90:10 train/test split.  ML-20M: 138,493 users x 26,744 items, 20.0M ratings
(median item degree ~18-20, largest item ~67K ratings, largest user ~9K).
"""
import numpy as np

SHAPES = {
    # name: (users, items, total ratings, max user degree, max item degree)
    "ml-100k": (943, 1682, 100_000, 737, 583),
    "ml-1m": (6040, 3706, 1_000_209, 2314, 3428),
    "ml-10m": (69878, 10677, 10_000_054, 7359, 34864),
    "ml-20m": (138493, 26744, 20_000_263, 9254, 67310),
    "netflix": (480189, 17770, 100_480_507, 17653, 232944),
}


FAST_ABOVE = 50_000_000  # shapes with more ratings use the sort-based generator


def _degrees(rng, n, total, dmin, dmax, kind):
    if kind == "pareto":
        d = dmin * (1.0 - rng.random(n)) ** (-1.0 / 1.2)
    else:  # log-normal item popularity
        d = np.exp(rng.normal(np.log(18.0), 2.3, n))
    d = np.clip(d, dmin, dmax)
    # rescale the unclipped middle so the total matches
    for _ in range(50):
        s = d.sum()
        if abs(s - total) < 0.001 * total:
            break
        free = (d > dmin) & (d < dmax)
        f = (total - d[~free].sum()) / max(d[free].sum(), 1.0)
        d = np.where(free, np.clip(d * f, dmin, dmax), d)
    d = np.maximum(np.round(d).astype(np.int64), 1)
    d[np.argmax(d)] = dmax  # pin the head exactly
    return d


def generate(shape="ml-20m", seed=2015, rank=10, noise=0.5, test_frac=0.1):
    """Returns (train, test, (num_users, num_items)); train/test are
    (user uint32, item uint32, rating float64) in random file order.
    With $SBMF_SYNTH_CACHE set, the arrays are cached there as .npz."""
    import os
    cache = os.environ.get("SBMF_SYNTH_CACHE")
    if cache:
        path = os.path.join(cache, "synth_%s_s%d_r%d_n%g_t%g.npz" % (shape, seed, rank, noise, test_frac))
        if os.path.exists(path):
            z = np.load(path)
            return ((z["tu"], z["ti"], z["tr"]), (z["su"], z["si"], z["sr"]), (int(z["I"]), int(z["J"])))
        train, test, dims = _generate(shape, seed, rank, noise, test_frac)
        os.makedirs(cache, exist_ok=True)
        np.savez(path, tu=train[0], ti=train[1], tr=train[2], su=test[0], si=test[1], sr=test[2], I=dims[0], J=dims[1])
        return train, test, dims
    return _generate(shape, seed, rank, noise, test_frac)


def _generate(shape, seed, rank, noise, test_frac):
    I, J, total, umax, imax = SHAPES[shape]
    rng = np.random.default_rng(seed)
    du = _degrees(rng, I, total, min(20, umax), umax, "pareto")
    di = _degrees(rng, J, total, 1, imax, "lognormal")
    # Chung-Lu: draw (user, item) pairs with probabilities proportional to
    # the target degrees, oversample, drop duplicate pairs, keep `total`.
    pu = du / du.sum()
    pi = di / di.sum()
    if total <= FAST_ABOVE:
        keys = np.zeros(0, np.int64)
        m = int(total * 1.3)
        while True:
            us = rng.choice(I, m, p=pu).astype(np.int64)
            its = rng.choice(J, m, p=pi).astype(np.int64)
            keys = np.concatenate([keys, us * J + its])
            _, first = np.unique(keys, return_index=True)
            if len(first) >= total:
                break
            m = int((total - len(first)) * 1.5) + 1000
        key = keys[np.sort(first)][:total]  # first occurrences, draw order = random file order
    else:
        # large shapes: sorted unique pairs (one plain sort per round), then a
        # random permutation as the file order -- minutes faster at 100 M
        uk = np.zeros(0, np.int64)
        m = int(total * 1.4)
        while len(uk) < total:
            us = rng.choice(I, m, p=pu).astype(np.int64)
            its = rng.choice(J, m, p=pi).astype(np.int64)
            uk = np.union1d(uk, us * J + its) if len(uk) else np.unique(us * J + its)
            m = int((total - len(uk)) * 2.0) + 100000
        key = rng.permutation(uk)[:total]
    u = (key // J).astype(np.uint32)
    i = (key % J).astype(np.uint32)
    P = rng.normal(0.0, (1.0 / rank) ** 0.25, (I, rank))
    Q = rng.normal(0.0, (1.0 / rank) ** 0.25, (J, rank))
    r = np.empty(len(u))
    step = 1 << 22
    for s in range(0, len(u), step):
        e = min(len(u), s + step)
        r[s:e] = 3.5 + np.einsum("nk,nk->n", P[u[s:e]], Q[i[s:e]]) + rng.normal(0.0, noise, e - s)
    r = np.clip(np.round(r), 1.0, 5.0)
    nt = int(len(u) * test_frac)
    test = (u[:nt].copy(), i[:nt].copy(), r[:nt].copy())
    train = (u[nt:].copy(), i[nt:].copy(), r[nt:].copy())
    return train, test, (I, J)


def relabel_by_degree(train, test, dims):
    """The same ratings with user and item ids renumbered by train degree,
    heaviest first (ties by old id).  Contiguous nnz-balanced row blocks then
    hold a few very long rows at the front and thousands of short ones at the
    back: at 8 ranks the first item block is empty (its 256-aligned cut falls
    at row 0), the last user block holds only Gram-block rows -- the partition
    edge cases a shuffled id order never produces."""
    out_tr, out_te = list(train), list(test)
    for a, n in ((0, dims[0]), (1, dims[1])):
        deg = np.bincount(train[a], minlength=n)
        order = np.argsort(-deg, kind="stable")
        new = np.empty(n, np.uint32)
        new[order] = np.arange(n, dtype=np.uint32)
        out_tr[a] = new[train[a]]
        out_te[a] = new[test[a]]
    return tuple(out_tr), tuple(out_te), dims


def describe(train, dims):
    u, i, _ = train
    du = np.bincount(u, minlength=dims[0])
    di = np.bincount(i, minlength=dims[1])
    q = lambda d: {"mean": float(d.mean()), "median": float(np.median(d)), "max": int(d.max()),
                   "p99": float(np.percentile(d, 99))}
    return {"n_train": int(len(u)), "user_deg": q(du), "item_deg": q(di)}
