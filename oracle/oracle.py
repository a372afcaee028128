"""oracle.py -- TEST INFRASTRUCTURE ONLY: ctypes wrapper of liboracle.so.

The CPU restatement of the reference sampler (sbpmf_oracle.c), used only by
tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline.
"""
import ctypes as C
import time
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
QUIRKS = {"final": 0, "sbpmf2": 1, "none": 2, "bias2": 3, "bias22": 4}


class OracleConfig(C.Structure):
    _fields_ = [("K", C.c_uint32), ("iters", C.c_uint32), ("burnin", C.c_uint32), ("seed", C.c_uint),
                ("quirks", C.c_int), ("init_stdev", C.c_double), ("clamp_lo", C.c_double),
                ("clamp_hi", C.c_double), ("sweep_seconds_limit", C.c_double), ("rng", C.c_int),
                ("threads", C.c_int)]


class OracleResult(C.Structure):
    _fields_ = [("rmse", C.POINTER(C.c_double)), ("rmse_this", C.POINTER(C.c_double)),
                ("tau", C.POINTER(C.c_double)), ("rmse_cap", C.c_uint32),
                ("U", C.POINTER(C.c_double)), ("V", C.POINTER(C.c_double)), ("hyper", C.POINTER(C.c_double)),
                ("pred_sum", C.POINTER(C.c_double)), ("num_users", C.c_uint32), ("num_items", C.c_uint32),
                ("sweeps_done", C.c_uint32), ("seconds", C.c_double), ("bu", C.POINTER(C.c_double)),
                ("bv", C.POINTER(C.c_double)), ("b0", C.c_double)]


class VBOConfig(C.Structure):
    _fields_ = [("K", C.c_uint32), ("epochs", C.c_uint32), ("seed", C.c_uint), ("num_batch", C.c_uint32),
                ("seconds_limit", C.c_double)]


class VBOResult(C.Structure):
    _fields_ = [("rmse", C.POINTER(C.c_double)), ("rmse_cap", C.c_uint32), ("pred", C.POINTER(C.c_double)),
                ("mu_w", C.POINTER(C.c_double)), ("mu_v", C.POINTER(C.c_double)), ("alpha", C.c_double),
                ("mu0", C.c_double), ("seconds", C.c_double), ("num_attribute", C.c_uint32),
                ("epochs_done", C.c_uint32)]


class FMMConfig(C.Structure):
    _fields_ = [("K", C.c_uint32), ("iters", C.c_uint32), ("seed", C.c_uint), ("k0", C.c_int), ("k1", C.c_int),
                ("do_sample", C.c_int), ("do_multilevel", C.c_int), ("init_stdev", C.c_double),
                ("reg0", C.c_double), ("regw", C.c_double), ("regv", C.c_double)]


class FMMResult(C.Structure):
    _fields_ = [("rmse_test", C.POINTER(C.c_double)), ("rmse_this", C.POINTER(C.c_double)),
                ("rmse_train", C.POINTER(C.c_double)), ("alpha", C.POINTER(C.c_double)), ("cap", C.c_uint32),
                ("pred", C.POINTER(C.c_double)), ("w", C.POINTER(C.c_double)), ("v", C.POINTER(C.c_double)),
                ("w0", C.c_double), ("min_target", C.c_double), ("max_target", C.c_double),
                ("num_attribute", C.c_uint32), ("iters_done", C.c_uint32)]


def build():
    import subprocess
    subprocess.run(["make", "-C", HERE, "all"], check=True, capture_output=True)


def _lib():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    lib.oracle_run_arrays.restype = C.c_int
    lib.oracle_config_default.argtypes = [C.POINTER(OracleConfig)]
    lib.oracle_ran_gaussian.restype = C.c_double
    lib.oracle_ran_gamma.restype = C.c_double
    lib.oracle_ran_gamma.argtypes = [C.c_double]
    lib.oracle_ran_uniform.restype = C.c_double
    lib.oracle_srand.argtypes = [C.c_uint]
    lib.oracle_vbo_run.restype = C.c_int
    lib.oracle_fmm_run.restype = C.c_int
    return lib


_L = None


def lib():
    global _L
    if _L is None:
        _L = _lib()
    return _L


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def run(train, test, K=20, iters=100, seed=1, quirks="final", burnin=0, num_users=0, num_items=0,
        seconds_limit=0.0, want_factors=True, rng="ref", threads=1):
    """train/test: (user, item, rating) arrays.  Returns dict with per-sweep
    'rmse' (running mean, the reference's "rmse is"), 'rmse_this', 'tau',
    final 'U' [I][K], 'V' [J][K], 'hyper', 'pred_sum', 'seconds', and for the
    biased samplers (quirks bias2 / bias22) 'bu', 'bv', 'b0'."""
    L = lib()
    cfg = OracleConfig()
    L.oracle_config_default(C.byref(cfg))
    cfg.K, cfg.iters, cfg.burnin, cfg.seed, cfg.quirks = K, iters, burnin, seed, QUIRKS[quirks]
    cfg.sweep_seconds_limit = seconds_limit
    if rng not in ("ref", "philox") or (rng == "philox" and quirks in ("bias2", "bias22")):
        raise ValueError("oracle rng %r with quirks %r" % (rng, quirks))
    cfg.rng = 1 if rng == "philox" else 0
    if threads > 1 and rng != "philox":
        raise ValueError("the parallel oracle needs the Philox stream (the glibc stream is sequential)")
    cfg.threads = threads
    tu, ti, tr = (np.ascontiguousarray(train[0], np.uint32), np.ascontiguousarray(train[1], np.uint32),
                  np.ascontiguousarray(train[2], np.float64))
    su, si, sr = (np.ascontiguousarray(test[0], np.uint32), np.ascontiguousarray(test[1], np.uint32),
                  np.ascontiguousarray(test[2], np.float64))
    I = num_users or int(max(tu.max(initial=0), su.max(initial=0))) + 1
    J = num_items or int(max(ti.max(initial=0), si.max(initial=0))) + 1
    n_sw = iters + burnin
    res = OracleResult()
    rm, rt, ta = np.full(n_sw, np.nan), np.full(n_sw, np.nan), np.full(n_sw, np.nan)
    res.rmse, res.rmse_this, res.tau, res.rmse_cap = _p(rm, C.c_double), _p(rt, C.c_double), _p(ta, C.c_double), n_sw
    U = V = None
    if want_factors:
        U, V = np.zeros((I, K)), np.zeros((J, K))
        res.U, res.V = _p(U, C.c_double), _p(V, C.c_double)
    hyper = np.zeros(4 * K)
    res.hyper = _p(hyper, C.c_double)
    ps = np.zeros(max(len(sr), 1))
    res.pred_sum = _p(ps, C.c_double)
    bu, bv = np.zeros(I), np.zeros(J)
    res.bu, res.bv = _p(bu, C.c_double), _p(bv, C.c_double)
    rc = L.oracle_run_arrays(C.byref(cfg), C.c_uint64(len(tr)), _p(tu, C.c_uint32), _p(ti, C.c_uint32),
                             _p(tr, C.c_double), C.c_uint64(len(sr)), _p(su, C.c_uint32), _p(si, C.c_uint32),
                             _p(sr, C.c_double), C.c_uint32(num_users), C.c_uint32(num_items), C.byref(res))
    assert rc == 0
    n = res.sweeps_done
    return {"rmse": rm[:n], "rmse_this": rt[:n], "tau": ta[:n], "U": U, "V": V, "hyper": hyper,
            "pred_sum": ps[:len(sr)], "seconds": res.seconds, "sweeps": n, "num_users": res.num_users,
            "num_items": res.num_items, "bu": bu, "bv": bv, "b0": res.b0}


def run_vbo(train, test, K=8, epochs=10, seed=1, num_users=0, num_items=0, seconds_limit=0.0, want_params=True):
    """The online VB oracle (vbo_oracle.c, the reference's -method vb_online on
    rating data).  Returns per-epoch test 'rmse', final clamped 'pred', the
    attribute means 'mu_w' [p] and 'mu_v' [p][K] (users first, then items),
    'alpha', 'mu0', 'seconds'."""
    L = lib()
    cfg = VBOConfig(K, epochs, seed, 0, seconds_limit)
    tu, ti, tr = (np.ascontiguousarray(train[0], np.uint32), np.ascontiguousarray(train[1], np.uint32),
                  np.ascontiguousarray(train[2], np.float64))
    su, si, sr = (np.ascontiguousarray(test[0], np.uint32), np.ascontiguousarray(test[1], np.uint32),
                  np.ascontiguousarray(test[2], np.float64))
    I = num_users or int(max(tu.max(initial=0), su.max(initial=0))) + 1
    J = num_items or int(max(ti.max(initial=0), si.max(initial=0))) + 1
    p = I + J
    res = VBOResult()
    rm = np.full(epochs, np.nan)
    res.rmse, res.rmse_cap = _p(rm, C.c_double), epochs
    pred = np.zeros(max(len(sr), 1))
    res.pred = _p(pred, C.c_double)
    mu_w = mu_v = None
    if want_params:
        mu_w, mu_v = np.zeros(p), np.zeros((p, K))
        res.mu_w, res.mu_v = _p(mu_w, C.c_double), _p(mu_v, C.c_double)
    rc = L.oracle_vbo_run(C.byref(cfg), C.c_uint64(len(tr)), _p(tu, C.c_uint32), _p(ti, C.c_uint32),
                          _p(tr, C.c_double), C.c_uint64(len(sr)), _p(su, C.c_uint32), _p(si, C.c_uint32),
                          _p(sr, C.c_double), C.c_uint32(I), C.c_uint32(J), C.byref(res))
    if rc != 0:
        raise ValueError("oracle_vbo_run failed (an empty batch: fewer ratings than the 30 batches need)")
    n = res.epochs_done
    return {"rmse": rm[:n], "pred": pred[:len(sr)], "mu_w": mu_w, "mu_v": mu_v, "alpha": res.alpha, "mu0": res.mu0,
            "seconds": res.seconds, "epochs": n, "num_attribute": res.num_attribute}


def libfm_attrs(train, test, num_users=0):
    """Rating triples -> libFM users-first attribute pairs (a0 = u, a1 = I + i,
    the layout of "r u:1 (I+i):1" lines) and the data sets' num_feature
    (largest attribute id + 1, Data.h:221)."""
    tu, ti = np.asarray(train[0], np.int64), np.asarray(train[1], np.int64)
    su, si = np.asarray(test[0], np.int64), np.asarray(test[1], np.int64)
    I = num_users or int(max(tu.max(initial=0), su.max(initial=0))) + 1
    ta = (tu.astype(np.uint32), (I + ti).astype(np.uint32))
    sa = (su.astype(np.uint32), (I + si).astype(np.uint32))
    p_train = int(ta[1].max(initial=0)) + 1
    p_test = int(sa[1].max(initial=0)) + 1 if len(su) else 0
    return ta, sa, p_train, p_test, I


def run_fmm(train, test, K=8, iters=10, seed=1, method="mcmc", k0=1, k1=1, init_stdev=0.1, regular=(0.0, 0.0, 0.0),
            num_users=0, want_params=True):
    """The libFM MCMC / ALS oracle (fmm_oracle.c: bin/libFM -method mcmc|als on
    users-first rating data).  Returns per-iteration 'rmse_test' (the "Test="
    value), 'rmse_this', 'rmse_train', 'alpha', the -out predictions 'pred',
    the final 'w' [p], 'v' [K][p], 'w0'."""
    L = lib()
    als = method == "als"
    cfg = FMMConfig(K, iters, seed, k0, k1, 0 if als else 1, 0 if als else 1, init_stdev, *regular)
    ta, sa, p_train, p_test, I = libfm_attrs(train, test, num_users)
    ty = np.ascontiguousarray(train[2], np.float64)
    sy = np.ascontiguousarray(test[2], np.float64)
    p = max(p_train, p_test) + 1
    res = FMMResult()
    rt, rh, rr, al = (np.full(iters, np.nan) for _ in range(4))
    res.rmse_test, res.rmse_this, res.rmse_train, res.alpha = (_p(a, C.c_double) for a in (rt, rh, rr, al))
    res.cap = iters
    pred = np.zeros(max(len(sy), 1))
    res.pred = _p(pred, C.c_double)
    w = v = None
    if want_params:
        w, v = np.zeros(p), np.zeros((K, p))
        res.w, res.v = _p(w, C.c_double), _p(v, C.c_double)
    a0, a1 = (np.ascontiguousarray(x, np.uint32) for x in ta)
    b0, b1 = (np.ascontiguousarray(x, np.uint32) for x in sa)
    t0 = time.perf_counter()
    rc = L.oracle_fmm_run(C.byref(cfg), C.c_uint64(len(ty)), _p(a0, C.c_uint32), _p(a1, C.c_uint32),
                          _p(ty, C.c_double), C.c_uint64(len(sy)), _p(b0, C.c_uint32), _p(b1, C.c_uint32),
                          _p(sy, C.c_double), C.c_uint32(p_train), C.c_uint32(p_test), C.byref(res))
    seconds = time.perf_counter() - t0  # set-up + the iterations
    if rc != 0:
        raise ValueError("oracle_fmm_run failed (%d)" % rc)
    n = res.iters_done
    return {"rmse_test": rt[:n], "rmse_this": rh[:n], "rmse_train": rr[:n], "alpha": al[:n],
            "pred": pred[:len(sy)], "w": w, "v": v, "w0": res.w0, "num_attribute": res.num_attribute,
            "num_users": I, "seconds": seconds}


def stream(seed, kind, n, shape=1.0):
    """The reference RNG via glibc itself: kind 0 rand(), 1 ran_gaussian(), 2 ran_gamma(shape)."""
    L = lib()
    L.oracle_srand(seed)
    if kind == 0:
        L.oracle_rand.restype = C.c_int
        return np.array([L.oracle_rand() for _ in range(n)], dtype=np.float64)
    if kind == 1:
        return np.array([L.oracle_ran_gaussian() for _ in range(n)])
    return np.array([L.oracle_ran_gamma(shape) for _ in range(n)])
