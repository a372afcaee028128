"""sbmf -- Python mirror of the reference's learner interface over the MI355X C ABI.

The reference's operator API for this path is libFM's ``fm_learn``
(src/libfm/src/fm_learn.h:38-308): ``init()``, ``learn(train, test)``,
``predict(data, out)``, ``evaluate(data)``, with the MCMC learner's knobs
``num_iter`` / ``num_eval_cases`` (fm_learn_mcmc.h:75-93) and the model's
``num_factor`` (fm_model.h:35-130).  ``FMLearnSBPMF`` keeps those names and
meanings; the work runs in ``libsbmf.so`` (HIP kernels for gfx950).  Errors
raise ``SBMFError`` (the reference throws ``std::string``).  There is no CPU
compute path: without a GPU, ``init()`` raises ``SBMFError`` (SBMF_E_DEVICE).

Runtime note: libsbmf binds ROCm's ``libamdhip64.so.7``.  PyTorch wheels ship
their own copy under the same soname; if torch is imported first, libsbmf
shares torch's runtime (fine).  If sbmf is imported first, create the learner
(``init()``) before the first ``torch.cuda`` call -- a second HSA runtime
initialised after the first one sees no device.
"""
import ctypes as C

import numpy as np

from . import _lib
from ._lib import (F32, F64, METHOD_ALS, METHOD_LIBFM_MCMC, METHOD_MCMC, METHOD_VB, QUIRKS_BIAS2, QUIRKS_BIAS22, QUIRKS_FINAL, QUIRKS_NONE, QUIRKS_SBPMF2, RNG_PHILOX, RNG_REFERENCE, SBMF_E_ARG,
                   SBMF_E_COMM, SBMF_E_DEVICE, SBMF_E_IO, SBMF_E_NOMEM, SBMF_E_STATE, SBMF_OK)

__all__ = ["FMLearnSBPMF", "FMLearnVBOnline", "Data", "SBMFError", "load_triples", "load_libfm", "load_libfm_binary", "save_libfm_binary", "libfm_binary_kind", "device_usage", "Communicator", "save_triples", "config_default",
           "RNG_REFERENCE", "RNG_PHILOX", "QUIRKS_FINAL", "QUIRKS_SBPMF2", "QUIRKS_NONE",
           "QUIRKS_BIAS2", "QUIRKS_BIAS22", "F64", "F32"]

lib = _lib.lib


class SBMFError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("sbmf error %d: %s" % (code, msg))
        self.code = code


def _u32(a):
    """ids as uint32, refusing values the cast would wrap (negative or >= 2^32)."""
    a = np.asarray(a)
    if a.dtype != np.uint32 and a.size:
        if a.dtype.kind == "f" and not np.all(np.isfinite(a) & (a == np.floor(a))):
            raise ValueError("ids must be integers")
        if a.min() < 0 or a.max() > 0xffffffff:
            raise ValueError("ids must be in [0, 2^32 - 1]")
    return np.ascontiguousarray(a, dtype=np.uint32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptr(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class Data:
    """Ratings triples (user, item, rating), 0-based ids; libFM's DataSubset role."""

    def __init__(self, user, item, rating):
        self.user, self.item, self.rating = _u32(user), _u32(item), _f64(rating)
        if not (len(self.user) == len(self.item) == len(self.rating)):
            raise ValueError("user/item/rating length mismatch")

    @property
    def num_cases(self):
        return len(self.rating)

    @property
    def target(self):
        return self.rating


def _from_ratings(r):
    n = int(r.n)
    if n == 0:
        return Data(np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0))
    u = np.ctypeslib.as_array(r.user, shape=(n,)).copy()
    i = np.ctypeslib.as_array(r.item, shape=(n,)).copy()
    v = np.ctypeslib.as_array(r.rating, shape=(n,)).copy()
    return Data(u, i, v)


def load_triples(path):
    """SBPMF triple file (gibbs_sbpmf_final.cpp:43 acceptance rule)."""
    r = _lib.Ratings()
    rc = lib.sbmf_load_triples(str(path).encode(), C.byref(r))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_loader_error().decode())
    try:
        return _from_ratings(r)
    finally:
        lib.sbmf_free_ratings(C.byref(r))


def load_libfm_binary(stem, item_offset=0, transpose=False):
    """libFM binary <stem>.x/.y (or .data/.target), Data.h:113-160; one user and
    one item feature per row.  transpose=True reads the feature-major
    <stem>.xt/.y (or .datat/.target) that tools/transpose.cpp writes and
    bin/libFM -method mcmc|als loads (libfm.cpp:140-149)."""
    r = _lib.Ratings()
    fn = lib.sbmf_load_libfm_binary_t if transpose else lib.sbmf_load_libfm_binary
    rc = fn(str(stem).encode(), item_offset, C.byref(r))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_loader_error().decode())
    try:
        return _from_ratings(r)
    finally:
        lib.sbmf_free_ratings(C.byref(r))


def libfm_binary_kind(stem, has_x, has_xt):
    """Data::load's file choice (Data.h:112-117): 1 = .data/.datat/.target,
    2 = .x/.xt/.y, 0 = none (libFM text)."""
    rc = lib.sbmf_libfm_binary_kind(str(stem).encode(), int(has_x), int(has_xt))
    if rc < 0:
        raise SBMFError(rc, "has_x or has_xt must be set")
    return rc


def save_libfm_binary(stem, data, item_offset=0, num_cols=0, transpose=False):
    """Write <stem>.x / <stem>.y as tools/convert.cpp does for rating data
    (transpose=True: <stem>.xt / <stem>.y, convert then tools/transpose.cpp)."""
    u, i = _u32(data.user), _u32(data.item)  # refuses negative / >= 2^32 ids before the cast
    # the .x format holds feature ids (user, item_offset + item) as uint32 with num_cols = max + 1
    if len(u) and (int(u.max()) > 0xfffffffe or int(i.max()) + int(item_offset) > 0xfffffffe):
        raise ValueError("feature ids must stay below 2^32 - 1 in the libFM binary format")
    v = np.ascontiguousarray(data.rating, dtype=np.float64)
    r = _lib.Ratings()
    r.n = len(u)
    r.user = u.ctypes.data_as(C.POINTER(C.c_uint32))
    r.item = i.ctypes.data_as(C.POINTER(C.c_uint32))
    r.rating = v.ctypes.data_as(C.POINTER(C.c_double))
    fn = lib.sbmf_save_libfm_binary_t if transpose else lib.sbmf_save_libfm_binary
    rc = fn(str(stem).encode(), C.byref(r), item_offset, num_cols)
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_loader_error().decode())


def save_triples(path, data):
    """Write the SBPMF triple format (u\ti\tr per line) that load_triples reads back bit for bit."""
    u, i = _u32(data.user), _u32(data.item)
    v = np.ascontiguousarray(data.rating, dtype=np.float64)
    r = _lib.Ratings()
    r.n = len(u)
    r.user = u.ctypes.data_as(C.POINTER(C.c_uint32))
    r.item = i.ctypes.data_as(C.POINTER(C.c_uint32))
    r.rating = v.ctypes.data_as(C.POINTER(C.c_double))
    rc = lib.sbmf_save_triples(str(path).encode(), C.byref(r))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_loader_error().decode())


def load_libfm(path, item_offset=0):
    """libFM text with one user and one item feature per line (Data.h:192-217)."""
    r = _lib.Ratings()
    rc = lib.sbmf_load_libfm(str(path).encode(), item_offset, C.byref(r))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_loader_error().decode())
    try:
        return _from_ratings(r)
    finally:
        lib.sbmf_free_ratings(C.byref(r))


def libfm_users_first(train, test=None):
    """libFM's attribute split of a users-first file loaded with item_offset=0:
    num_user = max first feature id + 1 over train and test (libfm.cpp:219-221,
    263-265,375).  Returns (train, test, num_user) with the item ids rebased onto
    num_user -- pass num_user as set_data(..., num_users=num_user) so libFM's
    learners see the file's attribute ids, as the CLI does.  A file whose item ids
    do not all lie above every user id has no users-first reading: ValueError."""
    sets = [d for d in (train, test) if d is not None and d.num_cases]
    if not sets:
        return train, test, 0
    I = max(int(np.max(d.user)) for d in sets) + 1
    for d in sets:
        if int(np.min(d.item)) < I:
            raise ValueError("libFM input: item feature id %d <= the largest user feature id %d: not users first"
                             % (int(np.min(d.item)), I - 1))
    rebase = lambda d: None if d is None else Data(d.user, np.asarray(d.item, np.int64) - I, d.rating)
    return rebase(train), rebase(test), I


def config_default():
    cfg = _lib.Config()
    lib.sbmf_config_default(C.byref(cfg))
    return cfg


class FMLearnSBPMF:
    """SBPMF Gibbs learner (fm_learn / fm_learn_mcmc shaped).

    Attributes mirror the reference: ``num_factor`` (K, -dim), ``num_iter``
    (-iter), ``seed``; plus the sampler's ``rng`` ("ref" | "philox"),
    ``quirks`` ("final" | "sbpmf2" | "none", or the biased sampler "bias2" |
    "bias22" = libFM ``-dim '1,1,K'``), ``precision`` ("f64" | "f32").
    ``rmse_trajectory`` collects the per-sweep running-mean test RMSE (the
    reference's ``rmse is`` lines / ``test_rmse_*`` file).
    """

    _QUIRKS = {"final": QUIRKS_FINAL, "sbpmf2": QUIRKS_SBPMF2, "none": QUIRKS_NONE, "bias2": QUIRKS_BIAS2,
               "bias22": QUIRKS_BIAS22}

    def __init__(self, num_factor=20, num_iter=100, seed=1, rng="ref", quirks="final", precision="f64", burnin=0,
                 device=0, init_stdev=None, recompute_every=1, eval_train=False,
                 stream_threshold=0, split_chunk=0, tune=0, method="mcmc", vb_batches=0, average="default",
                 order="sbpmf", k0=1, k1=1, regular=(0.0, 0.0, 0.0), **hyper):
        """method "mcmc" with order "sbpmf" (default): the SBPMF Gibbs sampler;
        method "mcmc" with order "libfm": libFM's own MCMC chain (f-outer, one
        hyperprior group, w0 / w with k0 / k1, -regular = ``regular``);
        "als": libFM's ALS (the same learner without sampling); "vb": online VB."""
        self.cfg = config_default()
        if method not in ("mcmc", "vb", "vb_online", "als") or order not in ("sbpmf", "libfm"):
            raise ValueError("method must be mcmc, als or vb (order sbpmf or libfm)")
        if method in ("vb", "vb_online"):
            self.cfg.method = METHOD_VB
        elif method == "als":
            self.cfg.method = METHOD_ALS
        else:
            self.cfg.method = METHOD_LIBFM_MCMC if order == "libfm" else METHOD_MCMC
        self.cfg.libfm_dim = (1 if k0 else 0) | (2 if k1 else 0)
        self.cfg.reg0, self.cfg.regw, self.cfg.regv = (float(x) for x in regular)
        self.cfg.vb_batches = vb_batches
        self.cfg.num_factor = num_factor
        self.cfg.num_iter = num_iter
        self.cfg.burnin = burnin
        self.cfg.seed = seed
        self.cfg.rng_mode = RNG_PHILOX if rng == "philox" else RNG_REFERENCE
        self.cfg.quirks = self._QUIRKS[quirks]
        self.cfg.precision = F32 if precision == "f32" else F64
        self.cfg.device = device
        if init_stdev is not None:
            self.cfg.init_stdev = init_stdev
        self.cfg.recompute_every = recompute_every
        self.cfg.eval_train = 1 if eval_train else 0
        self.cfg.stream_threshold = stream_threshold
        self.cfg.split_chunk = split_chunk
        self.cfg.tune = tune
        # running-mean divisor: "default" (quirk set), "collected" (collected sweeps), "reference" (sweep + 1)
        self.cfg.average = {"default": 0, "collected": 1, "reference": 2}[average]
        for k, v in hyper.items():
            setattr(self.cfg, k, v)
        self.ctx = None
        self.history = []
        self._train = self._test = None

    # -- fm_learn::init (fm_learn.h:80)
    def init(self, comm=None):
        if self.ctx is not None:
            return
        ctx = C.c_void_p()
        rc = lib.sbmf_create(C.byref(self.cfg), C.byref(ctx))
        if rc != SBMF_OK:
            raise SBMFError(rc, lib.sbmf_last_global_error().decode())
        self.ctx = ctx
        if isinstance(comm, Communicator):  # a process-wide communicator, shared by learners in turn
            self._comm = comm  # keeps it alive as long as this learner
            self._check(lib.sbmf_comm_attach(self.ctx, comm.handle))
        elif comm is not None:  # (nranks, rank, 128-byte id): a communicator of this learner's own
            nranks, rank, uid = comm
            buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
            self._check(lib.sbmf_comm_init(self.ctx, nranks, rank, buf))

    def _check(self, rc):
        if rc != SBMF_OK:
            raise SBMFError(rc, lib.sbmf_last_error(self.ctx).decode())

    def set_data(self, train, test=None, num_users=0, num_items=0):
        self.init()
        self._train, self._test = train, test
        self._check(lib.sbmf_set_train(self.ctx, train.num_cases, _ptr(train.user, C.c_uint32),
                                       _ptr(train.item, C.c_uint32), _ptr(train.rating, C.c_double)))
        if test is not None:
            self._check(lib.sbmf_set_test(self.ctx, test.num_cases, _ptr(test.user, C.c_uint32),
                                          _ptr(test.item, C.c_uint32), _ptr(test.rating, C.c_double)))
        if num_users or num_items:
            self._check(lib.sbmf_set_dims(self.ctx, num_users, num_items))
        self._check(lib.sbmf_prepare(self.ctx))

    # -- fm_learn::learn(train, test) (fm_learn.h:150; fm_learn_mcmc.h:1154)
    def learn(self, train=None, test=None, sweeps=None, callback=None):
        if train is not None:
            self.set_data(train, test)
        n = self.cfg.num_iter + self.cfg.burnin if sweeps is None else sweeps

        def _cb(info_p, _user):
            info = info_p.contents
            rec = {f: getattr(info, f) for f, _ in _lib.SweepInfo._fields_}
            self.history.append(rec)
            return 1 if (callback is not None and callback(rec)) else 0

        cb = _lib.SWEEP_CB(_cb)
        self._check(lib.sbmf_run(self.ctx, n, cb, None))
        return self.history

    @property
    def rmse_trajectory(self):
        return np.array([h["rmse_avg"] for h in self.history])

    # -- fm_learn::predict (fm_learn.h:191): averaged clamped predictions of the test set
    def predict(self):
        out = np.zeros(self._test.num_cases if self._test is not None else 0)
        self._check(lib.sbmf_predict(self.ctx, _ptr(out, C.c_double)))
        return out

    # -- fm_learn::evaluate (fm_learn.h:135): RMSE of the averaged prediction
    def evaluate(self):
        p = self.predict()
        return float(np.sqrt(np.mean((p - self._test.rating) ** 2)))

    def dims(self):
        nu, ni = C.c_uint32(), C.c_uint32()
        ntr, nte = C.c_uint64(), C.c_uint64()
        self._check(lib.sbmf_get_dims(self.ctx, C.byref(nu), C.byref(ni), C.byref(ntr), C.byref(nte)))
        return nu.value, ni.value, ntr.value, nte.value

    def factors(self):
        nu, ni, _, _ = self.dims()
        K = self.cfg.num_factor
        U = np.zeros((nu, K))
        V = np.zeros((ni, K))
        self._check(lib.sbmf_get_factors(self.ctx, _ptr(U, C.c_double), _ptr(V, C.c_double)))
        return U, V

    def set_factors(self, U, V):
        U, V = _f64(U), _f64(V)
        self._check(lib.sbmf_set_factors(self.ctx, _ptr(U, C.c_double), _ptr(V, C.c_double)))

    def hyper(self):
        K = self.cfg.num_factor
        h = np.zeros(4 * K)
        tau = C.c_double()
        self._check(lib.sbmf_get_hyper(self.ctx, _ptr(h, C.c_double), C.byref(tau)))
        return {"sigma_u": h[:K], "mu_u": h[K:2 * K], "sigma_v": h[2 * K:3 * K], "mu_v": h[3 * K:], "tau": tau.value}

    def biases(self):
        """Biased sampler: (b_i [users], b_j [items], b_0)."""
        nu, ni, _, _ = self.dims()
        bu, bv, b0 = np.zeros(nu), np.zeros(ni), C.c_double()
        self._check(lib.sbmf_get_biases(self.ctx, _ptr(bu, C.c_double), _ptr(bv, C.c_double), C.byref(b0)))
        return bu, bv, b0.value

    def timing(self):
        t = _lib.Timing()
        self._check(lib.sbmf_get_timing(self.ctx, C.byref(t)))
        return t

    def close(self):
        if self.ctx is not None:
            lib.sbmf_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FMLearnVBOnline(FMLearnSBPMF):
    """Online variational Bayes learner (the reference's fm_learn_vb_online,
    `bin/libFM -method vb_online`; src/libfm/src/fm_learn_vb_online.h).
    ``learn(sweeps=n)`` runs n epochs of 30 mini-batches; ``rmse_trajectory``
    holds the per-epoch test RMSE of the posterior-mean prediction,
    ``factors()`` / ``biases()`` the posterior means, ``hyper()["tau"]`` alpha."""

    def __init__(self, num_factor=8, num_iter=100, seed=1, rng="ref", device=0, vb_batches=0, **kw):
        super().__init__(num_factor=num_factor, num_iter=num_iter, seed=seed, rng=rng, device=device, method="vb",
                         vb_batches=vb_batches, **kw)


def device_usage(device=0):
    """sbmf_test_device_usage: hipMemGetInfo plus the library's live device / pinned
    buffers, streams, events, contexts and RCCL communicators (a dict)."""
    u = _lib.DeviceUsage()
    rc = lib.sbmf_test_device_usage(device, C.byref(u))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_last_global_error().decode())
    return {f: getattr(u, f) for f, _ in u._fields_}


class Communicator:
    """sbmf_comm_create: one RCCL communicator for the process (ncclCommInitRank once),
    attached in turn by every learner created with ``init(comm=<this>)``."""

    def __init__(self, nranks, rank, uid, device=0):
        h = C.c_void_p()
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        rc = lib.sbmf_comm_create(device, nranks, rank, buf, C.byref(h))
        if rc != SBMF_OK:
            raise SBMFError(rc, lib.sbmf_last_global_error().decode())
        self.handle, self.nranks, self.rank = h, nranks, rank

    def close(self):
        if self.handle is not None:
            lib.sbmf_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    buf = (C.c_uint8 * 128)()
    rc = lib.sbmf_comm_unique_id(buf)
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_last_global_error().decode())
    return bytes(buf)


def ref_stream(seed, kind, n, shape=1.0):
    """Host reference stream: kind 0 rand(), 1 ran_gaussian(), 2 ran_gamma(shape)."""
    out = np.zeros(n)
    rc = lib.sbmf_ref_stream(seed, kind, shape, n, _ptr(out, C.c_double))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_last_global_error().decode())
    return out


def partition_rows(ptr, nranks):
    """Row blocks [bounds[k], bounds[k+1]) of every rank (host-only, as the library partitions)."""
    ptr = _u32(ptr)
    out = np.zeros(nranks + 1, dtype=np.uint64)
    rc = lib.sbmf_partition_rows(_ptr(ptr, C.c_uint32), len(ptr) - 1, nranks, _ptr(out, C.c_uint64))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_last_global_error().decode())
    return out


def philox_normals(seed, sweep, tag, row, K):
    out = np.zeros(K)
    rc = lib.sbmf_philox_normals(seed, sweep, tag, row, K, _ptr(out, C.c_double))
    if rc != SBMF_OK:
        raise SBMFError(rc, lib.sbmf_last_global_error().decode())
    return out
