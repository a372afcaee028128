"""ctypes binding of include/sbmf.h (the drop-in C ABI).

Loads ``../build/libsbmf.so`` (built in-tree by ``csrc/Makefile`` /
``__graft_entry__.build()``).  There is no pure-Python fallback: if the
library is missing, importing this module raises.
"""
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SBMF_LIB", os.path.join(PKG_DIR, "build", "libsbmf.so"))
CLI_PATH = os.path.join(PKG_DIR, "build", "sbmf")

SBMF_OK, SBMF_E_ARG, SBMF_E_STATE, SBMF_E_DEVICE, SBMF_E_IO, SBMF_E_COMM, SBMF_E_NOMEM = 0, -1, -2, -3, -4, -5, -6
RNG_REFERENCE, RNG_PHILOX = 0, 1
QUIRKS_FINAL, QUIRKS_SBPMF2, QUIRKS_NONE, QUIRKS_BIAS2, QUIRKS_BIAS22 = 0, 1, 2, 3, 4
F64, F32 = 0, 1
METHOD_MCMC, METHOD_VB, METHOD_LIBFM_MCMC, METHOD_ALS = 0, 1, 2, 3
NKIND = 11  # SBMF_NKIND
KIND_NAMES = ['gblock_w4', 'gblock_w16', 'gblock_b2', 'gblock_b4', 'gblock_b8', 'gres_stage', 'rows_w2', 'rows_w8',
              'rows_b4', 'rows_b8', 'gram']


class Config(C.Structure):
    _fields_ = [
        ("num_factor", C.c_uint32), ("num_iter", C.c_uint32), ("burnin", C.c_uint32), ("seed", C.c_uint64),
        ("rng_mode", C.c_int32), ("quirks", C.c_int32), ("precision", C.c_int32), ("device", C.c_int32),
        ("init_stdev", C.c_double), ("clamp_lo", C.c_double), ("clamp_hi", C.c_double),
        ("a0", C.c_double), ("b0", C.c_double), ("alpha0", C.c_double), ("beta0", C.c_double),
        ("nu0", C.c_double), ("mu0", C.c_double),
        ("recompute_every", C.c_uint32), ("eval_train", C.c_uint32), ("eval_test", C.c_uint32),
        ("gram_threshold", C.c_uint32), ("row_kernel", C.c_uint32), ("stream_threshold", C.c_uint32),
        ("split_chunk", C.c_uint32), ("tune", C.c_uint32), ("method", C.c_uint32), ("vb_batches", C.c_uint32),
        ("average", C.c_uint32), ("libfm_dim", C.c_uint32), ("reg0", C.c_double), ("regw", C.c_double),
        ("regv", C.c_double), ("pipeline", C.c_uint32),
    ]


class SweepInfo(C.Structure):
    _fields_ = [
        ("sweep", C.c_uint32), ("collected", C.c_uint32), ("rmse_avg", C.c_double), ("rmse_this", C.c_double),
        ("rmse_train", C.c_double), ("tau", C.c_double), ("ms_sweep", C.c_double), ("ms_eval", C.c_double),
    ]


class Timing(C.Structure):
    _fields_ = [
        ("ms_user_half", C.c_double), ("ms_item_half", C.c_double), ("ms_hyper", C.c_double),
        ("ms_eval", C.c_double), ("ms_comm", C.c_double),
        ("kern_ms", (C.c_double * NKIND) * 2), ("kern_bytes", (C.c_uint64 * NKIND) * 2),
        ("kern_rows", (C.c_uint32 * NKIND) * 2),
        ("bytes_algorithmic", C.c_uint64), ("n_launch", C.c_uint32), ("ms_vb_factor", C.c_double),
    ]


class Ratings(C.Structure):
    _fields_ = [("n", C.c_uint64), ("user", C.POINTER(C.c_uint32)), ("item", C.POINTER(C.c_uint32)),
                ("rating", C.POINTER(C.c_double))]


SWEEP_CB = C.CFUNCTYPE(C.c_int, C.POINTER(SweepInfo), C.c_void_p)

_P_U32 = C.POINTER(C.c_uint32)
_P_F64 = C.POINTER(C.c_double)
_P_U8 = C.POINTER(C.c_uint8)

# name -> (restype, argtypes); every function declared in include/sbmf.h
class RcclSelftest(C.Structure):
    _fields_ = [
        ("ms_half", C.c_double), ("ms_rccl", C.c_double), ("ms_rccl_end", C.c_double),
        ("bad_bcast", C.c_uint64), ("bad_p2p", C.c_uint64), ("bad_allgather", C.c_uint64),
        ("n_calls", C.c_uint32), ("overlapped", C.c_uint32),
    ]


class DeviceUsage(C.Structure):
    _fields_ = [
        ("device_free", C.c_uint64), ("device_total", C.c_uint64),
        ("dev_bytes", C.c_int64), ("dev_allocs", C.c_int64), ("pinned_bytes", C.c_int64),
        ("pinned_allocs", C.c_int64), ("streams", C.c_int64), ("events", C.c_int64),
        ("contexts", C.c_int64), ("comms", C.c_int64),
    ]


SIGNATURES = {
    "sbmf_config_default": (C.c_int, [C.POINTER(Config)]),
    "sbmf_create": (C.c_int, [C.POINTER(Config), C.POINTER(C.c_void_p)]),
    "sbmf_destroy": (None, [C.c_void_p]),
    "sbmf_last_error": (C.c_char_p, [C.c_void_p]),
    "sbmf_last_global_error": (C.c_char_p, []),
    "sbmf_abi_version": (C.c_int, []),
    "sbmf_exit_guard": (C.c_int, [C.c_int]),
    "sbmf_set_train": (C.c_int, [C.c_void_p, C.c_uint64, _P_U32, _P_U32, _P_F64]),
    "sbmf_set_test": (C.c_int, [C.c_void_p, C.c_uint64, _P_U32, _P_U32, _P_F64]),
    "sbmf_set_dims": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "sbmf_prepare": (C.c_int, [C.c_void_p]),
    "sbmf_run": (C.c_int, [C.c_void_p, C.c_uint32, SWEEP_CB, C.c_void_p]),
    "sbmf_predict": (C.c_int, [C.c_void_p, _P_F64]),
    "sbmf_get_factors": (C.c_int, [C.c_void_p, _P_F64, _P_F64]),
    "sbmf_set_factors": (C.c_int, [C.c_void_p, _P_F64, _P_F64]),
    "sbmf_get_hyper": (C.c_int, [C.c_void_p, _P_F64, _P_F64]),
    "sbmf_get_biases": (C.c_int, [C.c_void_p, _P_F64, _P_F64, _P_F64]),
    "sbmf_get_dims": (C.c_int, [C.c_void_p, _P_U32, _P_U32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "sbmf_get_timing": (C.c_int, [C.c_void_p, C.POINTER(Timing)]),
    "sbmf_comm_unique_id": (C.c_int, [_P_U8]),
    "sbmf_comm_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _P_U8]),
    "sbmf_comm_create": (C.c_int, [C.c_int, C.c_int, C.c_int, _P_U8, C.POINTER(C.c_void_p)]),
    "sbmf_comm_attach": (C.c_int, [C.c_void_p, C.c_void_p]),
    "sbmf_comm_destroy": (None, [C.c_void_p]),
    "sbmf_load_triples": (C.c_int, [C.c_char_p, C.POINTER(Ratings)]),
    "sbmf_load_libfm": (C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(Ratings)]),
    "sbmf_load_libfm_binary": (C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(Ratings)]),
    "sbmf_save_libfm_binary": (C.c_int, [C.c_char_p, C.POINTER(Ratings), C.c_uint32, C.c_uint32]),
    "sbmf_load_libfm_binary_t": (C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(Ratings)]),
    "sbmf_save_libfm_binary_t": (C.c_int, [C.c_char_p, C.POINTER(Ratings), C.c_uint32, C.c_uint32]),
    "sbmf_libfm_binary_kind": (C.c_int, [C.c_char_p, C.c_int, C.c_int]),
    "sbmf_load_libfm_data": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_uint32, C.POINTER(Ratings)]),
    "sbmf_save_triples": (C.c_int, [C.c_char_p, C.POINTER(Ratings)]),
    "sbmf_free_ratings": (None, [C.POINTER(Ratings)]),
    "sbmf_partition_rows": (C.c_int, [_P_U32, C.c_uint32, C.c_int, C.POINTER(C.c_uint64)]),
    "sbmf_ref_stream": (C.c_int, [C.c_uint32, C.c_int, C.c_double, C.c_uint64, _P_F64]),
    "sbmf_philox_normals": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P_F64]),
    "sbmf_test_virtual_rank": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "sbmf_test_stage_ms": (C.c_int, [C.c_void_p, _P_F64, C.c_uint32, C.POINTER(C.c_uint32)]),
    "sbmf_test_rccl_selftest": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_double, C.POINTER(RcclSelftest)]),
    "sbmf_test_device_usage": (C.c_int, [C.c_int, C.POINTER(DeviceUsage)]),
}


def load(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError("libsbmf.so not built at %s: run __graft_entry__.build() "
                          "(or make -C scalable-bayesian-matrix-factorization_amd/csrc)" % path)
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib.sbmf_loader_error.restype = C.c_char_p
    lib.sbmf_loader_error.argtypes = []
    return lib


lib = load()


_guarded = False


def exit_guard(rc):
    """sbmf_exit_guard (include/sbmf.h): the first call, before anything starts
    the HIP runtime, makes the process leave with exit status rc once the exit
    handlers registered after it (rocprofv3 writes its output in one) have
    run, skipping the shared-library finalizers (the HIP runtime's faults under
    rocprofv3, ROCm 7.2: profiles/r03_rocprof_teardown.txt); later calls set
    rc.  For programs (bench.py), not for a library user's process."""
    global _guarded
    if lib.sbmf_exit_guard(int(rc)) != 0:
        raise RuntimeError(lib.sbmf_last_global_error().decode())
    _guarded = True


def unload():
    """dlclose libsbmf (every learner closed first; the module is unusable
    after).  A no-op once exit_guard is installed: the handler lives in libsbmf."""
    global lib
    import _ctypes
    if lib is not None and not _guarded:
        _ctypes.dlclose(lib._handle)
        lib = None
