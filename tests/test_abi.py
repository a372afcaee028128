"""The drop-in C ABI: library loads, exports every function include/sbmf.h
declares, ctypes struct layouts match the C compiler's, defaults match the
reference constants, and compute entry points fail loudly without a GPU."""
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO, gpu_available
import sbmf
from sbmf import _lib

HEADER = os.path.join(REPO, "include", "sbmf.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sbmf_[a-z_0-9]+)\s*\(", text)) - {"sbmf_sweep_cb"})


def test_every_declared_symbol_is_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (sbmf_\w+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    assert set(_lib.SIGNATURES) <= exported


def test_ctypes_signatures_cover_header():
    assert set(declared_functions()) <= set(_lib.SIGNATURES) | {"sbmf_loader_error"}


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "sbmf.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(sbmf_config), sizeof(sbmf_sweep_info), sizeof(sbmf_timing),
         sizeof(sbmf_ratings), offsetof(sbmf_config, init_stdev), offsetof(sbmf_config, recompute_every),
         offsetof(sbmf_timing, bytes_algorithmic));
  printf("%zu %zu %zu %zu\n", offsetof(sbmf_config, method), offsetof(sbmf_config, vb_batches),
         offsetof(sbmf_config, libfm_dim), offsetof(sbmf_config, regv));
  return 0; }''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    import ctypes as C
    want = [C.sizeof(_lib.Config), C.sizeof(_lib.SweepInfo), C.sizeof(_lib.Timing), C.sizeof(_lib.Ratings),
            _lib.Config.init_stdev.offset, _lib.Config.recompute_every.offset, _lib.Timing.bytes_algorithmic.offset,
            _lib.Config.method.offset, _lib.Config.vb_batches.offset, _lib.Config.libfm_dim.offset,
            _lib.Config.regv.offset]
    assert got == want


def test_defaults_are_the_reference_constants():
    c = sbmf.config_default()
    # gibbs_sbpmf_final.cpp:218 (D=20), :256-269 (hyperpriors), :299-300 (100 sweeps, no burn-in)
    assert (c.num_factor, c.num_iter, c.burnin) == (20, 100, 0)
    assert (c.a0, c.b0, c.alpha0, c.beta0, c.nu0, c.mu0) == (1, 1, 1, 1, 1, 0)
    assert c.clamp_hi == 5.0 and c.rng_mode == sbmf.RNG_REFERENCE and c.quirks == sbmf.QUIRKS_FINAL
    assert c.precision == sbmf.F64
    assert c.method == sbmf._lib.METHOD_MCMC and c.vb_batches == 0
    # libfm.cpp:130 (-dim 1,1,K), :484-490 (no -regular: 0)
    assert c.libfm_dim == 3 and (c.reg0, c.regw, c.regv) == (0.0, 0.0, 0.0)
    assert _lib.lib.sbmf_abi_version() == 2


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_no_cpu_fallback_without_gpu():
    L = sbmf.FMLearnSBPMF()
    with pytest.raises(sbmf.SBMFError) as ei:
        L.init()
    assert ei.value.code == sbmf.SBMF_E_DEVICE
    assert "no HIP device" in str(ei.value)


def test_bad_config_rejected_before_device():
    import ctypes as C
    cfg = sbmf.config_default()
    cfg.num_factor = 0
    ctx = C.c_void_p()
    assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG
    cfg.num_factor = 300
    assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG
    cfg = sbmf.config_default()
    cfg.method = 7
    assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG
    cfg.method = sbmf._lib.METHOD_VB
    cfg.precision = sbmf.F32  # the VB learner is f64 only
    assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG
    for m in (sbmf._lib.METHOD_LIBFM_MCMC, sbmf._lib.METHOD_ALS):  # so are libFM's MCMC and ALS
        cfg.method = m
        assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG
    cfg = sbmf.config_default()
    cfg.method = sbmf._lib.METHOD_ALS
    cfg.libfm_dim = 4
    assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG


def test_removed_row_kernels_are_refused():
    """row_kernel / gram_threshold are reserved since the per-coordinate and
    full-Gram row kernels were removed (round 4): a non-zero value fails with
    SBMF_E_ARG before any device is touched (so on CPU too)."""
    import sbmf
    for kw in ({"row_kernel": 1}, {"gram_threshold": 64}):
        L = sbmf.FMLearnSBPMF(num_factor=8, **kw)
        with pytest.raises(sbmf.SBMFError) as e:
            L.init()
        assert e.value.code == sbmf.SBMF_E_ARG and "reserved" in str(e.value)


def test_unassigned_tune_bits_are_refused():
    """A tune bit that selects nothing in this build (a variant removed in an earlier
    round) fails with SBMF_E_ARG before any device is touched, instead of being ignored
    or picking whatever the bit means now."""
    import ctypes as C
    ctx = C.c_void_p()
    for bit in (0, 4, 5, 6, 15, 16, 18, 19, 20, 21, 22, 31):
        cfg = sbmf.config_default()
        cfg.tune = 1 << bit
        assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_ARG, bit
        assert "tune bits" in _lib.lib.sbmf_last_global_error().decode()
    if not gpu_available():  # an assigned bit passes the check and reaches the device check
        cfg = sbmf.config_default()
        cfg.tune = (1 << 17) | (1 << 29)
        assert _lib.lib.sbmf_create(C.byref(cfg), C.byref(ctx)) == sbmf.SBMF_E_DEVICE


def test_shared_communicator_entry_points_check_arguments():
    """sbmf_comm_create / sbmf_comm_attach (one RCCL communicator per process, attached by
    every context in turn): bad ranks and null handles fail before any RCCL call."""
    import ctypes as C
    h = C.c_void_p()
    uid = (C.c_uint8 * 128)()
    assert _lib.lib.sbmf_comm_create(0, 2, 2, uid, C.byref(h)) == sbmf.SBMF_E_ARG
    assert _lib.lib.sbmf_comm_create(0, 0, 0, uid, C.byref(h)) == sbmf.SBMF_E_ARG
    assert _lib.lib.sbmf_comm_create(0, 1, 0, None, C.byref(h)) == sbmf.SBMF_E_ARG
    assert _lib.lib.sbmf_comm_create(-1, 1, 0, uid, C.byref(h)) == sbmf.SBMF_E_ARG
    # a one-rank communicator is a no-op object (no RCCL): created and destroyed without a device
    assert _lib.lib.sbmf_comm_create(0, 1, 0, uid, C.byref(h)) == sbmf.SBMF_OK and h.value
    assert _lib.lib.sbmf_comm_attach(None, h) == sbmf.SBMF_E_ARG
    _lib.lib.sbmf_comm_destroy(h)
