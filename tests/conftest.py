import gzip
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "scalable-bayesian-matrix-factorization_amd")
GOLD = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    if not os.path.exists(os.path.join(PKG, "build", "libsbmf.so")):
        subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j8"], check=True, capture_output=True)
    if not os.path.exists(os.path.join(REPO, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "all"], check=True, capture_output=True)


_ensure_built()


def read_triples_text(path):
    opener = gzip.open if path.endswith(".gz") else open
    u, i, r = [], [], []
    with opener(path, "rt") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 3:
                u.append(int(parts[0]))
                i.append(int(parts[1]))
                r.append(float(parts[2]))
    return np.array(u, np.uint32), np.array(i, np.uint32), np.array(r, np.float64)


@pytest.fixture(scope="session")
def ml100k():
    tr = read_triples_text(os.path.join(GOLD, "ml100k_train.tsv.gz"))
    te = read_triples_text(os.path.join(GOLD, "ml100k_test.tsv.gz"))
    return tr, te


@pytest.fixture(scope="session")
def ragged():
    tr = read_triples_text(os.path.join(GOLD, "ragged_train.tsv"))
    te = read_triples_text(os.path.join(GOLD, "ragged_test.tsv"))
    return tr, te


def read_libfm_text(path):
    """libFM text "r a:1 b:1" -> (first feature id, second feature id, target)."""
    opener = gzip.open if path.endswith(".gz") else open
    u, i, r = [], [], []
    with opener(path, "rt") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 3:
                r.append(float(parts[0]))
                u.append(int(parts[1].split(":")[0]))
                i.append(int(parts[2].split(":")[0]))
    return np.array(u, np.uint32), np.array(i, np.uint32), np.array(r, np.float64)


@pytest.fixture(scope="session")
def m1m100k():
    """The reference's own data/m1m/m100k/{train,test}_libfm (tests/golden/m1m100k_*_libfm.gz):
    users 0..942 as the first feature, items at their raw feature ids 943..2624.  Triples with
    the raw item ids are also exactly the {train,test}_sbpmf its converter writes."""
    return (read_libfm_text(os.path.join(GOLD, "m1m100k_train_libfm.gz")),
            read_libfm_text(os.path.join(GOLD, "m1m100k_test_libfm.gz")))


def write_m1m100k_libfm(dirpath):
    """Decompress the reference's libFM files into dirpath as train_libfm / test_libfm."""
    out = []
    for nm in ("train_libfm", "test_libfm"):
        dst = os.path.join(str(dirpath), nm)
        with gzip.open(os.path.join(GOLD, "m1m100k_%s.gz" % nm), "rb") as f, open(dst, "wb") as g:
            g.write(f.read())
        out.append(dst)
    return out


def golden_rmse(name):
    with open(os.path.join(GOLD, name)) as f:
        return np.array([float(x) for x in f.read().split()])


def gpu_available():
    """Device probe through the HIP runtime libsbmf is bound to (not torch's:
    initialising torch's bundled runtime first leaves a second HSA runtime in
    the process that then sees no device)."""
    import ctypes
    from sbmf import _lib  # noqa: F401  (binds libamdhip64.so.7 first)
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
    except OSError:
        return False
    n = ctypes.c_int(0)
    return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
