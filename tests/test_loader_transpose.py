"""libFM's transpose input (<stem>.xt + <stem>.y, or .datat + .target): the
file tools/transpose.cpp:54-172 writes and the only one bin/libFM -method
mcmc|als reads.  libfm.cpp:140-149 builds those data sets with has_x = false
(als is rewritten to mcmc first, :132-136), so Data::load (Data.h:112-117,
143-151) opens the transpose and never the row-major .x.

The fixtures are the reference's own data/m1m/m100k/{train,test}_libfm run
through tools/convert.cpp and tools/transpose.cpp compiled unmodified from
their sources (oracle/Makefile, `make_golden.py bindata`), so these tests pin
the reader and writer against the reference's bytes, not against a
restatement of the format."""
import gzip
import os
import struct
import subprocess

import numpy as np
import pytest

from conftest import GOLD, write_m1m100k_libfm
import sbmf
from sbmf._lib import CLI_PATH


def _fixture(tmp_path, nm, exts):
    """Decompress m1m100k_<nm>.<ext>.gz into tmp_path/<nm>.<ext>; returns the stem."""
    stem = str(tmp_path / nm)
    for ext in exts:
        with gzip.open(os.path.join(GOLD, "m1m100k_%s.%s.gz" % (nm, ext)), "rb") as f, open(stem + "." + ext, "wb") as g:
            g.write(f.read())
    return stem


@pytest.mark.parametrize("nm", ["train_libfm", "test_libfm"])
def test_transpose_equals_text_and_rowmajor(tmp_path, nm):
    """The .xt reader gives the text file's cases in file order (user = the lower feature
    id, item = the higher one minus the offset) and the same f32 targets as the .x reader."""
    write_m1m100k_libfm(tmp_path)
    (tmp_path / "b").mkdir()
    stem = _fixture(tmp_path / "b", nm, ("x", "y", "xt"))
    t = sbmf.load_libfm(str(tmp_path / nm), item_offset=943)
    x = sbmf.load_libfm_binary(stem, item_offset=943)
    xt = sbmf.load_libfm_binary(stem, item_offset=943, transpose=True)
    for d in (x, xt):
        assert np.array_equal(d.user, t.user) and np.array_equal(d.item, t.item)
        assert np.array_equal(d.rating, t.rating)
    assert t.num_cases == (79999 if nm == "train_libfm" else 19999)
    raw = sbmf.load_libfm_binary(stem, transpose=True)  # offset 0: raw feature ids
    assert np.array_equal(raw.item, t.item + 943)


@pytest.mark.parametrize("nm", ["train_libfm", "test_libfm"])
def test_writer_is_byte_identical_to_convert_and_transpose(tmp_path, nm):
    """save_libfm_binary(transpose=True) writes exactly the reference tools' .xt and .y, and
    the row-major writer exactly convert's .x (same num_cols: max feature id + 1)."""
    stem = _fixture(tmp_path, nm, ("x", "y", "xt"))
    d = sbmf.load_libfm_binary(stem, transpose=True)
    out = str(tmp_path / "mine")
    sbmf.save_libfm_binary(out, d, transpose=True)
    assert open(out + ".xt", "rb").read() == open(stem + ".xt", "rb").read()
    assert open(out + ".y", "rb").read() == open(stem + ".y", "rb").read()
    sbmf.save_libfm_binary(out, d)
    assert open(out + ".x", "rb").read() == open(stem + ".x", "rb").read()


def test_transpose_header_roles(tmp_path):
    """transpose.cpp:104-110: num_rows = features (the .x's num_cols), num_cols = cases."""
    stem = _fixture(tmp_path, "train_libfm", ("x", "xt"))
    fx = struct.unpack_from("<IIQII", open(stem + ".x", "rb").read(24))
    ft = struct.unpack_from("<IIQII", open(stem + ".xt", "rb").read(24))
    assert fx[:3] == ft[:3] == (2, 4, 159998)
    assert (ft[3], ft[4]) == (fx[4], fx[3]) == (2625, 79999)


def test_file_choice_is_data_load(tmp_path):
    """Data.h:112-117: .data[/.datat]/.target first, then .x[/.xt]/.y, each orientation
    required only when the set needs it; otherwise text (0)."""
    s = str(tmp_path / "s")
    k = sbmf.libfm_binary_kind
    assert (k(s, 0, 1), k(s, 1, 1), k(s, 1, 0)) == (0, 0, 0)
    for ext in ("x", "y"):
        open(s + "." + ext, "wb").close()
    assert (k(s, 0, 1), k(s, 1, 1), k(s, 1, 0)) == (0, 0, 2)  # mcmc needs the transpose
    open(s + ".xt", "wb").close()
    assert (k(s, 0, 1), k(s, 1, 1), k(s, 1, 0)) == (2, 2, 2)
    for ext in ("datat", "target"):
        open(s + "." + ext, "wb").close()
    assert (k(s, 0, 1), k(s, 1, 1), k(s, 1, 0)) == (1, 2, 2)  # .data missing: has_x sets fall to .x/.xt
    open(s + ".data", "wb").close()
    assert (k(s, 0, 1), k(s, 1, 1), k(s, 1, 0)) == (1, 1, 1)
    with pytest.raises(sbmf.SBMFError):
        k(s, 0, 0)


def test_load_libfm_data_reads_what_data_load_reads(tmp_path):
    """The MCMC / ALS set (has_x = 0) reads the transpose even beside a different .x; the
    row-major set reads the .x; with no binary files the stem is parsed as text."""
    import ctypes as C
    stem = _fixture(tmp_path, "test_libfm", ("xt", "y"))
    d = sbmf.load_libfm_binary(stem, item_offset=943, transpose=True)
    # a decoy .x beside it: the same cases with the users rolled by one (only has_x sets may read it)
    decoy = str(tmp_path / "decoy")
    sbmf.save_libfm_binary(decoy, sbmf.Data(np.roll(d.user, 1), d.item, d.rating), item_offset=943)
    os.replace(decoy + ".x", stem + ".x")

    def load(st, hx, ht):
        r = sbmf._lib.Ratings()
        rc = sbmf.lib.sbmf_load_libfm_data(st.encode(), hx, ht, 943, C.byref(r))
        assert rc == sbmf.SBMF_OK, sbmf.lib.sbmf_loader_error().decode()
        u = np.ctypeslib.as_array(r.user, (r.n,)).copy()
        sbmf.lib.sbmf_free_ratings(C.byref(r))
        return u
    assert np.array_equal(load(stem, 0, 1), d.user)  # the MCMC / ALS set: the transpose
    assert np.array_equal(load(stem, 1, 1), np.roll(d.user, 1))  # .x + .xt + .y: the row-major set reads .x
    (tmp_path / "t").mkdir()
    write_m1m100k_libfm(tmp_path / "t")
    assert np.array_equal(load(str(tmp_path / "t" / "test_libfm"), 0, 1), d.user)  # text


def _write_xt(path, rows, num_cases, nv=None):
    with open(path, "wb") as f:
        f.write(struct.pack("<IIQII", 2, 4, sum(len(r) for r in rows) if nv is None else nv, len(rows), num_cases))
        for r in rows:
            f.write(struct.pack("<I", len(r)))
            for c in r:
                f.write(struct.pack("<If", c, 1.0))


def _write_y(path, y):
    with open(path, "wb") as f:
        f.write(struct.pack("<III", 1, 4, len(y)))
        f.write(np.asarray(y, np.float32).tobytes())


def test_transpose_errors(tmp_path):
    s = str(tmp_path / "e")
    _write_y(s + ".y", [5.0, 3.0])
    # case 1 has three features
    _write_xt(s + ".xt", [[0], [1], [0, 1], [1]], 2)
    with pytest.raises(sbmf.SBMFError, match="case 1"):
        sbmf.load_libfm_binary(s, transpose=True)
    # a case id past the targets
    _write_xt(s + ".xt", [[0], [1, 2], [0, 1]], 2)
    with pytest.raises(sbmf.SBMFError, match="past the 2 targets"):
        sbmf.load_libfm_binary(s, transpose=True)
    # targets and cases disagree
    _write_xt(s + ".xt", [[0], [1], [0, 1]], 3)
    with pytest.raises(sbmf.SBMFError, match="3 cases but 2 targets"):
        sbmf.load_libfm_binary(s, transpose=True)
    # header value count wrong / truncated
    _write_xt(s + ".xt", [[0], [1], [0, 1]], 2, nv=5)
    with pytest.raises(sbmf.SBMFError, match="header says 5"):
        sbmf.load_libfm_binary(s, transpose=True)
    raw = open(s + ".xt", "rb").read()
    open(s + ".xt", "wb").write(raw[:-3])
    with pytest.raises(sbmf.SBMFError, match="truncated"):
        sbmf.load_libfm_binary(s, transpose=True)
    # the item offset splits users from items: user 0, item 2 - 2 = 0; user 1, item 0
    _write_xt(s + ".xt", [[0], [1], [0, 1]], 2)
    d = sbmf.load_libfm_binary(s, item_offset=2, transpose=True)
    assert d.user.tolist() == [0, 1] and d.item.tolist() == [0, 0] and d.rating.tolist() == [5.0, 3.0]
    with pytest.raises(sbmf.SBMFError, match="user id < item_offset"):
        sbmf.load_libfm_binary(s, item_offset=1, transpose=True)
    # an empty set
    _write_y(s + ".y", [])
    _write_xt(s + ".xt", [[], []], 0)
    assert sbmf.load_libfm_binary(s, transpose=True).num_cases == 0


def test_cli_reads_the_transpose_before_the_device(tmp_path):
    """bin/libFM's argv on a directory holding only .xt + .y: the loader takes the transpose
    (a missing or broken file would fail here, before the device check on a CPU-only host)."""
    for nm in ("train_libfm", "test_libfm"):
        _fixture(tmp_path, nm, ("xt", "y"))
    cmd = [CLI_PATH, "-task", "r", "-train", "train_libfm", "-test", "test_libfm", "-dim", "1,1,8", "-iter", "2",
           "-method", "mcmc"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    if r.returncode == 0:  # a GPU host: the run itself is test_gpu_cli's
        return
    assert "no HIP device" in r.stderr, r.stderr
    # a broken transpose surfaces as the loader's error, not as a device error
    raw = open(tmp_path / "train_libfm.xt", "rb").read()
    open(tmp_path / "train_libfm.xt", "wb").write(raw[:1000])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert r.returncode == 1 and "truncated" in r.stderr, r.stderr
