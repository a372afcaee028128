"""libFM binary input (<stem>.x + <stem>.y, or .data + .target), the format
tools/convert.cpp:55-205 writes and Data::load reads (Data.h:113-160).  The
byte layouts are restated here with struct (fmatrix.h:36-52 file_header and
sparse rows, matrix.h:280-328 DVector), independently of the library's writer,
and checked against the text libFM loader on the same ratings.  No reference
binary files ship with the reference, so these vectors are synthetic."""
import os
import struct

import numpy as np
import pytest

from conftest import GOLD, read_triples_text
import sbmf


def write_x(path, rows, num_cols, fid=2, fsize=4, num_values=None):
    nv = sum(len(r) for r in rows) if num_values is None else num_values
    with open(path, "wb") as f:
        f.write(struct.pack("<IIQII", fid, fsize, nv, len(rows), num_cols))
        for r in rows:
            f.write(struct.pack("<I", len(r)))
            for fid_, v in r:
                f.write(struct.pack("<If", fid_, v))


def write_y(path, y, version=1, fsize=4, n=None):
    with open(path, "wb") as f:
        f.write(struct.pack("<III", version, fsize, len(y) if n is None else n))
        f.write(np.asarray(y, np.float32).tobytes())


def test_header_is_24_bytes():
    assert struct.calcsize("<IIQII") == 24


def test_handbuilt_files_match_text_loader(tmp_path):
    u, i, r = read_triples_text(os.path.join(GOLD, "ragged_train.tsv"))
    off = int(u.max()) + 1
    stem = str(tmp_path / "ragged")
    write_x(stem + ".x", [[(int(a), 1.0), (off + int(b), 1.0)] for a, b in zip(u, i)], off + int(i.max()) + 1)
    write_y(stem + ".y", r)
    d = sbmf.load_libfm_binary(stem, item_offset=off)
    txt = tmp_path / "ragged.libfm"
    txt.write_text("".join("%r %d:1 %d:1\n" % (float(np.float32(v)), a, off + b) for a, b, v in zip(u, i, r)))
    t = sbmf.load_libfm(txt, item_offset=off)
    assert np.array_equal(d.user, u) and np.array_equal(d.item, i)
    assert np.array_equal(d.rating, r.astype(np.float32).astype(np.float64))
    assert np.array_equal(d.user, t.user) and np.array_equal(d.item, t.item)
    assert np.array_equal(d.rating, t.rating)


def test_writer_round_trip_and_layout(tmp_path):
    u, i, r = read_triples_text(os.path.join(GOLD, "ragged_train.tsv"))
    stem = str(tmp_path / "rt")
    sbmf.save_libfm_binary(stem, sbmf.Data(u, i, r), item_offset=1000)
    raw = open(stem + ".x", "rb").read()
    fid, fsize, nv, nrows, ncols = struct.unpack_from("<IIQII", raw, 0)
    assert (fid, fsize, nv, nrows) == (2, 4, 2 * len(u), len(u))
    assert ncols == 1000 + int(i.max()) + 1
    assert len(raw) == 24 + len(u) * (4 + 16)
    sz, a, va, b, vb = struct.unpack_from("<IIfIf", raw, 24)
    assert (sz, a, va, b, vb) == (2, u[0], 1.0, 1000 + i[0], 1.0)
    d = sbmf.load_libfm_binary(stem, item_offset=1000)
    assert np.array_equal(d.user, u) and np.array_equal(d.item, i)
    assert np.array_equal(d.rating, r.astype(np.float32).astype(np.float64))


def test_data_target_preferred_over_x_y(tmp_path):
    stem = str(tmp_path / "s")
    write_x(stem + ".x", [[(0, 1.0), (5, 1.0)]], 6)
    write_y(stem + ".y", [1.0])
    write_x(stem + ".data", [[(1, 1.0), (6, 1.0)], [(2, 1.0), (7, 1.0)]], 8)
    write_y(stem + ".target", [4.0, 2.5])
    d = sbmf.load_libfm_binary(stem, item_offset=5)
    assert d.user.tolist() == [1, 2] and d.item.tolist() == [1, 2] and d.rating.tolist() == [4.0, 2.5]


def test_empty_file_pair(tmp_path):
    stem = str(tmp_path / "e")
    write_x(stem + ".x", [], 0)
    write_y(stem + ".y", [])
    assert sbmf.load_libfm_binary(stem).num_cases == 0


@pytest.mark.parametrize("case", ["bad_id", "bad_float", "row_mismatch", "three_features", "one_feature",
                                  "item_below_offset", "two_items", "truncated", "num_values", "bad_y"])
def test_errors(tmp_path, case):
    stem = str(tmp_path / "b")
    rows = [[(0, 1.0), (9, 1.0)], [(1, 1.0), (10, 1.0)]]
    y = [5.0, 3.0]
    kw = {}
    if case == "bad_id":
        kw = {"fid": 1}
    elif case == "bad_float":
        kw = {"fsize": 8}
    elif case == "three_features":
        rows[1] = rows[1] + [(11, 1.0)]
    elif case == "one_feature":
        rows[0] = rows[0][:1]
    elif case == "item_below_offset":
        rows[0] = [(0, 1.0), (3, 1.0)]
    elif case == "two_items":  # both features in the item range: not a user id (item_offset 9)
        rows[0] = [(10, 1.0), (11, 1.0)]
    elif case == "num_values":
        kw = {"num_values": 5}
    write_x(stem + ".x", rows, 12, **kw)
    if case == "truncated":
        raw = open(stem + ".x", "rb").read()
        open(stem + ".x", "wb").write(raw[:-6])
    write_y(stem + ".y", y, **({"n": 3} if case == "row_mismatch" else {"version": 2} if case == "bad_y" else {}))
    with pytest.raises(sbmf.SBMFError):
        sbmf.load_libfm_binary(stem, item_offset=9)


def test_missing_pair(tmp_path):
    with pytest.raises(sbmf.SBMFError) as e:
        sbmf.load_libfm_binary(str(tmp_path / "nothing"))
    assert "unable to open" in str(e.value)


def test_writer_refuses_ids_that_would_wrap(tmp_path):
    """Feature ids are uint32 in the .x format and num_cols = max id + 1: ids
    that would wrap are refused (no silently wrong files)."""
    stem = str(tmp_path / "w")
    with pytest.raises(ValueError):  # item_offset + item past 2^32 - 2
        sbmf.save_libfm_binary(stem, sbmf.Data([0], [5], [3.0]), item_offset=0xfffffffc)
    assert not os.path.exists(stem + ".x")
    with pytest.raises(ValueError):  # negative ids never reach the uint32 cast
        sbmf.Data([-1], [0], [3.0])
    with pytest.raises(ValueError):
        sbmf.Data([2 ** 32], [0], [3.0])
    # the C entry point checks on its own (64-bit arithmetic)
    import ctypes as C
    from sbmf import _lib
    u = np.array([0], np.uint32)
    i = np.array([0xfffffffe], np.uint32)
    v = np.array([3.0])
    r = _lib.Ratings()
    r.n, r.user, r.item = 1, u.ctypes.data_as(C.POINTER(C.c_uint32)), i.ctypes.data_as(C.POINTER(C.c_uint32))
    r.rating = v.ctypes.data_as(C.POINTER(C.c_double))
    assert sbmf.lib.sbmf_save_libfm_binary(stem.encode(), C.byref(r), 1, 0) == sbmf.SBMF_E_ARG
    assert not os.path.exists(stem + ".x")
