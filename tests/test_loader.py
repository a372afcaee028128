"""Input formats of the boundary: SBPMF triples (acceptance rule of
gibbs_sbpmf_final.cpp:43: sscanf("%u%c%u%c%lf") >= 5) and libFM text with one
user and one item feature per line (Data.h:192-217)."""
import gzip
import os

import numpy as np
import pytest

import oracle
from conftest import GOLD
import sbmf


def test_triples_match_oracle_sscanf_on_ml100k(tmp_path):
    p = tmp_path / "train.tsv"
    with gzip.open(os.path.join(GOLD, "ml100k_train.tsv.gz"), "rb") as f:
        p.write_bytes(f.read())
    d = sbmf.load_triples(p)
    L = oracle.lib()
    import ctypes as C
    n = C.c_uint64()
    u, i, r = C.POINTER(C.c_uint32)(), C.POINTER(C.c_uint32)(), C.POINTER(C.c_double)()
    assert L.oracle_load_triples(str(p).encode(), C.byref(n), C.byref(u), C.byref(i), C.byref(r)) == 0
    assert d.num_cases == n.value == 90570
    assert np.array_equal(d.user, np.ctypeslib.as_array(u, (n.value,)))
    assert np.array_equal(d.item, np.ctypeslib.as_array(i, (n.value,)))
    assert np.array_equal(d.rating, np.ctypeslib.as_array(r, (n.value,)))


def test_triples_edge_cases(tmp_path):
    p = tmp_path / "edge.txt"
    p.write_text("0\t1\t5\n"          # plain
                 "2 3 4.5\n"          # space separated, half star
                 "\n"                 # empty: skipped
                 "# comment\n"        # not a rating: skipped
                 "4,5,1e0\n"          # any one-char separator
                 "6\t 7\t2\n"         # %u skips blanks after the separator
                 "8\t9\n"             # missing rating: skipped
                 "10\t11\t3 trailing\n"
                 "12\t13\t4")         # no final newline
    d = sbmf.load_triples(p)
    assert d.user.tolist() == [0, 2, 4, 6, 10, 12]
    assert d.item.tolist() == [1, 3, 5, 7, 11, 13]
    assert d.rating.tolist() == [5, 4.5, 1, 2, 3, 4]


def test_libfm_loader(tmp_path):
    p = tmp_path / "a.libfm"
    p.write_text("5 0:1 944:1\n  3 1:1 945:1 # c\n\n# x\n4.5 2:1 950:1\n")
    d = sbmf.load_libfm(p)
    assert d.user.tolist() == [0, 1, 2] and d.item.tolist() == [944, 945, 950]
    assert d.rating.tolist() == [5, 3, 4.5]
    d2 = sbmf.load_libfm(p, item_offset=944)
    assert d2.item.tolist() == [0, 1, 6]
    # with an item offset, a line whose first feature is in the item range is not a user
    q = tmp_path / "b.libfm"
    q.write_text("5 0:1 944:1\n4 1005:1 1007:1\n")
    with pytest.raises(sbmf.SBMFError):
        sbmf.load_libfm(q, item_offset=944)


@pytest.mark.parametrize("bad", ["5 0:1\n", "5 0:1 3:1 4:1\n", "x 0:1 1:1\n", "5 0-1 1:1\n"])
def test_libfm_loader_errors(tmp_path, bad):
    p = tmp_path / "bad.libfm"
    p.write_text(bad)
    with pytest.raises(sbmf.SBMFError):
        sbmf.load_libfm(p)


def test_missing_file():
    with pytest.raises(sbmf.SBMFError) as e:
        sbmf.load_triples("/nonexistent/file")
    assert "unable to open" in str(e.value)
