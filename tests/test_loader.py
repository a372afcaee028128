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


def test_libfm_users_first_split_is_libfms_num_user(m1m100k, tmp_path):
    """libFM's num_user = max first feature id + 1 over train and test (libfm.cpp:375): on the
    reference's data/m1m/m100k/*_libfm that is 943 and the items rebase to 0..1681."""
    from conftest import write_m1m100k_libfm
    trp, tep = write_m1m100k_libfm(tmp_path)
    tr, te = sbmf.load_libfm(trp), sbmf.load_libfm(tep)
    assert np.array_equal(tr.item, m1m100k[0][1])
    tr2, te2, I = sbmf.libfm_users_first(tr, te)
    assert I == 943 and int(tr2.item.min()) == 0 and max(tr2.item.max(), te2.item.max()) == 2624 - 943
    assert np.array_equal(tr2.item, tr.item - 943) and np.array_equal(te2.user, te.user)
    with pytest.raises(ValueError):
        sbmf.libfm_users_first(sbmf.Data([0, 4], [944, 3], [5.0, 3.0]))


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


def _oracle_triples(path):
    import ctypes as C
    L = oracle.lib()
    n = C.c_uint64()
    u, i, r = C.POINTER(C.c_uint32)(), C.POINTER(C.c_uint32)(), C.POINTER(C.c_double)()
    assert L.oracle_load_triples(str(path).encode(), C.byref(n), C.byref(u), C.byref(i), C.byref(r)) == 0
    m = n.value
    return (np.ctypeslib.as_array(u, (m,)).copy(), np.ctypeslib.as_array(i, (m,)).copy(),
            np.ctypeslib.as_array(r, (m,)).copy())


@pytest.fixture
def chunked(monkeypatch):
    """Small line-aligned chunks on several threads (the ML-20M path's shape, at test size)."""
    def set_(threads, chunk):
        monkeypatch.setenv("SBMF_LOAD_THREADS", str(threads))
        monkeypatch.setenv("SBMF_LOAD_CHUNK", str(chunk))
    return set_


def test_triples_chunked_parse_matches_sscanf(tmp_path, chunked):
    """The threaded loader (line-aligned chunks, per-chunk arrays joined in file
    order, m / 10^k fast path for short decimals) against the oracle's plain
    sscanf("%u%c%u%c%lf") loop (gibbs_sbpmf_final.cpp:43), bit for bit, on lines
    that take every path: integers, half stars, long and exponent decimals, hex,
    signs, blanks, CRLF, garbage and a final line without newline."""
    rng = np.random.default_rng(3)
    forms = ["{u}\t{i}\t{r}\n", "{u} {i} {r}\n", "{u},{i},{r}\r\n", "{u}\t{i}\t{r} trailing\n", "{u}\t{i}\n",
             "# note\n", "\n", "{u}\t {i}\t{r}\n"]
    vals = ["4", "3.5", "0.1", "2.675", "1e0", "4.", ".5", "-3", "+2", "0x1A", "3.14159265358979323846",
            "1.7976931348623157e308", "5e-324", "0.30000000000000004", "nan", "007", "12345678901234567890",
            "9007199254740993", "0.1234567890123456789012345"]
    lines = []
    for _ in range(30000):
        f = forms[rng.integers(len(forms))]
        lines.append(f.format(u=int(rng.integers(0, 2 ** 32)), i=int(rng.integers(0, 30000)),
                              r=vals[rng.integers(len(vals))]))
    p = tmp_path / "mixed.txt"
    p.write_text("".join(lines) + "7\t8\t2.5")
    ou, oi, orr = _oracle_triples(p)
    for threads, chunk in ((1, 1 << 30), (7, 1000), (16, 1)):
        chunked(threads, chunk)
        d = sbmf.load_triples(p)
        assert np.array_equal(d.user, ou) and np.array_equal(d.item, oi)
        assert np.array_equal(d.rating.view(np.uint64), orr.view(np.uint64)), threads


def test_save_triples_round_trip(tmp_path, chunked):
    rng = np.random.default_rng(5)
    n = 50000
    u = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    i = rng.integers(0, 70000, n).astype(np.uint32)
    r = np.where(rng.random(n) < 0.5, rng.integers(1, 6, n).astype(np.float64), rng.normal(3, 2, n))
    r[:4] = [0.5, -0.0, 1e300, 4.9e-324]
    p = tmp_path / "out.tsv"
    sbmf.save_triples(p, sbmf.Data(u, i, r))
    chunked(5, 4096)
    d = sbmf.load_triples(p)
    assert np.array_equal(d.user, u) and np.array_equal(d.item, i)
    assert np.array_equal(d.rating.view(np.uint64), r.view(np.uint64))


def test_libfm_chunked_error_line(tmp_path, chunked):
    """A bad line far into a multi-chunk file is reported with its file line number."""
    good = "".join("%d %d:1 %d:1\n" % (1 + k % 5, k % 900, 1000 + k % 700) for k in range(5000))
    p = tmp_path / "big.libfm"
    p.write_text(good + "4 17:1\n" + good)
    chunked(8, 512)
    with pytest.raises(sbmf.SBMFError) as e:
        sbmf.load_libfm(p)
    assert "line 5001 of" in str(e.value)
    q = tmp_path / "ok.libfm"
    q.write_text(good * 3)
    d = sbmf.load_libfm(q)
    chunked(1, 1 << 30)
    d1 = sbmf.load_libfm(q)
    assert d.num_cases == 15000 and np.array_equal(d.item, d1.item) and np.array_equal(d.rating, d1.rating)
