"""The `sbmf` command line end to end on the GPU: the libFM outputs a user of
`bin/libFM -task r -method mcmc` reads (fm_learn_mcmc_simultaneous.h:57-62,
146, 244; libfm.cpp:629-634), checked against the compiled reference's
golden trajectory and the oracle.

Tolerances: the libFM-format files carry the reference's default 6
significant digits, so they are compared within half a unit of the sixth
digit plus the 1e-6 parity bar (_close6); the full-precision -rlog is
compared within 1e-6."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from conftest import REPO, golden_rmse, write_m1m100k_libfm
from sbmf._lib import CLI_PATH

pytestmark = pytest.mark.gpu

ITER_RE = re.compile(r"^#Iter=([ \d]{3,})\tTrain=([-+0-9.eEnai]+)\tTest=([-+0-9.eEnai]+)$")


def _close6(printed, exact):
    """`printed` is `exact` written with 6 significant digits (std::ostream default)."""
    printed, exact = np.asarray(printed, float), np.asarray(exact, float)
    return bool(np.all(np.abs(printed - exact) <= 5e-6 * np.maximum(np.abs(exact), 1e-300) + 1e-6))


def _write(path, data):
    u, i, r = data
    with open(path, "w") as f:
        for a, b, c in zip(u, i, r):
            f.write("%d\t%d\t%g\n" % (a, b, c))


def _cli(tmp_path, ml100k, *args):
    tr, te = tmp_path / "train.tsv", tmp_path / "test.tsv"
    _write(tr, ml100k[0])
    _write(te, ml100k[1])
    cmd = [CLI_PATH, "-task", "r", "-train", str(tr), "-test", str(te), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    return r


def _rlog(path, col="sbmf_rmse_all"):
    lines = open(path).read().splitlines()
    head = lines[0].split("\t")
    return np.array([float(l.split("\t")[head.index(col)]) for l in lines[1:]])


def _libfm_rlog_header(K, groups=1, but5=True):
    """libFM's RLog field order for regression MCMC: fm_learn::init (fm_learn.h:82-127),
    then fm_learn_mcmc::init (fm_learn_mcmc.h:1121-1148)."""
    h = ["rmse", "mae", "time_pred", "time_learn", "time_learn2", "time_learn4", "alpha", "rmse_mcmc_this",
         "rmse_mcmc_all"] + (["rmse_mcmc_all_but5"] if but5 else [])
    for g in range(groups):
        h += ["wmu[%d]" % g, "wlambda[%d]" % g]
        for f in range(K):
            h += ["vmu[%d,%d]" % (g, f), "vlambda[%d,%d]" % (g, f)]
    return h


def test_cli_mcmc_k20_matches_reference_golden(tmp_path, ml100k):
    """bin/libFM-style run: stdout #Iter lines, test_rmse_0020_mcmc (truncated,
    one running-mean RMSE per line), -out predictions, -rlog."""
    r = _cli(tmp_path, ml100k, "-dim", "0,0,20", "-iter", "100", "-seed", "1", "-method", "mcmc",
             "-out", str(tmp_path / "pred.txt"), "-rlog", str(tmp_path / "rlog.tsv"))
    gold = golden_rmse("ref_final_ml100k_k20_s1.txt")
    lines = [l for l in r.stdout.splitlines() if l.startswith("#Iter")]
    assert len(lines) == 100
    for k, l in enumerate(lines):
        m = ITER_RE.match(l)
        assert m, repr(l)
        assert int(m.group(1)) == k and len(m.group(1)) == 3  # std::setw(3)
        assert _close6(float(m.group(3)), gold[k])
    f = tmp_path / "test_rmse_0020_mcmc"
    vals = np.array([float(x) for x in f.read_text().split()])
    assert vals.shape == gold.shape
    assert _close6(vals, gold)
    assert np.abs(_rlog(tmp_path / "rlog.tsv") - gold).max() < 1e-6
    # libFM's -rlog columns first (the SBPMF sampler's two hyperprior groups), ours after them:
    # the header bin/libFM itself writes for two -meta groups at K=20 (oracle/make_golden.py rlog)
    head = (tmp_path / "rlog.tsv").read_text().splitlines()[0].split("\t")
    with open(os.path.join(REPO, "tests", "golden", "ref_libfm_rlog_header_k20_g2.txt")) as f:
        libfm_head = f.read().rstrip("\n").split("\t")
    assert libfm_head == _libfm_rlog_header(20, groups=2)
    assert head[:len(libfm_head)] == libfm_head
    assert _close6(_rlog(tmp_path / "rlog.tsv", "rmse"), gold)
    assert _close6(_rlog(tmp_path / "rlog.tsv", "rmse_mcmc_all"), gold)
    tau = _rlog(tmp_path / "rlog.tsv", "sbmf_tau")
    assert _close6(_rlog(tmp_path / "rlog.tsv", "alpha"), tau)
    o = oracle.run(*ml100k, K=20, iters=100, seed=1, want_factors=False)
    pred = np.array([float(x) for x in (tmp_path / "pred.txt").read_text().split()])
    assert pred.shape == (len(ml100k[1][0]),)
    assert _close6(pred, o["pred_sum"] / 100)
    # mae of the running mean after the last sweep, from the same predictions
    mae = _rlog(tmp_path / "rlog.tsv", "mae")
    assert _close6(mae[-1], np.mean(np.abs(pred - ml100k[1][2])))


def test_cli_truncates_rmse_file_and_runs_config1_k8(tmp_path, ml100k):
    """BASELINE config 1 (ML-100k, K=8) through the CLI; a stale
    test_rmse_008_mcmc is truncated at start (fm_learn_mcmc_simultaneous.h:61)."""
    (tmp_path / "test_rmse_008_mcmc").write_text("stale\n" * 500)
    _cli(tmp_path, ml100k, "-dim", "0,0,8", "-iter", "30", "-seed", "7", "-rlog", str(tmp_path / "rlog.tsv"))
    o = oracle.run(*ml100k, K=8, iters=30, seed=7, want_factors=False)
    vals = (tmp_path / "test_rmse_008_mcmc").read_text().split()
    assert len(vals) == 30
    assert _close6([float(x) for x in vals], o["rmse"])
    assert np.abs(_rlog(tmp_path / "rlog.tsv") - o["rmse"]).max() < 1e-6


def test_cli_philox_bench_mode_matches_oracle(tmp_path, ml100k):
    """The benchmark's throughput configuration through the CLI: Philox stream,
    residuals carried across sweeps (-recompute_every 0)."""
    _cli(tmp_path, ml100k, "-dim", "0,0,32", "-iter", "20", "-seed", "2015", "--rng", "philox",
         "--recompute_every", "0", "-rlog", str(tmp_path / "rlog.tsv"))
    o = oracle.run(*ml100k, K=32, iters=20, seed=2015, rng="philox", want_factors=False)
    assert np.abs(_rlog(tmp_path / "rlog.tsv") - o["rmse"]).max() < 1e-6


def _write_libfm(path, data, item_offset):
    """users-first libFM text "r u:1 (item_offset + i):1" (Data.h:192-217)."""
    u, i, r = data
    with open(path, "w") as f:
        for a, b, c in zip(u, i, r):
            f.write("%g %d:1 %d:1\n" % (c, a, item_offset + b))


@pytest.mark.parametrize("method,offset_flag", [("mcmc", False), ("als", False), ("mcmc", True)])
def test_cli_libfm_methods_reproduce_libfm_output(tmp_path, ml100k, method, offset_flag):
    """`sbmf` as a drop-in for `bin/libFM -method mcmc|als` on the same libFM
    text files: the "#Iter=" lines equal libFM's own (tests/golden/ref_libfm_*,
    libfm.cpp compiled unmodified, time() pinned to the seed), the -out file
    and test_rmse_118_mcmc within the printed digits.  The users-first split is
    libFM's own num_user rule (libfm.cpp:375); -item_offset, when given, overrides it."""
    I = int(max(ml100k[0][0].max(), ml100k[1][0].max())) + 1
    tr, te = tmp_path / "train.libfm", tmp_path / "test.libfm"
    _write_libfm(tr, ml100k[0], I)
    _write_libfm(te, ml100k[1], I)
    extra = ["-order", "libfm"] if method == "mcmc" else ["-regular", "0,0,10"]
    if offset_flag:
        extra += ["-item_offset", str(I)]
    cmd = [CLI_PATH, "-task", "r", "-train", str(tr), "-test", str(te), "-dim", "1,1,8", "-iter", "10",
           "-method", method, "-seed", "1", "-out", str(tmp_path / "pred.txt"), *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    name = "ref_libfm_%s_ml100k_d118_s1_i10" % method
    gold_lines = open(os.path.join(os.path.dirname(__file__), "golden", name + ".txt")).read().splitlines()
    lines = [l for l in r.stdout.splitlines() if l.startswith("#Iter")]
    assert lines == gold_lines
    import gzip
    with gzip.open(os.path.join(os.path.dirname(__file__), "golden", name + "_pred.txt.gz"), "rt") as f:
        ref_pred = np.array([float(x) for x in f.read().split()])
    pred = np.loadtxt(tmp_path / "pred.txt")
    assert np.abs(pred - ref_pred).max() <= 1.1e-5
    rm = np.loadtxt(tmp_path / "test_rmse_118_mcmc")
    assert len(rm) == 10 and abs(rm[-1] - float(gold_lines[-1].split("Test=")[1])) < 1e-5


def test_cli_mcmc_on_libfm_input_is_libfms_chain(tmp_path, ml100k):
    """`bin/libFM -method mcmc -dim 1,1,8` on libFM text runs fm_learn_mcmc (libfm.cpp:411-419):
    without -order, sbmf does the same (no note on stdout), and -rlog carries libFM's
    one-group field set with rmse_mcmc_all_but5 per fm_learn_mcmc_simultaneous.h:158-161,241."""
    I = int(max(ml100k[0][0].max(), ml100k[1][0].max())) + 1
    tr, te = tmp_path / "train.libfm", tmp_path / "test.libfm"
    _write_libfm(tr, ml100k[0], I)
    _write_libfm(te, ml100k[1], I)
    cmd = [CLI_PATH, "-task", "r", "-train", str(tr), "-test", str(te), "-dim", "1,1,8", "-iter", "10",
           "-method", "mcmc", "-seed", "1", "-rlog", str(tmp_path / "rlog.tsv")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "note" not in r.stdout
    name = "ref_libfm_mcmc_ml100k_d118_s1_i10"
    gold_lines = open(os.path.join(os.path.dirname(__file__), "golden", name + ".txt")).read().splitlines()
    assert [l for l in r.stdout.splitlines() if l.startswith("#Iter")] == gold_lines
    head = (tmp_path / "rlog.tsv").read_text().splitlines()[0].split("\t")
    assert head[:len(_libfm_rlog_header(8))] == _libfm_rlog_header(8)
    b5 = _rlog(tmp_path / "rlog.tsv", "rmse_mcmc_all_but5")
    allr = _rlog(tmp_path / "rlog.tsv", "rmse_mcmc_all")
    assert np.all(np.isfinite(b5)) and b5[5] == pytest.approx(_rlog(tmp_path / "rlog.tsv", "rmse_mcmc_this")[5], abs=1e-5)
    assert abs(allr[-1] - float(gold_lines[-1].split("Test=")[1])) < 1e-5
    # the explicit SBPMF order on the same file keeps its note off stdout
    r2 = subprocess.run(cmd[:-2] + ["-order", "sbpmf"], capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r2.returncode == 0, r2.stderr
    assert "note" in r2.stderr and "note" not in r2.stdout


@pytest.mark.parametrize("method", ["mcmc", "als"])
def test_cli_is_bin_libfm_on_the_reference_files(tmp_path, method):
    """bin/libFM's exact command line on the reference's own data/m1m/m100k/{train,test}_libfm
    (users 0..942, items at raw feature ids 943..2624), nothing added:
        -task r -train train_libfm -test test_libfm -dim '1,1,8' -iter 10 -method mcmc
        (-method als -regular '0,0,10')
    libFM's attributes are the file's feature ids (num_user = max first feature + 1,
    libfm.cpp:375; num_all_attribute = max feature + 1, :328), so the chain is libFM's:
    "#Iter" lines equal as text to the compiled libfm.cpp's (time() pinned to 1 = sbmf's
    default -seed), -out within libFM's printed digits, test_rmse_118_mcmc equal."""
    write_m1m100k_libfm(tmp_path)
    cmd = [CLI_PATH, "-task", "r", "-train", "train_libfm", "-test", "test_libfm", "-dim", "1,1,8", "-iter", "10",
           "-method", method, "-out", "pred.txt"] + (["-regular", "0,0,10"] if method == "als" else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "#users=943\t#items=1682" in r.stdout  # libFM's 2625 attributes: 943 users + 1682 items
    name = "ref_libfm_%s_m1m100k_d118_s1_i10" % method
    gold_lines = open(os.path.join(REPO, "tests", "golden", name + ".txt")).read().splitlines()
    lines = [l for l in r.stdout.splitlines() if l.startswith("#Iter")]
    assert lines == gold_lines
    import gzip
    with gzip.open(os.path.join(REPO, "tests", "golden", name + "_pred.txt.gz"), "rt") as f:
        ref_pred = np.array([float(x) for x in f.read().split()])
    pred = np.loadtxt(tmp_path / "pred.txt")
    ulp6 = 10.0 ** (np.floor(np.log10(np.abs(ref_pred))) - 5)
    assert np.all(np.abs(pred - ref_pred) <= 0.5 * ulp6 * (1 + 1e-9) + 1e-12)
    rm = (tmp_path / "test_rmse_118_mcmc").read_text().split()
    assert rm == [l.split("Test=")[1] for l in gold_lines]


@pytest.mark.parametrize("method", ["mcmc", "als"])
def test_cli_reads_the_transpose_as_bin_libfm_does(tmp_path, method):
    """A reference user who ran tools/convert then tools/transpose and points -train / -test at
    the stem: bin/libFM -method mcmc|als builds its sets with has_x = false (libfm.cpp:132-149),
    so Data::load opens <stem>.xt + <stem>.y (Data.h:113-117,143-151).  The directory holds
    only those files (the reference tools' own output on data/m1m/m100k, compiled from source:
    `make_golden.py bindata`); the argv is bin/libFM's, nothing added.  The "#Iter" lines equal
    as text the compiled libfm.cpp's on the same files (time() pinned to 1), -out within
    libFM's printed digits, test_rmse_118_mcmc equal."""
    import gzip
    for nm in ("train_libfm", "test_libfm"):
        for ext in ("xt", "y"):
            with gzip.open(os.path.join(REPO, "tests", "golden", "m1m100k_%s.%s.gz" % (nm, ext)), "rb") as f:
                (tmp_path / ("%s.%s" % (nm, ext))).write_bytes(f.read())
    assert sorted(p.name for p in tmp_path.iterdir()) == ["test_libfm.xt", "test_libfm.y", "train_libfm.xt",
                                                          "train_libfm.y"]
    cmd = [CLI_PATH, "-task", "r", "-train", "train_libfm", "-test", "test_libfm", "-dim", "1,1,8", "-iter", "10",
           "-method", method, "-out", "pred.txt"] + (["-regular", "0,0,10"] if method == "als" else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "#users=943\t#items=1682" in r.stdout
    name = "ref_libfm_%s_m1m100k_xt_d118_s1_i10" % method
    gold_lines = open(os.path.join(REPO, "tests", "golden", name + ".txt")).read().splitlines()
    assert [l for l in r.stdout.splitlines() if l.startswith("#Iter")] == gold_lines
    with gzip.open(os.path.join(REPO, "tests", "golden", name + "_pred.txt.gz"), "rt") as f:
        ref_pred = np.array([float(x) for x in f.read().split()])
    pred = np.loadtxt(tmp_path / "pred.txt")
    ulp6 = 10.0 ** (np.floor(np.log10(np.abs(ref_pred))) - 5)
    assert np.all(np.abs(pred - ref_pred) <= 0.5 * ulp6 * (1 + 1e-9) + 1e-12)
    assert (tmp_path / "test_rmse_118_mcmc").read_text().split() == [l.split("Test=")[1] for l in gold_lines]


def test_cli_sbpmf_order_on_the_reference_libfm_file(tmp_path):
    """`-order sbpmf` on the same libFM file is gibbs_sbpmf_final on the reference's converted
    data/m1m/m100k/{train,test}_sbpmf (create_file_scalable_bpmf.py keeps the raw item ids,
    so items 0..942 are empty rows): K=20 (gibbs_sbpmf_final.cpp's baked D), 100 sweeps,
    seed 1, the running-mean test RMSE of every sweep within the 6 printed digits."""
    write_m1m100k_libfm(tmp_path)
    cmd = [CLI_PATH, "-task", "r", "-train", "train_libfm", "-test", "test_libfm", "-dim", "1,1,20", "-iter", "100",
           "-method", "mcmc", "-order", "sbpmf"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert "#users=943\t#items=2625" in r.stdout
    gold = golden_rmse("ref_final_m1m100k_k20_s1.txt")
    lines = [l for l in r.stdout.splitlines() if l.startswith("#Iter")]
    assert len(lines) == 100
    assert _close6([float(ITER_RE.match(l).group(3)) for l in lines], gold)
    assert _close6([float(x) for x in (tmp_path / "test_rmse_1120_mcmc").read_text().split()], gold)


def test_cli_vb_on_libfm_text_follows_reference_learner(tmp_path, ml100k):
    """`-method vb` on users-first libFM text with libFM's own argv (no offset flag): the
    online VB learner over the file's attributes, per-epoch "Test=" within the printed
    digits of the reference learner's trajectory (tests/golden/ref_vbo_ml100k_k8_s1_e10.txt,
    fm_learn_vb_online*.h compiled unmodified, oracle/ref_vbo_harness.cpp)."""
    I = int(max(ml100k[0][0].max(), ml100k[1][0].max())) + 1
    tr, te = tmp_path / "train.libfm", tmp_path / "test.libfm"
    _write_libfm(tr, ml100k[0], I)
    _write_libfm(te, ml100k[1], I)
    cmd = [CLI_PATH, "-task", "r", "-train", str(tr), "-test", str(te), "-dim", "1,1,8", "-iter", "10",
           "-method", "vb", "-seed", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    gold = golden_rmse("ref_vbo_ml100k_k8_s1_e10.txt")
    vals = [float(l.split("Test=")[1]) for l in r.stdout.splitlines() if l.startswith("#Iter")]
    assert len(vals) == 10 and _close6(vals, gold)
