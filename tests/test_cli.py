"""`sbmf` command line: libFM flag grammar (src/util/cmdline.h:33-70,113-119)
and the errors a libFM user gets, checked without a GPU."""
import subprocess

import pytest

from conftest import gpu_available
from sbmf._lib import CLI_PATH


def run(*args):
    return subprocess.run([CLI_PATH, *args], capture_output=True, text=True, timeout=60)


def test_help_lists_libfm_flags():
    r = run("-help")
    assert r.returncode == 0
    for flag in ("-task", "-train", "-test", "-dim", "-iter", "-method", "-init_stdev", "-seed", "-out", "-rlog"):
        assert flag in r.stdout


def test_no_arguments_prints_help():
    r = run()
    assert r.returncode == 0 and "-train" in r.stdout


@pytest.mark.parametrize("args,msg", [
    (["-task", "r", "-task", "r"], "already specified"),
    (["-task", "r", "-bogus", "1"], "does not exist"),
    (["task", "r"], "cannot parse"),
    (["-task", "c", "-train", "a", "-test", "b"], "only -task r"),
    (["-task", "r", "-train", "a", "-test", "b", "-method", "sgd"], "not supported"),
    (["-task", "r", "-train", "a", "-test", "b", "-method", "vb", "-dim", "0,0,8"], "-dim '1,1,K'"),
    (["-task", "r", "-train", "a"], "mandatory"),
    (["-task", "r", "-train", "a", "-test", "b", "-dim", "1,1"], "dim must have 3"),
    (["-task", "r", "-train", "/nonexistent", "-test", "b"], "unable to open"),
    (["-task", "r", "-train", "a", "-test", "b", "-quirks", "bias2", "-dim", "0,0,8"], "-dim '1,1,K'"),
    (["-task", "r", "-train", "a", "-test", "b", "-quirks", "bogus"], "unknown -quirks"),
])
def test_grammar_errors(args, msg):
    r = run(*args)
    assert r.returncode == 1
    assert "ERROR:" in r.stderr and msg in r.stderr


def test_double_dash_form_accepted(tmp_path):
    r = run("--task", "r", "--train", "/nonexistent", "--test", "x")
    assert "unable to open" in r.stderr


@pytest.mark.skipif(gpu_available(), reason="no-GPU path")
def test_valid_command_fails_loudly_without_gpu(tmp_path):
    tr = tmp_path / "t.tsv"
    tr.write_text("0\t0\t5\n1\t1\t3\n")
    r = run("-task", "r", "-train", str(tr), "-test", str(tr), "-dim", "1,1,8", "-iter", "2")
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.skipif(gpu_available(), reason="no-GPU path")
def test_binary_stem_loaded_before_device(tmp_path):
    """-train <stem> with <stem>.x/.y present takes the binary branch (Data.h:113-117);
    a loader error would surface before the device check."""
    import sbmf
    stem = str(tmp_path / "bin")
    sbmf.save_libfm_binary(stem, sbmf.Data([0, 1], [0, 1], [5.0, 3.0]), item_offset=2)
    r = run("-task", "r", "-train", stem, "-test", stem, "-dim", "1,1,8", "-iter", "2", "--item_offset", "2")
    assert r.returncode == 1 and "no HIP device" in r.stderr
    r = run("-task", "r", "-train", stem, "-test", stem, "-dim", "1,1,8", "-iter", "2", "--format", "binary",
            "--item_offset", "3")
    assert r.returncode == 1 and "one user and one item" in r.stderr


def test_libfm_input_must_be_users_first(tmp_path):
    """libFM's learners read the file's feature ids as attributes with the users first
    (num_user = max first feature + 1, libfm.cpp:375): an item feature id at or below a
    user id has no such reading and is refused before any device work (no GPU needed)."""
    tr = tmp_path / "t.libfm"
    tr.write_text("5 0:1 3:1\n3 4:1 6:1\n")  # item 3 <= user 4
    r = run("-task", "r", "-train", str(tr), "-test", str(tr), "-dim", "1,1,8", "-iter", "2", "-method", "mcmc")
    assert r.returncode == 1 and "users first" in r.stderr and "item feature id 3" in r.stderr
    # the SBPMF order reads the same file as raw (user, item) triples, as the reference's converter does
    r = run("-task", "r", "-train", str(tr), "-test", str(tr), "-dim", "0,0,8", "-iter", "2", "-order", "sbpmf")
    assert "users first" not in r.stderr
