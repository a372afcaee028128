#!/usr/bin/env python3
"""make_golden.py -- TEST INFRASTRUCTURE ONLY: regenerate tests/golden/.

Runs the reference itself (oracle/_ref/, compiled unmodified from
/root/reference by `make -C oracle ref`) and stores its outputs as small
fixtures.  The reference samplers read their inputs from the hard-coded
relative paths ../../data/m100k/{train_sbpmf,test_sbpmf} (final,
gibbs_sbpmf_final.cpp:33,96), ../../data/m100k/{train,test} (sbpmf2,
gibbs_sbpmf2.cpp:33,96), ../../data/ra.{train,test}_sbpmf (the biased
sampler at the top level, gibbs_sbpmf2.cpp:32,98; D=20) and
../../data/m1m/{train,test}_sbpmf (src/libfm/gibbs_sbpmf22.cpp:33,74; D=100),
with 100 sweeps baked in.  We satisfy those paths with a scratch directory tree in /tmp
so any triple file can be fed in without touching the sources.

Fixtures written (all data, no reference source):
  ml100k_train.tsv.gz / ml100k_test.tsv.gz   inputs (copy of data/m100k/*_sbpmf)
  ragged_train.tsv / ragged_test.tsv          synthetic edge-case inputs
  ref_<variant>_<data>_k<K>_s<seed>.txt       100 lines "%.17g" test RMSE
                                              (variants final, sbpmf2, bias2, bias22)
  ref_rng_s<seed>.txt                         rand / ran_gaussian / ran_gamma
Only runnable in the build container (needs /root/reference).
"""
import gzip
import os
import shutil
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
REF = os.environ.get("SBMF_REFERENCE", "/root/reference")


def run_ref(binary, train_path, test_path, seed):
    """Run a reference sampler with its hard-coded relative input paths."""
    root = "/tmp/sbmf_refrun_%d" % os.getpid()
    cwd = os.path.join(root, "a", "b")
    os.makedirs(cwd, exist_ok=True)
    links = [("m100k/train_sbpmf", train_path), ("m100k/test_sbpmf", test_path), ("m100k/train", train_path),
             ("m100k/test", test_path), ("ra.train_sbpmf", train_path), ("ra.test_sbpmf", test_path),
             ("m1m/train_sbpmf", train_path), ("m1m/test_sbpmf", test_path)]
    for name, src in links:
        dst = os.path.join(root, "data", name)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        if os.path.lexists(dst):
            os.remove(dst)
        os.symlink(os.path.abspath(src), dst)
    env = dict(os.environ, SBMF_REF_SEED=str(seed))
    p = subprocess.run([binary], cwd=cwd, env=env, capture_output=True, text=True)
    shutil.rmtree(root)
    vals = [l.split()[-1] for l in p.stdout.splitlines() if l.startswith("rmse is")]
    # The top-level biased sampler dies in its exit cleanup when a user or item
    # id has no training ratings: the b_i / b_j step's `user_item_count[i]`
    # (gibbs_sbpmf2.cpp:520,568) inserts the id into the map, and the cleanup
    # (:651-667) then deletes an R[i] / R_t[j] that was never allocated.  Every
    # "rmse is" line is printed before that, so the trajectory is complete.
    if p.returncode != 0 and not (len(vals) == 100 and p.returncode == -11):
        raise RuntimeError("%s exited with %d" % (binary, p.returncode))
    return vals


def ragged_dataset(seed=3):
    """Small triples with id gaps (empty users/items), a user present only in
    test, heavy and single-rating rows, half-star ratings."""
    rng = np.random.default_rng(seed)
    n_users, n_items = 61, 47
    rows = []
    for u in range(n_users):
        if u % 7 == 3:
            continue  # empty user row
        deg = 1 if u % 11 == 0 else int(rng.integers(2, 30))
        if u == 5:
            deg = 40  # heavy row, all items
        items = rng.choice([i for i in range(n_items) if i % 9 != 4], size=min(deg, 41), replace=False)
        for i in items:
            rows.append((u, int(i), float(rng.integers(1, 11)) / 2.0))
    rng.shuffle(rows)
    n_test = len(rows) // 8
    test = rows[:n_test] + [(n_users + 2, 3, 4.0)]  # user id beyond train max
    train = rows[n_test:]
    return train, test


def write_tsv(path, rows):
    with open(path, "w") as f:
        for u, i, r in rows:
            f.write("%d\t%d\t%g\n" % (u, i, r))


def main():
    subprocess.run(["make", "-C", HERE, "all", "ref"], check=True, capture_output=True)
    os.makedirs(GOLD, exist_ok=True)
    ml_train = os.path.join(REF, "data", "m100k", "train_sbpmf")
    ml_test = os.path.join(REF, "data", "m100k", "test_sbpmf")
    for src, name in ((ml_train, "ml100k_train.tsv.gz"), (ml_test, "ml100k_test.tsv.gz")):
        with open(src, "rb") as f, gzip.GzipFile(os.path.join(GOLD, name), "wb", mtime=0) as g:
            g.write(f.read())
    rtrain, rtest = ragged_dataset()
    rtrain_p = os.path.join(GOLD, "ragged_train.tsv")
    rtest_p = os.path.join(GOLD, "ragged_test.tsv")
    write_tsv(rtrain_p, rtrain)
    write_tsv(rtest_p, rtest)

    runs = [("final", "ml100k", ml_train, ml_test, 1), ("final", "ml100k", ml_train, ml_test, 7),
            ("sbpmf2", "ml100k", ml_train, ml_test, 1), ("final", "ragged", rtrain_p, rtest_p, 1),
            ("sbpmf2", "ragged", rtrain_p, rtest_p, 5), ("bias2", "ml100k", ml_train, ml_test, 1),
            ("bias2", "ragged", rtrain_p, rtest_p, 3), ("bias22", "ml100k", ml_train, ml_test, 1)]
    binaries = {"final": ("gibbs_sbpmf_final", 20), "sbpmf2": ("gibbs_sbpmf2", 20),
                "bias2": ("gibbs_sbpmf2_bias", 20), "bias22": ("gibbs_sbpmf22", 100)}
    for variant, dname, tr, te, seed in runs:
        binary, K = binaries[variant]
        vals = run_ref(os.path.join(HERE, "_ref", binary), tr, te, seed)
        assert len(vals) == 100, (variant, dname, len(vals))
        with open(os.path.join(GOLD, "ref_%s_%s_k%d_s%d.txt" % (variant, dname, K, seed)), "w") as f:
            f.write("\n".join(vals) + "\n")
        print("golden", variant, dname, seed, vals[0], vals[-1])
    for seed in (1, 7):
        out = subprocess.run([os.path.join(HERE, "_ref", "ref_rng_dump"), str(seed), "2000"],
                             capture_output=True, text=True, check=True).stdout
        with open(os.path.join(GOLD, "ref_rng_s%d.txt" % seed), "w") as f:
            f.write(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
