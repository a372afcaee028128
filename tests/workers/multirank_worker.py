"""One rank of the multi-rank sampler (spawned by tests/test_gpu_multirank.py).

usage: python multirank_worker.py <rank> <nranks> <id-hex> <out.npz> <K> <sweeps> <seed> <rng> [tune] [quirks] [method]
The ranks share one GPU and exchange their row blocks through the host comm
backend (the id was made with SBMF_COMM=host); the result must equal a
single-rank run in the same residual form.  method "vb": the online VB
learner (user ranges per rank, item sums all-gathered), `sweeps` epochs.
"""
import gzip
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "scalable-bayesian-matrix-factorization_amd"))


def read(path):
    u, i, r = [], [], []
    if not os.path.exists(path):
        path = path[:-3]  # the ragged set is plain text
    with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as f:
        for line in f:
            p = line.split()
            if len(p) >= 3:
                u.append(int(p[0]))
                i.append(int(p[1]))
                r.append(float(p[2]))
    return np.array(u, np.uint32), np.array(i, np.uint32), np.array(r)


def main():
    rank, nranks, idhex, out, K, sweeps, seed, rng = sys.argv[1:9]
    tune = int(sys.argv[9]) if len(sys.argv) > 9 else 0
    quirks = sys.argv[10] if len(sys.argv) > 10 else "final"
    method = sys.argv[11] if len(sys.argv) > 11 else "mcmc"
    from sbmf import Data, FMLearnSBPMF, FMLearnVBOnline
    g = os.path.join(REPO, "tests", "golden")
    data = os.environ.get("SBMF_WORKER_DATA", "ml100k")
    dims = (0, 0)
    if data.startswith("synth:"):  # a full-size synthetic shape (sbmf/synth.py), identical in every rank
        from sbmf import synth
        tr, te, dims = synth.generate(data[6:])
        if os.environ.get("SBMF_WORKER_RELABEL") == "degree":
            tr, te, dims = synth.relabel_by_degree(tr, te, dims)
    else:
        tr, te = read(os.path.join(g, data + "_train.tsv.gz")), read(os.path.join(g, data + "_test.tsv.gz"))
    if method == "vb":
        L = FMLearnVBOnline(num_factor=int(K), seed=int(seed), rng=rng, device=0)
    elif method in ("libfm", "als"):  # libFM's own chain: quirks carries "k0,k1;regular"
        dim, reg = quirks.split(";")
        k0, k1 = (int(x) for x in dim.split(","))
        L = FMLearnSBPMF(num_factor=int(K), seed=int(seed), rng=rng, device=0, order="libfm",
                         method="als" if method == "als" else "mcmc", k0=k0, k1=k1,
                         regular=tuple(float(x) for x in reg.split(",")), init_stdev=0.1)
    else:
        L = FMLearnSBPMF(num_factor=int(K), seed=int(seed), rng=rng, device=0, tune=tune, quirks=quirks,
                         pipeline=int(os.environ.get("SBMF_WORKER_PIPELINE", "0")))
    L.init(comm=(int(nranks), int(rank), bytes.fromhex(idhex)))
    L.set_data(Data(*tr), Data(*te), num_users=dims[0], num_items=dims[1])
    L.learn(sweeps=int(sweeps))
    U, V = L.factors()
    if os.environ.get("SBMF_WORKER_DIGEST"):  # full-size tables: digests instead of the arrays
        import hashlib
        U = np.frombuffer(hashlib.sha256(np.ascontiguousarray(U).tobytes()).digest(), np.uint8)
        V = np.frombuffer(hashlib.sha256(np.ascontiguousarray(V).tobytes()).digest(), np.uint8)
    extra = {}
    if quirks in ("bias2", "bias22") or method in ("vb", "libfm", "als"):
        bu, bv, b0 = L.biases()
        extra = {"bu": bu, "bv": bv, "b0": np.array([b0])}
    if method in ("vb", "libfm", "als"):
        extra["pred"] = L.predict()
        extra["rmse_train"] = np.array([h["rmse_train"] for h in L.history])
    np.savez(out, U=U, V=V, rmse=L.rmse_trajectory, tau=np.array([h["tau"] for h in L.history]), **extra)
    L.close()


if __name__ == "__main__":
    main()
