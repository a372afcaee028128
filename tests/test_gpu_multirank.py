"""Several ranks on one GPU (host comm backend instead of RCCL, which refuses
two ranks on one device): the row-block partition, the per-half block
exchange, the point-to-point residual exchange and the fixed-order partial
sums must reproduce a single-rank run bit for bit.  tune=2 runs every rank
(and the single-rank reference) with residuals recomputed from r - own.partner
instead of exchanged.  The biased sampler (quirks bias2) also exchanges the
fresh user / item bias blocks and sums the sweep-start residuals per row."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
from sbmf import Data, FMLearnSBPMF, comm_unique_id

pytestmark = pytest.mark.gpu
WORKER = os.path.join(REPO, "tests", "workers", "multirank_worker.py")


@pytest.mark.parametrize("nranks,rng,tune,quirks", [(2, "ref", 0, "final"), (3, "philox", 0, "final"),
                                                   (2, "philox", 2, "final"), (2, "ref", 0, "bias2"),
                                                   (3, "philox", 0, "bias22")])
def test_ranks_on_one_gpu_match_single_rank(ml100k, tmp_path, nranks, rng, tune, quirks):
    K, sweeps, seed = 30, 3, 6
    tr, te = ml100k
    # single rank, same residual form as every rank of the multi-rank run
    L = FMLearnSBPMF(num_factor=K, seed=seed, rng=rng, tune=tune, quirks=quirks)
    L.set_data(Data(*tr), Data(*te))
    L.learn(sweeps=sweeps)
    U1, V1 = L.factors()
    rmse1 = L.rmse_trajectory
    biased = quirks in ("bias2", "bias22")
    if biased:
        bu1, bv1, b01 = L.biases()
    L.close()

    old = os.environ.get("SBMF_COMM")
    os.environ["SBMF_COMM"] = "host"
    try:
        uid = comm_unique_id()
    finally:
        if old is None:
            del os.environ["SBMF_COMM"]
        else:
            os.environ["SBMF_COMM"] = old
    outs = [str(tmp_path / ("r%d.npz" % r)) for r in range(nranks)]
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), str(nranks), uid.hex(), outs[r], str(K), str(sweeps),
                               str(seed), rng, str(tune), quirks], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(nranks)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-2000:]
    for r in range(nranks):
        z = np.load(outs[r])
        # every rank ends with the full, identical factor tables
        assert np.array_equal(z["U"], U1) and np.array_equal(z["V"], V1), \
            (r, np.abs(z["U"] - U1).max(), np.abs(z["V"] - V1).max())
        assert np.array_equal(z["rmse"], rmse1)
        if biased:
            assert np.array_equal(z["bu"], bu1) and np.array_equal(z["bv"], bv1) and z["b0"][0] == b01
