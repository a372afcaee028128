"""N>1 layout and exchange protocol, on CPU with gloo (world_size 2).

On the GPU the ranks exchange freshly sampled row blocks with one grouped
set of in-place ncclBroadcast calls (comm.cpp: rank k is root of rows
[bounds[k], bounds[k+1])).  Here two gloo processes run the same protocol
with torch.distributed.broadcast over numpy-backed tables, using the
library's own partition (sbmf_partition_rows), and check that every rank
ends with the identical full table and that the partition tiles the rows,
balances ratings and keeps 256-row alignment."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from conftest import PKG  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, PKG)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from sbmf import partition_rows, synth
        train, _, dims = synth.generate("ml-100k", seed=3)
        ptr = np.concatenate([[0], np.cumsum(np.bincount(train[0], minlength=dims[0]))]).astype(np.uint32)
        bounds = partition_rows(ptr, world)
        allb = [None] * world
        dist.all_gather_object(allb, bounds.tolist())
        assert all(b == allb[0] for b in allb)
        K = 24
        full = np.random.default_rng(0).normal(size=(dims[0], K))
        mine = np.zeros_like(full)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        mine[r0:r1] = full[r0:r1] * 1.0  # this rank's freshly sampled block
        t = torch.from_numpy(mine)
        for k in range(world):  # == Comm::bcast_ranges(base, K*8, bounds)
            a, b = int(bounds[k]), int(bounds[k + 1])
            if b > a:
                view = t[a:b].contiguous()
                dist.broadcast(view, src=k)
                t[a:b] = view
        ok = np.array_equal(t.numpy(), full)
        q.put((rank, ok, bounds.tolist(), [int(ptr[int(bounds[k + 1])] - ptr[int(bounds[k])]) for k in range(world)]))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e), None))


@pytest.mark.parametrize("world", [2])
def test_two_rank_block_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok, bounds, nnz in res:
        assert ok, (rank, bounds)
        assert bounds[0] == 0 and all(b % 256 == 0 for b in bounds[1:-1])
        assert all(x > 0 for x in nnz)
        assert max(nnz) / min(nnz) < 1.5  # ratings balanced across ranks


def test_partition_properties_many_ranks():
    from sbmf import partition_rows
    rng = np.random.default_rng(1)
    deg = rng.pareto(1.1, 50_000).astype(np.int64) + 1
    ptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint32)
    for n in (1, 2, 3, 4, 8):
        b = partition_rows(ptr, n).astype(np.int64)
        assert b[0] == 0 and b[-1] == 50_000 and np.all(np.diff(b) >= 0)
        assert all(x % 256 == 0 for x in b[1:-1])
        share = np.diff(ptr[b].astype(np.int64)) / ptr[-1]
        # contiguous 256-aligned blocks: a boundary can move by at most one
        # 256-row window past the ideal split (plus the row it lands in)
        p64 = ptr.astype(np.int64)
        win = (p64[np.minimum(np.arange(len(p64)) + 384, len(p64) - 1)] - p64).max() / p64[-1]
        assert share.max() <= 1.0 / n + win + 1e-12


def _vb_worker(rank, world, port, q):
    """Online VB's item-pass protocol (vbo.cpp item_pass): users split by the
    library's partition, every case local to its user's rank; per batch each
    rank sums its cases' terms per item of the batch's global item list, the
    per-rank sums are all-gathered and added in rank order."""
    try:
        sys.path.insert(0, PKG)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from sbmf import partition_rows, synth
        train, _, dims = synth.generate("ml-100k", seed=5)
        u, it, r = train
        ptr = np.concatenate([[0], np.cumsum(np.bincount(u, minlength=dims[0]))]).astype(np.uint32)
        b = partition_rows(ptr, world)
        mine = (u >= b[rank]) & (u < b[rank + 1])
        nb = 30
        bid = np.random.default_rng(11).permutation(len(u)) % nb  # the same shuffle on every rank
        x = r * np.cos(u.astype(np.float64))  # a per-case term (e1-like)
        ok, maxerr = True, 0.0
        for batch in range(nb):
            inb = bid == batch
            items, gcnt = np.unique(it[inb], return_counts=True)  # the batch's global item list
            g = np.searchsorted(items, it)
            send = np.zeros((len(items), 2))
            sel = inb & mine
            np.add.at(send[:, 0], g[sel], x[sel])
            np.add.at(send[:, 1], g[sel], 1.0)
            parts = [torch.zeros_like(torch.from_numpy(send)) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(send))
            tot = np.zeros_like(send)
            for p in parts:  # rank order
                tot += p.numpy()
            ref = np.zeros(len(items))
            np.add.at(ref, g[inb], x[inb])
            ok &= bool(np.array_equal(tot[:, 1], gcnt.astype(np.float64)))  # every case counted once
            maxerr = max(maxerr, float(np.abs(tot[:, 0] - ref).max()))
            gathered = [None] * world
            dist.all_gather_object(gathered, tot[:, 0].tobytes())
            ok &= all(gb == gathered[0] for gb in gathered)  # bit-identical on every rank
        q.put((rank, ok, maxerr, int(mine.sum())))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e), None))


def test_two_rank_vb_item_sums_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_vb_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok, maxerr, nloc in res:
        assert ok, (rank, maxerr)
        assert maxerr < 1e-9
        assert nloc > 0
