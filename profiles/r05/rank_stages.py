#!/usr/bin/env python3
"""Per-rank stage compute of the 8-way split, on one GPU.

BASELINE config 4 (ML-20M-shaped, K=200, f64) as rank r of an N=8 run, every rank
in turn, through sbmf_test_virtual_rank: the rank runs exactly its own row blocks,
nnz-balanced stages per half (2, the default for several ranks), bins and streaming tasks, with the exchange
skipped (timing only; other ranks' rows keep their initial values, their
residuals read 0; SBMF_STAGES sets the stages per half).  Per rank and stage: the device time on the compute stream
(HIP events), the stage's rows / ratings and its longest row.  The stage holding
the rank's longest split item row is marked.  Philox stream, residuals carried
(recompute_every 0): the benchmarked configuration.

  python3 profiles/r05/rank_stages.py [--ranks 8] [--K 200] [--shape ml-20m] [--sweeps 3] [--only R]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "scalable-bayesian-matrix-factorization_amd"))
from sbmf import Data, FMLearnSBPMF, lib, partition_rows, synth  # noqa: E402


def stage_cuts(ptr, b0, b1, nst):
    """sbmf.cpp partition(): a block cut into nst nnz-balanced stages."""
    sb = [b0]
    for p in range(1, nst + 1):
        row = b1
        if p < nst:
            target = ptr[b0] + (ptr[b1] - ptr[b0]) * p / nst
            row = int(np.searchsorted(ptr[b0:b1 + 1], np.uint32(round(target)), side="left")) + b0
            row = min(max(row, b0), b1)
        sb.append(max(sb[-1], row))
    return sb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--shape", default="ml-20m")
    ap.add_argument("--sweeps", type=int, default=3)
    ap.add_argument("--only", type=int, default=-1)
    ap.add_argument("--tune", type=int, default=0)
    args = ap.parse_args()
    tr, te, dims = synth.generate(args.shape)
    I, J = dims
    uptr = np.zeros(I + 1, np.int64)
    np.add.at(uptr, tr[0].astype(np.int64) + 1, 1)
    uptr = np.cumsum(uptr).astype(np.uint32)
    iptr = np.zeros(J + 1, np.int64)
    np.add.at(iptr, tr[1].astype(np.int64) + 1, 1)
    iptr = np.cumsum(iptr).astype(np.uint32)
    N = args.ranks
    ub, ib = partition_rows(uptr, N), partition_rows(iptr, N)
    trd, ted = Data(*tr), Data(*te)
    NST = int(os.environ.get("SBMF_STAGES", "2"))  # the library's default for several ranks
    out = {"shape": args.shape, "K": args.K, "ranks": N, "stages": NST, "tune": args.tune, "n_train": int(len(tr[0])), "per_rank": []}
    ranks = [args.only] if args.only >= 0 else list(range(N))
    for r in ranks:
        L = FMLearnSBPMF(num_factor=args.K, seed=2015, rng="philox", recompute_every=0, tune=args.tune)
        L.init()
        rc = lib.sbmf_test_virtual_rank(L.ctx, N, r)
        assert rc == 0, lib.sbmf_last_error(L.ctx).decode()
        t0 = time.time()
        L.set_data(trd, ted)
        prep = time.time() - t0
        L.learn(sweeps=1)  # warm-up (first sweep: residual recompute, launch-kind events)
        L.learn(sweeps=args.sweeps)
        ms = np.zeros(2 * NST)
        ns = C.c_uint32()
        assert lib.sbmf_test_stage_ms(L.ctx, ms.ctypes.data_as(C.POINTER(C.c_double)), 2 * NST, C.byref(ns)) == 0
        assert ns.value == NST
        t = L.timing()
        hist = L.history[-args.sweeps:]
        rec = {"rank": r, "prepare_s": prep, "ms_sweep": float(np.mean([h["ms_sweep"] for h in hist])),
               "ms_user_half": t.ms_user_half, "ms_item_half": t.ms_item_half, "ms_hyper": t.ms_hyper,
               "ms_eval": t.ms_eval, "halves": {}}
        for sd, (name, ptr, bnd) in enumerate((("user", uptr, ub), ("item", iptr, ib))):
            b0, b1 = int(bnd[r]), int(bnd[r + 1])
            sb = stage_cuts(ptr, b0, b1, NST)
            deg = np.diff(ptr.astype(np.int64))
            longest = int(np.argmax(deg[b0:b1])) + b0 if b1 > b0 else -1
            stages = []
            for p in range(NST):
                s0, s1 = sb[p], sb[p + 1]
                d = deg[s0:s1]
                stages.append({"ms": float(ms[sd * NST + p]), "rows": s1 - s0, "ratings": int(d.sum()),
                               "longest_row": int(d.max()) if len(d) else 0,
                               "split_rows_gt1024": int((d > 1024).sum()),
                               "holds_longest_row": bool(s0 <= longest < s1)})
            rec["halves"][name] = {"rows": b1 - b0, "ratings": int(ptr[b1]) - int(ptr[b0]),
                                   "longest_row": int(deg[longest]) if longest >= 0 else 0, "stages": stages}
        L.close()
        out["per_rank"].append(rec)
        print("rank %d: sweep %.3f ms  user %.3f  item %.3f | user stages %s | item stages %s" % (
            r, rec["ms_sweep"], t.ms_user_half, t.ms_item_half,
            " ".join("%.3f%s" % (s["ms"], "*" if s["holds_longest_row"] else "")
                     for s in rec["halves"]["user"]["stages"]),
            " ".join("%.3f%s" % (s["ms"], "*" if s["holds_longest_row"] else "")
                     for s in rec["halves"]["item"]["stages"])), file=sys.stderr, flush=True)
    pr = out["per_rank"]
    if len(pr) == N:
        # the pipelined half ends with its slowest rank's stages; per stage p, the exchange of p
        # runs while p+1 computes, so the compute critical path is max over ranks per half
        out["max_over_ranks"] = {h: max(sum(s["ms"] for s in x["halves"][h]["stages"]) for x in pr)
                                 for h in ("user", "item")}
        out["max_stage_ms"] = {h: [max(x["halves"][h]["stages"][p]["ms"] for x in pr) for p in range(NST)]
                               for h in ("user", "item")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
