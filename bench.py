#!/usr/bin/env python3
"""bench.py -- ratings/sec per SBPMF Gibbs sweep on MI355X (BASELINE.json metric).

Workload: ML-20M K=100 (BASELINE.json `metric`), as a synthetic stand-in with
the ML-20M shape (138,493 users x 26,744 items, 18,000,237 train / 2,000,026
test ratings; sbmf/synth.py) -- the MovieLens files are not available offline.
A "step" is one full Gibbs sweep: residual statistics + host
hyperparameter draws (tau, sigma, mu), user half-sweep, item half-sweep and
test evaluation (running-mean RMSE), all with inputs resident in HBM.
RNG: Philox in-kernel (throughput mode); arithmetic: f64 (the reference's).

Online VB (BASELINE config 5, `-method vb`): python bench.py --method vb
  [--shape netflix --K 200]; a step is one epoch (30 mini-batches) of the
  online variational-Bayes learner over a Netflix-shaped synthetic set of
  100 M ratings.  Under torchrun (N GPUs) the users are split into N ranges
  (one rank each, every case of those users local) and the item rows' sums
  are all-gathered per pass (RCCL); the dataset is fixed, so scaling is strong.

Single GPU:  python bench.py [--steps K --warmup W]
Multi GPU:   python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
  one process per GPU; users/items are row-block partitioned (nnz balanced)
  and the fresh U / V blocks are exchanged with RCCL (grouped in-place
  broadcasts over xGMI) between half-sweeps, the cross-rank residuals with a
  grouped ncclSend/ncclRecv exchange.  The dataset is fixed, so the
  scaling is strong.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "scalable-bayesian-matrix-factorization_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_RPS = 309e3   # SBMF-P, ML-20M K=100, paper Table 3 derived per-sweep throughput


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--method", default="mcmc", choices=["mcmc", "vb", "libfm", "als"],
                    help="mcmc: SBPMF Gibbs (headline); vb: online VB; libfm / als: libFM's own MCMC chain / ALS")
    ap.add_argument("--shape", default=None, help="ml-20m (mcmc default) | netflix (vb default) | ml-1m | ...")
    ap.add_argument("--K", type=int, default=None, help="factors (default 100 mcmc / 200 vb)")
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--quirks", default="final",
                    help="final (gibbs_sbpmf_final.cpp, headline) | bias2 (the biased sampler of the top-level "
                         "gibbs_sbpmf2.cpp: the paper's SBMF-P model) | bias22 | sbpmf2 | none")
    ap.add_argument("--no-f32", action="store_true", help="skip the extra f32 measurement")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-ttr", action="store_true", help="skip the time-to-RMSE runs")
    ap.add_argument("--no-load", action="store_true", help="skip the text / binary load timing")
    ap.add_argument("--tune", type=int, default=0, help="kernel-variant bits (sbmf_config.tune)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="sbmf_config.pipeline = 0: each sweep is reported before the next one is queued")
    ap.add_argument("--split-chunk", type=int, default=0, help="streaming task size (0 = the register capacity of the workgroup shape: 512 / 1024 / 2048 f64 ratings for 4 / 8 / 16 waves)")
    ap.add_argument("--stream-threshold", type=int, default=0, help="rows above this use the streaming kernel")
    ap.add_argument("--device", type=int, default=-1,
                    help="HIP device for every rank (testing only; default: LOCAL_RANK)")
    ap.add_argument("--shape-override", default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if args.device < 0 else args.device
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints its "[Gloo] Rank k is connected to ..." banner on stdout while it
        # connects: keep it on stderr so rank 0's stdout is the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(world, x):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


_HIP = None


def device_sync():
    """hipDeviceSynchronize through the HIP runtime libsbmf is bound to (the
    role torch.cuda.synchronize() plays in the bench contract; calling torch's
    would start torch's own bundled runtime as a second HSA runtime here)."""
    global _HIP
    if _HIP is None:
        import ctypes
        from sbmf import _lib  # noqa: F401  (binds libamdhip64.so.7)
        _HIP = ctypes.CDLL("libamdhip64.so.7")
    rc = _HIP.hipDeviceSynchronize()
    if rc != 0:
        raise RuntimeError("hipDeviceSynchronize failed: %d" % rc)


def _lib_kind_names():
    from sbmf._lib import KIND_NAMES
    return KIND_NAMES


def make_learner(args, world, rank, local, precision, comm):
    from sbmf import Data, FMLearnSBPMF
    L = FMLearnSBPMF(num_factor=args.K, seed=2015, rng="philox", precision=precision, device=local,
                     quirks=args.quirks, recompute_every=0, eval_train=False, tune=args.tune,
                     split_chunk=args.split_chunk, stream_threshold=args.stream_threshold,
                     pipeline=0 if args.no_pipeline else 1)
    L.init(comm=comm)
    return L, Data


def measure(args, world, rank, local, precision, train, test, comm):
    L, Data = make_learner(args, world, rank, local, precision, comm)
    t0 = time.time()
    L.set_data(Data(*train), Data(*test))
    prep_s = time.time() - t0
    for _ in range(args.warmup):
        L.learn(sweeps=1)
    barrier(world)
    device_sync()
    t0 = time.perf_counter()
    from sbmf._lib import NKIND
    kern_ms = np.zeros((2, NKIND))

    # each sweep's streaming-kind times (HIP events), read from the callback; the other kinds are
    # timed on a run's first sweep only (their values then stay), so they are read once below
    KS = list(_lib_kind_names()).index("gres_stage")
    stream_ms = np.zeros(2)

    def per_sweep(_rec):
        t = L.timing()
        stream_ms[0] += t.kern_ms[0][KS]
        stream_ms[1] += t.kern_ms[1][KS]
        return False

    # one run of K sweeps (sweep s+1's start is queued at the end of sweep s; the Gram-block
    # kinds are timed on the run's first sweep, the streaming kind on every sweep)
    L.learn(sweeps=args.steps, callback=per_sweep)
    device_sync()
    barrier(world)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(world, dt)
    t = L.timing()
    kern_ms[:] = np.array([[t.kern_ms[s][k] for k in range(NKIND)] for s in range(2)]) * args.steps
    kern_ms[:, KS] = stream_ms
    kbytes = np.array([[t.kern_bytes[s][k] for k in range(NKIND)] for s in range(2)], dtype=np.float64)
    krows = np.array([[t.kern_rows[s][k] for k in range(NKIND)] for s in range(2)])
    res = {
        "seconds": dt, "prep_s": prep_s, "kern_ms": kern_ms / args.steps, "kern_bytes": kbytes, "kern_rows": krows,
        "bytes_alg": t.bytes_algorithmic, "rmse": L.history[-1]["rmse_avg"],
        "sweeps_run": len(L.history), "ms_user": t.ms_user_half, "ms_item": t.ms_item_half, "ms_hyper": t.ms_hyper,
        "ms_eval": t.ms_eval, "ms_comm": t.ms_comm,
    }
    L.close()
    return res


def standalone_kinds(args, local, train, test, reps=3):
    """Every launch kind's device time ALONE: the serial schedule (tune bit 29: a half's
    launches one after the other on one stream, nothing beside them), the kinds timed with
    HIP events on the first sweep of each run.  The default schedule overlaps a half's
    launches, so its per-kind windows include the time a kind waits for CU slots beside
    the persistent streaming launch; these are the rates the bins quote."""
    from sbmf import Data, FMLearnSBPMF
    from sbmf._lib import NKIND
    L = FMLearnSBPMF(num_factor=args.K, seed=2015, rng="philox", precision=args.precision, device=local,
                     quirks=args.quirks, recompute_every=0, eval_train=False, tune=args.tune | (1 << 29),
                     split_chunk=args.split_chunk, stream_threshold=args.stream_threshold)
    L.set_data(Data(*train), Data(*test))
    L.learn(sweeps=1)
    acc = np.zeros((2, NKIND))
    for _ in range(reps):
        L.learn(sweeps=1)  # a run's first sweep times every kind
        t = L.timing()
        acc += np.array([[t.kern_ms[s][k] for k in range(NKIND)] for s in range(2)])
    L.close()
    return acc / reps


def time_to_rmse(args, world, rank, local, train, test, comm, burnin, quirks="final", target=0.85, max_sweeps=200):
    """Wall-clock from the end of data load to the first sweep whose running-mean
    test RMSE <= target, with the reference's averaging rule.
    Two clocks: `seconds` starts after set_data (host CSR/CSC build, task lists,
    uploads, factor init: `prepare_s`), `seconds_from_load` before it."""
    from sbmf import Data, FMLearnSBPMF
    # quirks "final": the reference sampler gibbs_sbpmf_final.cpp (no biases);
    # "bias2": the paper's SBMF-P model with biases, top-level gibbs_sbpmf2.cpp:335-637
    # (init N(0, 0.1), clamp [0.5, 5]).  Both use the variance as the stdev.
    # Burn-in 0: the reference default and its averaging rule (sum / (sweep+1));
    # burn-in 50 (paper protocol): the running mean is taken over the collected
    # sweeps only -- the one change from the reference, whose divisor also counts
    # the burn-in sweeps (gibbs_sbpmf_final.cpp:559).
    L = FMLearnSBPMF(num_factor=args.K, seed=2015, rng="philox", precision=args.precision, device=local,
                     recompute_every=0, burnin=burnin, tune=args.tune,
                     split_chunk=args.split_chunk, stream_threshold=args.stream_threshold,
                     quirks=quirks, average="collected" if burnin else "reference")
    L.init(comm=comm)
    barrier(world)
    tl = time.perf_counter()
    L.set_data(Data(*train), Data(*test))
    barrier(world)
    t0 = time.perf_counter()
    hit = None
    # stop rule depends only on the (rank-identical) running-mean RMSE and the
    # sweep count, so every rank leaves the loop after the same sweep
    while len(L.history) < max_sweeps:
        L.learn(sweeps=1)
        if L.history[-1]["sweep"] >= burnin and L.history[-1]["rmse_avg"] <= target:
            hit = time.perf_counter() - t0
            break
    n = len(L.history)
    last = L.history[-1]["rmse_avg"]
    this = np.array([h["rmse_this"] for h in L.history])
    tau = np.array([h["tau"] for h in L.history])
    L.close()
    out = {"seconds": hit, "seconds_from_load": None if hit is None else hit + (t0 - tl), "prepare_s": t0 - tl,
           "sweeps": n, "rmse": last, "burnin": burnin, "quirks": quirks,
           "average": "collected sweeps" if burnin else "sum / (sweep + 1) (reference)",
           "target": "synthetic proxy: RMSE %.2f on the planted rank-10 set (noise floor ~0.58), not MovieLens" % target,
           "clock": "end of data load -> first sweep with running-mean test RMSE <= %.2f" % target,
           "min_rmse_this": float(np.nanmin(this)), "min_rmse_this_sweep": int(np.nanargmin(this)),
           "rmse_this_last": float(this[-1]), "tau_last": float(tau[-1])}
    if hit is None and quirks == "bias2":
        out["note"] = ("not reached: the biased sampler (top-level gibbs_sbpmf2.cpp, the paper's SBMF-P model) never "
                       "leaves the bias-only fit on this set (best per-sweep test RMSE %.3f; factor precisions drawn "
                       "with shape alpha0 + I and the posterior variance passed as the stdev shrink every factor to "
                       "~0); the compiled reference does the same on the ML-1M-shaped set (tests/golden/"
                       "ref_bias2_ml1msynth_k20_s1.txt: 1.0632 -> 1.0587, test_gpu_collapse.py)" % out["min_rmse_this"])
    elif hit is None:
        bad = np.flatnonzero(~np.isfinite(tau) | (tau < 1e-3))
        out["note"] = ("not reached: the reference sampler's chain (posterior variance used as the stdev) leaves its "
                       "best per-sweep test RMSE %.3f at sweep %d%s; the CPU oracle, bit-exact to "
                       "gibbs_sbpmf_final.cpp, collapses the same way on an ML-1M-shaped set (DESIGN.md §6), so the "
                       "mean of the sweeps collected after burn-in %d stays above the target"
                       % (out["min_rmse_this"], out["min_rmse_this_sweep"],
                          " and collapses from sweep %d (tau -> 0 -> NaN, predictions clamp)" % bad[0] if len(bad)
                          else "", burnin))
    return out


def load_times(train, world, rank):
    """the input formats at this workload's size, from the page
    cache on the bench host -- the SBPMF triple text (gibbs_sbpmf_final.cpp:26-215's
    format) and libFM's binary .x/.y (tools/convert.cpp:55-205), each written once
    by the library's writers and read back through the boundary loaders
    (sbmf_load_triples / sbmf_load_libfm_binary: one read or mapping, line-aligned
    chunks on threads).  The read-back is checked against the generated arrays."""
    import shutil
    import tempfile
    import sbmf
    if world > 1 and rank != 0:
        return None
    d = tempfile.mkdtemp(prefix="sbmf_load_")
    try:
        data = sbmf.Data(*train)
        txt, stem = os.path.join(d, "train.tsv"), os.path.join(d, "train")
        t = time.perf_counter()
        sbmf.save_triples(txt, data)
        w_txt = time.perf_counter() - t
        t = time.perf_counter()
        sbmf.save_libfm_binary(stem, data)
        w_bin = time.perf_counter() - t
        out = {"n": len(train[0]), "threads": int(os.environ.get("SBMF_LOAD_THREADS") or
                                                  min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS") or 64))),
               "text_bytes": os.path.getsize(txt),
               "binary_bytes": os.path.getsize(stem + ".x") + os.path.getsize(stem + ".y"),
               "write_text_s": w_txt, "write_binary_s": w_bin}
        for key, fn in (("load_text_s", lambda: sbmf.load_triples(txt)),
                        ("load_binary_s", lambda: sbmf.load_libfm_binary(stem))):
            best = None
            for _ in range(2):  # first read (cold process memory) and a second one
                t = time.perf_counter()
                got = fn()
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
                out.setdefault(key + "_first", dt)
            out[key] = best
            ok = np.array_equal(got.user, train[0]) and np.array_equal(got.item, train[1])
            # the text round trip is bit-exact; the binary format stores f32 targets (ratings 1..5: exact)
            ok = ok and np.array_equal(got.rating, train[2])
            if not ok:
                raise RuntimeError("%s read back different ratings" % key)
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


# Restatement-to-reference speed, measured in the build container (one core) on the
# reference's own inputs: the CPU baselines below time the restatements (the compiled
# reference does not travel to the GPU box), so each line states how they compare.
RESTATEMENT_VS_REFERENCE = {
    "final": "oracle 0.83 s vs oracle/_ref/gibbs_sbpmf_final 0.90 s (incl. its text load) for 100 sweeps of "
             "ML-100k K=20 on one build-container core: the restatement runs at the reference's speed "
             "(ratio ~1.07; 1.18 on a busier rerun)",
    "bias2": "oracle 2.15 s vs oracle/_ref/gibbs_sbpmf2_bias (top-level gibbs_sbpmf2.cpp) 2.27 s for 100 sweeps "
             "of ML-100k K=20 on one build-container core: ratio 1.06",
    "libfm": "fmm_oracle 13.4 ms vs oracle/_ref/libFM (libfm.cpp compiled unmodified) 25.7 ms per MCMC iteration "
             "(ALS 14.1 vs 25.6 ms) on the reference's data/m1m/m100k/*_libfm, -dim 1,1,8, one build-container "
             "core: the restatement is ~1.9x faster than libFM, so this baseline overstates the reference CPU",
    "vb": "vbo_oracle 0.042 s vs oracle/_ref/ref_vbo_harness (fm_learn_vb_online*.h compiled unmodified) 0.26 s per "
          "epoch, ML-100k K=8, 10 epochs, one build-container core (the reference writes and re-reads its "
          "per-epoch batch files): the restatement is ~6x faster, so this baseline overstates the reference CPU",
}


# the reference source each oracle quirk set restates (oracle/sbpmf_oracle.c)
QUIRK_SOURCE = {"final": "gibbs_sbpmf_final.cpp", "sbpmf2": "src/libfm/gibbs_sbpmf2.cpp",
                "none": "gibbs_sbpmf_final.cpp with sqrt(variance) as the stdev (no reference file)",
                "bias2": "the top-level biased gibbs_sbpmf2.cpp", "bias22": "src/libfm/gibbs_sbpmf22.cpp"}


def cpu_baseline(train, test, dims, K, seconds, quirks="final"):
    """The oracle (serial CPU restatement of gibbs_sbpmf_final.cpp -- or, quirks
    bias2, of the top-level biased gibbs_sbpmf2.cpp -- 1 thread) on a bounded
    random subsample of the same workload (same users/items)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    n = len(train[0])
    tsub = tuple(a[:1000] for a in test)
    # one sweep of the FULL set when it fits ~`seconds` at the oracle's speed on one core (measured
    # 1.24 M ratings/s at K=100 on the GPU box, r05; scaled by 100 / K): ML-20M K=100 is ~15 s.
    # Larger sets: a random subsample sized to `seconds`, and the line says so.
    est = 1.24e6 * 100.0 / max(K, 1)
    take = n if n <= est * seconds else int(max(100_000, est * seconds))
    if take < n:
        idx = np.random.default_rng(7).permutation(n)[:take]
        sub = tuple(a[idx] for a in train)
    else:
        sub = train
    r = oracle.run(sub, tsub, K=K, iters=1, seed=1, num_users=dims[0], num_items=dims[1], want_factors=False,
                   quirks=quirks)
    src = QUIRK_SOURCE.get(quirks, QUIRK_SOURCE["final"])
    what = ("1 sweep of the full %d-rating set" % n if take == n else
            "1 sweep on a random %d-rating subsample of the %d-rating set (all users and items kept; the rate "
            "per rating is the measured one, not extrapolated to the full set)" % (take, n))
    out = {"value": take / r["seconds"], "unit": "ratings/s", "cores": 1, "kind": "port",
           "sample": "oracle (serial C restatement of %s, glibc RNG, f64): %s, %d users x %d items, K=%d, %.1f s"
                     % (src, what, dims[0], dims[1], K, r["seconds"]),
           "restatement_vs_reference": RESTATEMENT_VS_REFERENCE.get(quirks)}
    if quirks != "final":
        return out
    # the same restatement, rows of each half in parallel
    # (OpenMP) with the Philox stream, on the host's cores, one sweep of the full set
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    rp = oracle.run(train, tsub, K=K, iters=1, seed=1, num_users=dims[0], num_items=dims[1], want_factors=False,
                    rng="philox", threads=threads)
    out["all_cores"] = {"value": n / rp["seconds"], "unit": "ratings/s", "cores": threads, "kind": "port",
                        "sample": "oracle, OpenMP row-parallel over %d threads, Philox stream, f64, 1 sweep of the "
                                  "full %d-rating set, K=%d, %.2f s" % (threads, n, K, rp["seconds"])}
    return out


def mk_comm(world, rank, local):
    """The process's one communicator (sbmf_comm_create: ncclCommInitRank once), from a
    fresh RCCL unique id made by rank 0 and shared over the gloo bootstrap group; every
    learner of this process attaches to it in turn (sbmf_comm_attach)."""
    if world == 1:
        return None
    import torch.distributed as dist
    from sbmf import Communicator, comm_unique_id
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return Communicator(world, rank, obj[0], device=local)


def vb_main(args):
    """BASELINE config 5: online VB epochs (ratings/s per epoch)."""
    from sbmf import Data, FMLearnVBOnline, synth
    world, rank, local = dist_setup(args)
    say = (lambda *a: print(*a, file=sys.stderr, flush=True)) if rank == 0 else (lambda *a: None)
    say("[bench vb] generating the %s-shaped set" % args.shape)
    t0 = time.time()
    train, test, dims = synth.generate(args.shape)
    say("[bench vb] %d train ratings in %.0f s" % (len(train[0]), time.time() - t0))
    n_train = len(train[0])
    comm = mk_comm(world, rank, local)
    L = FMLearnVBOnline(num_factor=args.K, seed=2015, rng="philox", device=local)
    L.init(comm=comm)
    t0 = time.time()
    L.set_data(Data(*train), Data(*test))
    prep_s = time.time() - t0
    for _ in range(args.warmup):
        L.learn(sweeps=1)
        say("[bench vb] warm-up epoch %.0f ms (GPU)" % L.history[-1]["ms_sweep"])
    barrier(world)
    device_sync()
    t0 = time.perf_counter()
    L.learn(sweeps=args.steps, callback=lambda h: say("[bench vb] epoch %.0f ms (GPU)" % h["ms_sweep"]) and False)
    device_sync()
    barrier(world)
    dt = max_over_ranks(world, time.perf_counter() - t0)
    hist = L.history[-args.steps:]
    gpu_ms = float(np.mean([h["ms_sweep"] for h in hist]))
    K = args.K
    one_device = world > 1 and (os.environ.get("SBMF_COMM") == "host" or args.device >= 0)
    # algorithmic bytes per epoch (f64): per case the two partner rows of
    # means and variances for the prediction (4 * 8K), and per factor pass
    # (2K of them) the {e,t} record read + written (32), the partner mean and
    # variance (16) and its ids (8)
    bytes_epoch = n_train * (32.0 * K + 2 * K * 56.0)
    bytes_factor = n_train * 2 * K * 56.0  # the factor passes alone: the epoch's dominant kernels
    factor_ms = float(L.timing().ms_vb_factor)
    vb_traffic = vb_traffic_src = None
    pv = os.path.join(REPO, "profiles", "pmc_vb_traffic.json")
    if os.path.exists(pv) and not one_device and world == 1:
        pm = json.load(open(pv))
        vb_traffic = pm.get("vb_factor_passes")
        vb_traffic_src = "profiles/pmc_vb_traffic.json (%s)" % pm.get("_run", "run not recorded")
    out = {
        "metric": "ratings/sec per online-VB epoch, %s K=%d" % ({"netflix": "synthetic 100M (Netflix-shaped)"}.get(
            args.shape, args.shape), K),
        "value": n_train * args.steps / dt, "unit": "ratings/s", "n_gpus": 1 if one_device else world,
        "n_ranks": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True,
        "scaling": "not a scaling number (%d ranks on one GPU)" % world if one_device else "strong",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic %s-shaped (sbmf/synth.py)" % args.shape,
        "config": {"workload": "online VB epoch (30 mini-batches: e/t terms, update_w0, update_w, factor-outer "
                               "update_v, hyperparameter blends) + test RMSE", "method": "vb",
                   "parallelism": "user ranges x%d (%s)" % (world, "host-shm exchange, testing only"
                                                             if os.environ.get("SBMF_COMM") == "host"
                                                             else "RCCL all-gather of the item sums"),
                   "num_users": dims[0], "num_items": dims[1], "n_train": n_train, "n_test": len(test[0]), "K": K,
                   "rng": "philox", "prep_s": prep_s, "gpu_ms_per_epoch": gpu_ms,
                   "test_rmse_after": hist[-1]["rmse_avg"], "epochs_run": len(L.history)},
        "roofline": {"kernel": "factor passes (every mini-batch's 2K k_user_v / k_item_vp launches)", "bound": "hbm",
                     "achieved": bytes_factor / (factor_ms * 1e-3) / 1e9 if factor_ms > 0 else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": bytes_factor / (factor_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if factor_ms > 0 else None,
                     "traffic": vb_traffic, "traffic_source": vb_traffic_src or (
                         "none: rocprofv3 --pmc FETCH_SIZE over this line segfaulted in a profiler thread right "
                         "after HSA init (profiles/r06/r06s19_vb_pmc_fetch_crash.log); round 3's VB passes "
                         "(profiles/r03_vb_*) predate the current kernels"), "bytes_per_epoch": bytes_factor,
                     "ms_per_epoch": factor_ms,
                     "timing": "HIP events around each mini-batch's factor loop on the compute stream "
                               "(sbmf_timing.ms_vb_factor), mean over the timed epochs",
                     "epoch_aggregate": {"kernels": "every VB kernel of the epoch", "bytes": bytes_epoch,
                                         "ms": gpu_ms, "frac": bytes_epoch / (gpu_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}},
    }
    L.close()
    if not args.no_cpu and rank == 0 and world == 1:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle
        n = len(train[0])
        take = int(min(n, 2_000_000))
        idx = np.random.default_rng(7).permutation(n)[:take]
        sub = tuple(a[idx] for a in train)
        tsub = tuple(a[:1000] for a in test)
        r = oracle.run_vbo(sub, tsub, K=K, epochs=1, seed=1, num_users=dims[0], num_items=dims[1],
                           seconds_limit=args.cpu_seconds, want_params=False)
        out["cpu_baseline"] = {"value": take * r["epochs"] / r["seconds"], "unit": "ratings/s", "cores": 1,
                               "kind": "port",
                               "sample": "oracle (vbo_oracle.c, serial C restatement of fm_learn_vb_online, f64) for "
                                         "1 epoch on a random %d-rating subsample (all %d users x %d items kept), "
                                         "K=%d, %.1f s" % (take, dims[0], dims[1], K, r["seconds"]),
                               "restatement_vs_reference": RESTATEMENT_VS_REFERENCE["vb"]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    from sbmf import _lib
    _lib.unload()


def libfm_cpu_baseline(train, test, dims, K, als, seconds):
    """fmm_oracle (serial C restatement of libFM's fm_learn_mcmc / ALS, glibc RNG,
    1 thread) for one iteration on a random subsample of the same set, sized from
    a small calibration run to about `seconds`."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    n = len(train[0])
    rng = np.random.default_rng(7)
    perm = rng.permutation(n)
    tsub = tuple(a[:1000] for a in test)
    kw = dict(K=K, iters=1, seed=1, method="als" if als else "mcmc",
              regular=(0.0, 0.0, 10.0) if als else (0.0, 0.0, 0.0), num_users=dims[0], want_params=False)
    cal = min(n, 200_000)
    r = oracle.run_fmm(tuple(a[perm[:cal]] for a in train), tsub, **kw)
    # one iteration = (2 iterations) - (1 iteration) on the sample, about seconds / 3 each
    take = int(min(n, max(cal, cal * seconds / 3 / max(r["seconds"], 1e-3))))
    sub = tuple(a[perm[:take]] for a in train)
    r1 = oracle.run_fmm(sub, tsub, **kw)
    r2 = oracle.run_fmm(sub, tsub, **dict(kw, iters=2))
    it_s = max(r2["seconds"] - r1["seconds"], 1e-9)
    return {"value": take / it_s, "unit": "ratings/s", "cores": 1, "kind": "port",
            "sample": "fmm_oracle (serial C restatement of libFM's %s, glibc RNG, f64): the second iteration on a "
                      "random %d-rating subsample of the same synthetic set (all %d users x %d items kept), K=%d, "
                      "%.1f s (set-up excluded: 2 iterations %.1f s - 1 iteration %.1f s)"
                      % ("ALS" if als else "fm_learn_mcmc", take, dims[0], dims[1], K, it_s, r2["seconds"],
                         r1["seconds"]),
            "restatement_vs_reference": RESTATEMENT_VS_REFERENCE["libfm"]}


def libfm_main(args):
    """libFM's own MCMC chain (-method mcmc -order libfm) or ALS on the ML-20M
    shape: ratings/s per iteration (draw_all + re-prediction + test RMSE)."""
    from sbmf import Data, FMLearnSBPMF, synth
    world, rank, local = dist_setup(args)
    train, test, dims = synth.generate(args.shape)
    n_train, n_test, K = len(train[0]), len(test[0]), args.K
    als = args.method == "als"
    comm = mk_comm(world, rank, local)
    L = FMLearnSBPMF(num_factor=K, seed=2015, rng="philox", method="als" if als else "mcmc", order="libfm",
                     regular=(0.0, 0.0, 10.0) if als else (0.0, 0.0, 0.0), init_stdev=0.1, device=local)
    L.init(comm=comm)
    L.set_data(Data(*train), Data(*test))
    L.learn(sweeps=args.warmup)
    barrier(world)
    device_sync()
    t0 = time.perf_counter()
    L.learn(sweeps=args.steps)
    device_sync()
    barrier(world)
    dt = max_over_ranks(world, time.perf_counter() - t0)
    one_device = world > 1 and (os.environ.get("SBMF_COMM") == "host" or args.device >= 0)
    hist = L.history[-args.steps:]
    gpu_ms = float(np.mean([h["ms_sweep"] + h["ms_eval"] for h in hist]))
    # algorithmic bytes per iteration (f64): 2K + 2 passes over every case, each reading
    # the residual (8), writing it in the other order (8), the case's partner id and
    # position (8) and the partner value (8; the item side also the user's old value, 8);
    # the re-prediction reads two attribute rows of K doubles per train and test case
    # and writes the train residual
    passes = 2 * (K + 1)
    bytes_it = n_train * passes * 32.0 + n_train * K * 8.0 + (n_train + n_test) * (16.0 * K + 8.0)
    out = {
        "metric": "ratings/sec per libFM %s iteration, %s K=%d" % ("ALS" if als else "MCMC", args.shape, K),
        "value": n_train * args.steps / dt, "unit": "ratings/s", "n_gpus": 1 if one_device else world,
        "n_ranks": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * dt / args.steps,
        "higher_is_better": True,
        "scaling": "not a scaling number (%d ranks on one GPU)" % world if one_device else "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic %s-shaped (sbmf/synth.py)" % args.shape,
        "config": {"workload": "libFM fm_learn_mcmc iteration (alpha, w0, w, f-outer v passes, re-prediction, "
                               "test RMSE)%s" % (" without sampling (ALS)" if als else ""),
                   "method": "als" if als else "mcmc -order libfm",
                   "parallelism": "user ranges x%d (%s)" % (world, "host-shm exchange, testing only"
                                                             if os.environ.get("SBMF_COMM") == "host"
                                                             else "RCCL all-gather of the item sums"),
                   "num_users": dims[0], "num_items": dims[1],
                   "n_train": n_train, "n_test": n_test, "K": K, "rng": "philox", "gpu_ms_per_iter": gpu_ms,
                   "launches_per_iter": int(L.timing().n_launch), "test_rmse_after": hist[-1]["rmse_avg"]},
        "roofline": {"kernel": "iteration (all libFM-learner kernels)", "bound": "hbm",
                     "achieved": bytes_it / (gpu_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": bytes_it / (gpu_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "bytes_per_iter": bytes_it},
    }
    L.close()
    if not args.no_cpu and rank == 0 and world == 1:
        out["cpu_baseline"] = libfm_cpu_baseline(train, test, dims, K, als, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    from sbmf import _lib
    _lib.unload()


def main():
    args = parse()
    if args.method in ("libfm", "als"):
        if args.shape is None:
            args.shape = "ml-20m"
        if args.K is None:
            args.K = 100
        return libfm_main(args)
    if args.shape is None:
        args.shape = "netflix" if args.method == "vb" else "ml-20m"
    if args.K is None:
        args.K = 200 if args.method == "vb" else 100
    if args.method == "vb":
        return vb_main(args)
    # load libsbmf (ROCm's HIP runtime) before torch.distributed pulls in torch's bundled copy
    from sbmf import synth
    world, rank, local = dist_setup(args)
    from sbmf._lib import KIND_NAMES, NKIND
    KIND_STREAM_IDX = list(KIND_NAMES).index("gres_stage")
    train, test, dims = synth.generate(args.shape)
    comm = mk_comm(world, rank, local)  # one communicator for every leg below
    main_res = measure(args, world, rank, local, args.precision, train, test, comm)
    if args.quirks != "final":  # the extra legs (f32, time-to-RMSE, loads) belong to the headline sampler
        args.no_f32 = args.no_ttr = args.no_load = True
    f32 = None
    if not args.no_f32 and args.precision != "f32":
        f32 = measure(args, world, rank, local, "f32", train, test, comm)
    # time to 0.85: the reference sampler (final) and the paper's biased SBMF-P model (bias2),
    # burn-in 0 and 50 each
    ttr = [time_to_rmse(args, world, rank, local, train, test, comm, b, q)
           for q in ("final", "bias2") for b in (0, 50)] if not args.no_ttr else []
    loads = None if args.no_load else load_times(train, world, rank)
    n_train = len(train[0])
    value = n_train * args.steps / main_res["seconds"]
    ms = 1e3 * main_res["seconds"] / args.steps
    # dominant kernel: the (half, bin) that moves the most algorithmic bytes (the item streaming
    # stage on every sampler line).  Not the largest HIP-event time: a small Gram-block kind that
    # waits for CU slots beside the persistent streaming launch spans about as long as that launch
    # (the r05s3 / r05s23 bias2 lines picked such a window, 0.02 of peak)
    km = main_res["kern_ms"]
    s, k = np.unravel_index(np.argmax(main_res["kern_bytes"]), km.shape)
    achieved = main_res["kern_bytes"][s, k] / (km[s, k] * 1e-3) / 1e9
    kernel = "%s_half/%s" % ("user" if s == 0 else "item", KIND_NAMES[k])
    # HBM traffic and LDS bank conflicts of the dominant launch come from separate rocprofv3 --pmc
    # passes (profiles/collect.sh fetch / write / lds, never in this run); the line names the file
    # and the run they were taken in
    traffic = traffic_src = None
    lds = None
    # the PMC passes were taken on the default single-rank ML-20M K=100 f64 line: only that config quotes them
    profiled = world == 1 and args.shape == "ml-20m" and args.K == 100 and args.quirks == "final" and not args.tune
    if profiled:
        try:
            pm = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
            traffic = pm.get(kernel)
            traffic_src = "profiles/pmc_traffic.json (%s)" % pm.get("_run", "run not recorded")
        except Exception:
            traffic = None
        try:
            pl = json.load(open(os.path.join(REPO, "profiles", "pmc_lds.json")))
            e = pl.get(kernel) or {}
            bc = e.get("bank_conflict_cycles")
            if bc is not None:
                # conflict cycles per CU-cycle of the launch (its live HIP-event time here, every CU
                # at the 2.4 GHz engine clock): the share of the CU time the LDS pipe stalls
                cu_cycles = km[s, k] * 1e-3 * 2.4e9 * 256
                lds = {"conflict_cycles_per_launch": bc, "lds_issue_cycles_per_launch": e.get("lds_active_cycles"),
                       "conflict_cycles_per_cu_cycle": bc / cu_cycles,
                       "source": "profiles/pmc_lds.json (%s)" % pl.get("_run", "run not recorded")}
        except Exception:
            lds = None
    # every launch kind of both halves against its own bound: algorithmic bytes (per
    # launch) / its standalone device time (serial schedule, standalone_kinds); the user side gathers
    # from the 24 MB V table (measured random-row gather ceiling 8.1 TB/s), the item side from the
    # 124 MB U table (6.3 TB/s; profiles/r01_gather_ceiling.txt), both quoted as fractions of the
    # 8 TB/s spec too.  The default schedule's per-kind windows are reported beside them, without a
    # rate: a kind waiting for CU slots beside the persistent streaming launch spans that wait too.
    solo = standalone_kinds(args, local, train, test) if world == 1 else None
    ceil = {0: 8100.0, 1: 6300.0}
    bins = {}
    for s_ in range(2):
        for k_ in range(NKIND):
            if km[s_, k_] <= 0:
                continue
            e = {"rows": int(main_res["kern_rows"][s_, k_]),
                 "GB": round(float(main_res["kern_bytes"][s_, k_]) / 1e9, 4),
                 "ms_default_window": round(float(km[s_, k_]), 4)}
            if k_ != KIND_STREAM_IDX and not (args.tune & (1 << 29)):
                e["overlapped"] = True  # the window shares the device: not a rate
            if solo is not None and solo[s_, k_] > 0:
                gbs = main_res["kern_bytes"][s_, k_] / (solo[s_, k_] * 1e-3) / 1e9
                e.update({"ms_standalone": round(float(solo[s_, k_]), 4), "GB/s": round(float(gbs), 1),
                          "frac_peak": round(float(gbs / HBM_PEAK_GBS), 4),
                          "frac_gather_ceiling": round(float(gbs / ceil[s_]), 4)})
            bins[("user_" if s_ == 0 else "item_") + KIND_NAMES[k_]] = e
    # several ranks on one device (SBMF_COMM=host or --device): a protocol rehearsal, not a scaling point
    one_device = world > 1 and (os.environ.get("SBMF_COMM") == "host" or args.device >= 0)
    out = {
        "metric": "ratings/sec per Gibbs sweep, %s K=%d" % ({"ml-20m": "ML-20M", "ml-10m": "ML-10M", "ml-1m": "ML-1M",
                                                             "ml-100k": "ML-100k", "netflix": "Netflix"}[args.shape],
                                                            args.K),
        "value": value, "unit": "ratings/s", "n_gpus": 1 if one_device else world, "n_ranks": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms, "higher_is_better": True,
        "scaling": "not a scaling number (%d ranks on one GPU)" % world if one_device else "strong",
        "vs_baseline": None if one_device else value / BASELINE_RPS,
        "dtype": args.precision,
        "data": "synthetic %s-shaped (sbmf/synth.py: planted rank-10, Pareto users, log-normal items)"
                % {"ml-20m": "ML-20M", "ml-10m": "ML-10M", "ml-1m": "ML-1M", "ml-100k": "ML-100k",
                   "netflix": "Netflix"}[args.shape],
        "config": {"workload": "%s K=%d SBPMF Gibbs sweep (%suser+item half-sweeps, hyperparameters, test RMSE)"
                               % (args.shape, args.K, "bias draws + " if args.quirks.startswith("bias") else ""),
                   "num_users": dims[0], "num_items": dims[1], "n_train": n_train, "n_test": len(test[0]),
                   "K": args.K, "rng": "philox", "quirks": args.quirks,
                   "parallelism": "rows x%d (%s)" % (world, "host-shm exchange, testing only" if os.environ.get("SBMF_COMM") == "host" else "RCCL block broadcast + p2p residual exchange"),
                   "test_rmse_after": main_res["rmse"], "sweeps_run": main_res["sweeps_run"],
                   "prepare_s": main_res["prep_s"], "load": loads,
                   "time_to_test_rmse_0.85": ttr,
                   "ms_user_half": main_res["ms_user"], "ms_item_half": main_res["ms_item"],
                   "ms_hyper": main_res["ms_hyper"], "ms_eval": main_res["ms_eval"], "ms_comm": main_res["ms_comm"],
                   "kernel_ms": {("user_" if s_ == 0 else "item_") + KIND_NAMES[k_]: round(float(km[s_, k_]), 4)
                                 for s_ in range(2) for k_ in range(NKIND) if km[s_, k_] > 0}},
        "roofline": {"kernel": kernel, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "lds_bank_conflicts": lds,
                     "bytes_per_launch": float(main_res["kern_bytes"][s, k]),
                     "rows_per_launch": int(main_res["kern_rows"][s, k]),
                     "ms_per_launch": float(km[s, k]),
                     "sweep_alg_GBs": main_res["bytes_alg"] / (main_res["seconds"] / args.steps) / 1e9,
                     "bins": bins,
                     "bins_note": "rates from each kind's standalone device time (serial schedule, tune bit 29, "
                     "measured in this run); ms_default_window is the kind's start-to-end span in the default "
                     "schedule, where a half's Gram-block launches run on two side streams beside its "
                     "streaming launch (overlapped: no rate)",
                     "bins_kernels": "bins are row-length classes; by default (f64) gblock_w16 (9-64 ratings) and "
                     "gblock_b4 (65-128) run k_grow<double,1>, gblock_b8 (129-256) k_grow<double,2>, "
                     "gblock_w4 (<= 8) k_gblock, gres_stage k_gres (DESIGN.md 3.1b); f32: k_grow for 17-512"},
    }
    if f32 is not None:
        out["f32_value"] = n_train * args.steps / f32["seconds"]
        out["f32_ms_per_step"] = 1e3 * f32["seconds"] / args.steps
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(train, test, dims, args.K, args.cpu_seconds, args.quirks)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    device_sync()
    from sbmf import _lib
    _lib.unload()


if __name__ == "__main__":
    from sbmf import _lib as _sbmf_lib
    if os.environ.get("SBMF_EXIT") == "guard":
        # opt-in (round 3's default): leave through libsbmf's exit handler after
        # rocprofv3's has written its output.  The finalizer fault it skipped came with
        # RCCL linked at load time; libsbmf now dlopens RCCL for a multi-GPU communicator
        # only, and a plain exit under rocprofv3 is clean
        _sbmf_lib.exit_guard(1)
    rc = 0
    try:
        main()
    except SystemExit as e:  # argparse --help / errors, sys.exit(n): keep their status
        rc = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
        if e.code is not None and not isinstance(e.code, int):
            print(e.code, file=sys.stderr)
    sys.stdout.flush()
    sys.stderr.flush()
    if os.environ.get("SBMF_EXIT") == "guard":
        _sbmf_lib.exit_guard(rc)
    sys.exit(rc)
