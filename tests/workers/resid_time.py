import sys, time, os
sys.path.insert(0, "scalable-bayesian-matrix-factorization_amd")
os.environ.setdefault("SBMF_SYNTH_CACHE", "/tmp/c")
from sbmf import synth, Data, FMLearnSBPMF
tr, te, dims = synth.generate("ml-20m")
L = FMLearnSBPMF(num_factor=100, seed=1, rng="philox", recompute_every=1)
L.set_data(Data(*tr), Data(*te))
L.learn(sweeps=3)
t = L.timing()
print("ms_hyper (includes resid recompute) %.3f, user %.3f, item %.3f, sweep %.3f" % (t.ms_hyper, t.ms_user_half, t.ms_item_half, L.history[-1]["ms_sweep"]))
