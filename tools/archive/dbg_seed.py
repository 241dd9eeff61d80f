import sys, numpy as np
sys.path[:0] = ["/root/repo/tests", "/root/repo/yieldfactormodels.jl_amd", "/root/repo"]
import torch  # noqa
from test_gpu_random import random_case, c_oracle
from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL, get_engine
eng = get_engine(0)
for seed in [int(a) for a in sys.argv[1:]]:
    rng = np.random.default_rng(1000 + seed)
    kind = [KIND_DNS, KIND_GNS, KIND_TVL][seed % 3]
    N, T, mats, Y, Th, space, T_use = random_case(rng, kind)
    eng.set_panel(Y, mats)
    g1 = eng.loglik(kind, Th, space=space, T_use=T_use); d1 = eng.last_deferred(); f1 = eng.last_flags()
    g2 = eng.loglik(kind, Th, space=space, T_use=T_use); d2 = eng.last_deferred()
    g3 = eng.loglik(kind, np.asfortranarray(Th[:, :1]), space=space, T_use=None if T_use is None else T_use[:1])
    ref = c_oracle(kind, space, Y, mats, Th, T_use)
    print("seed", seed, "N", N, "T", T, "deferred", d1, d2, "flags", f1)
    print("  got1", g1[:5]); print("  got2", g2[:5]); print("  single", g3); print("  ref ", ref[:5])
