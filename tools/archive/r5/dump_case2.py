"""Find the 1,024-sample candidate furthest from the truth (in-tree library), then (second invocation with
--dump b) run it alone so a YFM_TVL_DUMP build prints its per-step loading-basis sums."""
import sys
sys.path[:0] = ["/root/repo", "/root/repo/yieldfactormodels.jl_amd"]
import numpy as np
import torch
from yfm_amd import KIND_TVL, get_engine, synthetic as S
eng = get_engine(0)
mats = S.maturities_360()
Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
eng.set_panel(Y, mats)
with np.load("/root/repo/tests/golden/config3/tvl_config3_1024.npz", allow_pickle=False) as z:
    Th, tru = z["Theta"], z["loglik_truth"]
if sys.argv[1] == "--find":
    got = eng.loglik(KIND_TVL, Th)
    fin = np.isfinite(tru) & np.isfinite(got)
    e = np.zeros(len(got)); e[fin] = np.abs(got[fin] - tru[fin]) / np.abs(tru[fin])
    o = np.argsort(-e)[:8]
    print("worst", [(int(b), float(e[b])) for b in o])
else:
    b = int(sys.argv[2])
    ll = eng.loglik(KIND_TVL, np.asfortranarray(Th[:, b:b + 1]))
    torch.cuda.synchronize()
    print("ll", b, ll, "truth", tru[b], "rel", abs(ll[0] - tru[b]) / abs(tru[b]))
