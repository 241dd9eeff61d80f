import sys
sys.path[:0] = ["/root/repo", "/root/repo/yieldfactormodels.jl_amd"]
import numpy as np, torch
from yfm_amd import KIND_TVL, get_engine, synthetic as S
eng = get_engine(0)
mats = S.maturities_30()
Y = S.simulate_panel(KIND_TVL, 80, maturities=mats)
Th = S.theta_batch(KIND_TVL, 16, seed=43, bad_frac=0.0, scale=0.02)
eng.set_panel(Y, mats)
import os
os.environ["YFM_TVL_LANES"] = "4"
ll = eng.loglik(KIND_TVL, np.asfortranarray(Th[:, 14:15]))
torch.cuda.synchronize()
print("ll", ll)
