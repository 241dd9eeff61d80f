"""Diagnose sweep case 4985 (TVλ, N = 12, T = 3): candidate 4 at every group width, both precisions."""
import os
import sys

import numpy as np

sys.path[:0] = ["yieldfactormodels.jl_amd", "tests", "."]
import torch  # noqa: F401
from test_gpu_random import random_case
from yfm_amd import KIND_TVL, _lib, get_engine
from oracle.truth import loglik_truth

rng = np.random.default_rng(1000 + 4985)
N, T, mats, Y, Th, space, T_use = random_case(rng, KIND_TVL)
print("N", N, "T", T, "B", Th.shape[1], "space", space, "T_use", T_use, "mats", mats)
eng = get_engine(0)
eng.set_panel(Y, mats)
tr = loglik_truth(KIND_TVL, Y, mats, Th, space=space, T_use=T_use)
print("truth[4]", tr[4])
for prec in (_lib.PREC_CERTIFIED, _lib.PREC_FP64):
    eng.precision = prec
    for L in ("", "4", "8", "16", "32", "64"):
        if L:
            os.environ["YFM_TVL_LANES"] = L
        else:
            os.environ.pop("YFM_TVL_LANES", None)
        got = eng.loglik(KIND_TVL, Th, space=space, T_use=T_use)
        print("prec", prec, "L", L or "auto", "got[4]", got[4], "n -inf", int(np.isneginf(got).sum()), "n -inf truth", int(np.isneginf(tr).sum()))
    os.environ.pop("YFM_TVL_LANES", None)
