"""Diagnose the two-function update form (YFM_FZ_SPLIT_FORM=1) on the 7a42719 cases: per candidate the
one-body and two-function logliks, the dense oracle and the binary128 truth, and the deferral count.

    python tools/dbg_split.py [seed ...]          (YFM_LIB selects a variant library)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "yieldfactormodels.jl_amd"), ROOT]
import torch  # noqa: E402,F401
from oracle.truth import loglik_oracle, loglik_truth  # noqa: E402
from test_gpu_random import random_case  # noqa: E402
from yfm_amd import KIND_GNS, get_engine  # noqa: E402

eng = get_engine(0)
os.environ["YFM_DNS_STEADY"] = "0"
for seed in [int(a) for a in sys.argv[1:]] or [292, 916, 2431]:
    rng = np.random.default_rng(1000 + seed)
    N, T, mats, Y, Th, space, T_use = random_case(rng, KIND_GNS)
    eng.set_panel(Y, mats)
    os.environ.pop("YFM_FZ_SPLIT_FORM", None)
    one = eng.loglik(KIND_GNS, Th, space=space, T_use=T_use)
    d1 = eng.last_deferred()
    one_b = eng.loglik(KIND_GNS, Th, space=space, T_use=T_use)
    os.environ["YFM_FZ_SPLIT_FORM"] = "1"
    two = eng.loglik(KIND_GNS, Th, space=space, T_use=T_use)
    d2 = eng.last_deferred()
    two_b = eng.loglik(KIND_GNS, Th, space=space, T_use=T_use)
    os.environ.pop("YFM_FZ_SPLIT_FORM", None)
    orc = loglik_oracle(KIND_GNS, Y, mats, Th, space=space, T_use=T_use)
    tru = loglik_truth(KIND_GNS, Y, mats, Th, space=space, T_use=T_use)
    print(f"seed {seed}: N {N} T {T} space {space} T_use {None if T_use is None else T_use.tolist()} "
          f"nan-cols {int(np.isnan(Y).any(axis=0).sum())} deferred {d1}/{d2} "
          f"repeat-equal one {np.array_equal(one, one_b, equal_nan=True)} two {np.array_equal(two, two_b, equal_nan=True)}")
    for b in range(Th.shape[1]):
        flag = "" if (one[b] == two[b] or (np.isnan(one[b]) and np.isnan(two[b]))) else "  <-- differ"
        print(f"  b {b:2d}: one {one[b]: .17e} two {two[b]: .17e} oracle {orc[b]: .17e} truth {tru[b]: .17e}{flag}")
