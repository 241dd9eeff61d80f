"""Diagnose one case of tests/test_gpu_steady_sweep.py: per candidate the steady and full-recursion logliks,
the dense FP64 oracle and the binary128 truth, for the candidates where steady and full differ most.

    python tools/dbg_sweep_case.py <case> [case ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "yieldfactormodels.jl_amd"), ROOT]
import torch  # noqa: E402,F401
from oracle.truth import loglik_oracle, loglik_truth  # noqa: E402
from test_gpu_steady_sweep import CASES, make_case  # noqa: E402
from yfm_amd import get_engine  # noqa: E402
from yfm_amd import params as PR  # noqa: E402

eng = get_engine(0)
for case in [int(a) for a in sys.argv[1:]] or [9]:
    kind, T, reg, pattern, space = CASES[case]
    N, mats, Y, Th, T_use = make_case(kind, T, reg, pattern, space, 7000 + case)
    eng.set_panel(Y, mats)
    os.environ["YFM_GNS5_STEADY"] = "1"
    got = eng.loglik(kind, Th, space=space, T_use=T_use)
    os.environ["YFM_DNS_STEADY"] = "0"
    ref = eng.loglik(kind, Th, space=space, T_use=T_use)
    os.environ.pop("YFM_DNS_STEADY")
    os.environ.pop("YFM_GNS5_STEADY")
    orc = loglik_oracle(kind, Y, mats, Th, space=space, T_use=T_use)
    tru = loglik_truth(kind, Y, mats, Th, space=space, T_use=T_use)
    fin = np.isfinite(ref) & np.isfinite(got)
    d = np.zeros_like(got)
    d[fin] = np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])
    print(f"case {case}: kind {kind} T {T} N {N} {reg} {pattern} space {space}")
    thc = Th if space == 1 else PR.transform_params(kind, Th)
    lay = PR.param_layout(kind)
    for b in np.argsort(-d)[:8]:
        M = lay.M
        phi = thc[lay.phi_offset:lay.phi_offset + M * M, b].reshape(M, M)
        ev = np.abs(np.linalg.eigvals(phi))
        e = lambda x: abs(x - tru[b]) / abs(tru[b])  # noqa: E731
        print(f"  b {b:3d}: steady-full {d[b]:.2e}  |steady-truth| {e(got[b]):.2e}  |full-truth| {e(ref[b]):.2e}  "
              f"|oracle-truth| {e(orc[b]):.2e}  |oracle-full| {abs(orc[b]-ref[b])/abs(tru[b]):.2e}  "
              f"sigma2 {thc[lay.base_offset, b]:.3e}  |eig Phi| max {ev.max():.4f}  ll {tru[b]:.6e}")
