"""Which (θ, window) of bench config 4 moves most between the steady state and the full recursion?
Prints the worst candidates with the dense oracle and the binary128 truth beside both GPU values.

    python tools/dbg_c4_steady.py [--top 8]
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]
import torch  # noqa: E402,F401
from oracle.truth import loglik_oracle, loglik_truth  # noqa: E402
from yfm_amd import KIND_DNS, get_engine  # noqa: E402
from yfm_amd import params as PR  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--top", type=int, default=8)
a = ap.parse_args()
eng = get_engine(0)
T, per = 600, 4096
wins = np.arange(361, 601)
Th_all = S.theta_batch(KIND_DNS, per, seed=S.BATCH_SEED)
Th = np.asfortranarray(np.tile(Th_all, (1, len(wins))))
tu = np.repeat(wins, per).astype(np.int32)
mats = S.maturities_30()
Y = S.simulate_panel(KIND_DNS, T)
eng.set_panel(Y, mats)
st = eng.loglik(KIND_DNS, Th, space=0, T_use=tu)
os.environ["YFM_DNS_STEADY"] = "0"
fu = eng.loglik(KIND_DNS, Th, space=0, T_use=tu)
os.environ.pop("YFM_DNS_STEADY")
fin = np.isfinite(fu) & np.isfinite(st)
d = np.zeros(len(fu))
d[fin] = np.abs(st[fin] - fu[fin]) / np.abs(fu[fin])
print(f"max rel {d.max():.3e}; > 1e-12: {(d > 1e-12).sum()} of {fin.sum()} finite; "
      f"distinct θ among them {len(set((np.flatnonzero(d > 1e-12) % per).tolist()))}")
top = np.argsort(-d)[:a.top]
sub = np.asfortranarray(Th[:, top])
orc = loglik_oracle(KIND_DNS, Y, mats, sub, T_use=tu[top])
tru = loglik_truth(KIND_DNS, Y, mats, sub, T_use=tu[top])
lay = PR.param_layout(KIND_DNS)
thc = PR.transform_params(KIND_DNS, sub)
for i, k in enumerate(top):
    phi = thc[lay.phi_offset:lay.phi_offset + 9, i].reshape(3, 3)
    e = lambda x: abs(x - tru[i]) / abs(tru[i])  # noqa: E731
    print(f"θ {k % per:4d} window {tu[k]}: steady-full {d[k]:.2e}  steady-truth {e(st[k]):.2e}  full-truth {e(fu[k]):.2e}  "
          f"oracle-truth {e(orc[i]):.2e}  ll {tru[i]:.6e}  σ² {thc[lay.base_offset, i]:.3e}  "
          f"|eig Φ| {np.abs(np.linalg.eigvals(phi)).max():.4f}")
