"""Generate the committed golden fixtures (tests/golden/*.npz) from the NumPy oracle.

    python tests/golden/make_golden.py

Inputs are seeded synthetic panels/batches (yfm_amd.synthetic); expected outputs
come from oracle/kalman_oracle.py — a line-by-line restatement of the reference
(parity unpinned against Julia itself: no julia here, no reference fixtures;
see oracle/kalman_oracle.py's header).  Each fixture stores the inputs and the
expected logliks (+ filtered-state trajectories for a few candidates).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))
sys.path.insert(0, str(ROOT))

from concurrent.futures import ProcessPoolExecutor  # noqa: E402

from oracle import kalman_mp as MP  # noqa: E402
from oracle import kalman_oracle as O  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402
from yfm_amd.params import KIND_DNS, KIND_GNS, KIND_TVL, param_layout, state_dim  # noqa: E402

OUT = Path(__file__).resolve().parent


def run(kind, Y, mats, Th, space=0, T_use=None, n_traj=0):
    M = state_dim(kind)
    B = Th.shape[1]
    ll = np.empty(B)
    trajs_b, trajs_P = [], []
    for b in range(B):
        Yb = Y if T_use is None else Y[:, :T_use[b]]
        rec = [] if b < n_traj else None
        ll[b] = O.loglik(kind, mats, M, Yb, Th[:, b], space=space, record=rec)
        if rec is not None:
            trajs_b.append(np.stack([r[0] for r in rec], axis=1))
            trajs_P.append(np.stack([r[1] for r in rec], axis=2))
    d = dict(kind=kind, space=space, Y=np.asfortranarray(Y), maturities=mats, Theta=np.asfortranarray(Th), loglik=ll)
    if T_use is not None:
        d["T_use"] = np.asarray(T_use, dtype=np.int32)
    if n_traj:
        d["beta_traj"] = np.stack(trajs_b, axis=-1)  # M × (T-1) × n
        d["P_traj"] = np.stack(trajs_P, axis=-1)  # M × M × (T-1) × n
        # 40-digit ground truth of the same recursion on the same FP64 inputs (oracle/kalman_mp.py)
        with ProcessPoolExecutor(max_workers=min(n_traj, 6)) as ex:
            futs = [ex.submit(MP.loglik_mp, kind, mats, Y, Th[:, b], space) for b in range(n_traj)]
            truth = [f.result() for f in futs]
        d["ll_truth"] = np.array([t[0] for t in truth])
        d["beta_truth"] = np.stack([t[1] for t in truth], axis=-1)
        d["P_truth"] = np.stack([t[2] for t in truth], axis=-1)
    return d


def main():
    mats30 = S.maturities_30()
    fixtures = {}

    # 1. DNS on the headline panel shape (N = 30), T = 160, 24 candidates incl. non-stationary Φ
    Y = S.simulate_panel(KIND_DNS, 600)[:, :160].copy(order="F")
    Th = S.theta_batch(KIND_DNS, 24, seed=11, bad_frac=0.125)
    Th[:, 0] = S.theta0(KIND_DNS)
    fixtures["dns_basic"] = run(KIND_DNS, Y, mats30, Th, n_traj=3)

    # 2. DNS, constrained space (set_params! input) incl. a Φ with an exact unit root (reference throws)
    tc = np.stack([S.theta0_constrained(KIND_DNS)] * 4, axis=1)
    lay = param_layout(KIND_DNS)
    tc[lay.phi_offset:lay.phi_offset + 9, 1] = np.diag([1.0, 0.9, 0.8]).reshape(-1)  # I-Φ singular -> NaN
    tc[lay.base_offset, 2] = 0.05  # larger σ²
    tc[lay.phi_offset:lay.phi_offset + 9, 3] = 0.0  # Φ = 0: iid innovations
    fixtures["dns_constrained"] = run(KIND_DNS, Y[:, :60], mats30, tc, space=1, n_traj=1)

    # 3. DNS with NaN columns (prediction-only steps; stale F/v re-added) incl. leading NaNs
    Yn = Y[:, :80].copy(order="F")
    Yn[:, [7, 8, 40]] = np.nan
    Yn[3, 60] = np.nan
    Th3 = S.theta_batch(KIND_DNS, 8, seed=13, bad_frac=0.0)
    fixtures["dns_nan_cols"] = run(KIND_DNS, Yn, mats30, Th3, n_traj=2)
    Yl = Y[:, :30].copy(order="F")
    Yl[:, [0, 1]] = np.nan  # NaN at t=1 and t=2: stale zero F -> -Inf
    fixtures["dns_leading_nan"] = run(KIND_DNS, Yl, mats30, Th3[:, :4])

    # 4. DNS expanding windows (T_use), including the degenerate T_use = 1, 2
    Th4 = S.theta_batch(KIND_DNS, 12, seed=17, bad_frac=0.0)
    tu = np.array([1, 2, 3, 10, 50, 99, 100, 100, 64, 65, 33, 77], dtype=np.int32)
    fixtures["dns_windows"] = run(KIND_DNS, Y[:, :100], mats30, Th4, T_use=tu)

    # 5. DNS with an odd maturity count (padding path) N = 7
    m7 = mats30[[0, 3, 7, 11, 17, 24, 29]].copy()
    Y7 = Y[[0, 3, 7, 11, 17, 24, 29], :90].copy(order="F")
    fixtures["dns_n7"] = run(KIND_DNS, Y7, m7, S.theta_batch(KIND_DNS, 8, seed=19, bad_frac=0.0))

    # 6. 5-factor GNS extension (parity of the build's own restatement; not in the reference)
    Y5 = S.simulate_panel(KIND_GNS, 120)
    fixtures["gns5_basic"] = run(KIND_GNS, Y5, mats30, S.theta_batch(KIND_GNS, 8, seed=23, bad_frac=0.0), n_traj=1)

    # 7. TVλ EKF, N = 40 maturities 1..40, T = 80
    m40 = np.arange(1, 41, dtype=np.float64)
    Yt = S.simulate_panel(KIND_TVL, 80, maturities=m40)
    Tht = S.theta_batch(KIND_TVL, 8, seed=29, bad_frac=0.0, scale=0.02)
    Tht[:, 0] = S.theta0(KIND_TVL)
    fixtures["tvl_basic"] = run(KIND_TVL, Yt, m40, Tht, n_traj=1)

    # 8. Headline shape (T = 600, N = 30): four columns of the bench batch on which the
    #    reference's own dense FP64 arithmetic is far (up to 5e-6) from exact arithmetic,
    #    plus two benign ones; ll_truth is the 40-digit value (oracle/kalman_mp.py).
    Y600 = S.simulate_panel(KIND_DNS, 600)
    idx = [10283, 1679, 5390, 22413, 0, 1]
    Thh = np.asfortranarray(S.theta_batch(KIND_DNS, 65536)[:, idx])
    d = run(KIND_DNS, Y600, mats30, Thh)
    with ProcessPoolExecutor(max_workers=6) as ex:
        futs = [ex.submit(MP.loglik_mp, KIND_DNS, mats30, Y600, Thh[:, b], 0) for b in range(len(idx))]
        d["ll_truth"] = np.array([f.result()[0] for f in futs])
    d["bench_index"] = np.asarray(idx)
    fixtures["dns_hard_T600"] = d

    for name, d in fixtures.items():
        np.savez_compressed(OUT / f"{name}.npz", **d)
        print(name, d["loglik"])


if __name__ == "__main__":
    main()
