"""Generate tests/golden/states/*.npz: filtered-state and predict trajectories at the BASELINE
configuration shapes, with binary128 truth (VERDICT r2 "what's missing" 1).

    python tests/golden/states/make_states_golden.py        (≈ 3 min on 8 cores; TVλ dominates)

Per fixture, 8 candidates θ (unconstrained, param_space 0) on the workload's own panel (regenerated
from its seed, yfm_amd.synthetic.simulate_panel — not stored):

* dns_c2   config 2: DNS, N = 30, T = 600 — 7 finite candidates of the bench batch (seed BATCH_SEED)
           plus a near-unit-root one (θ₀ with Φ₁₁ = 0.9995, constrained);
* gns5_c5  config 5: GNS5, N = 30, T = 600 — 8 finite candidates of the global search stream;
* tvl_c3   config 3: TVλ, N = 360, T = 600 — the first 8 candidates of the bench batch (the
           tests/golden/config3 sample).

Stored (P upper triangles packed row-major, i ≤ k):
  ll_{truth,oracle}          get_loss (filter.jl:182-209)
  beta_{truth,oracle}        M × (T−1) × B: a_{t+1|t} after filter! call t = 1..T−1 (filter.jl:125-179, :12-80)
  Pu_{truth,oracle}          U × (T−1) × B: the same P_{t+1|t}
  A_{truth,oracle}           M × (T+1) × B: predict's state trajectory (filter.jl:250-282, horizon 1):
                             A[:, j] = β after filter! step j+1 of hcat(Y, NaN), the final NaN step included
truth = oracle/yfm_truth.c (binary128, pinned to the 40-digit dense restatement); oracle =
oracle/yfm_oracle.c (the dense FP64 restatement: getrf+getri and a logdet LU every step).
"""
from __future__ import annotations

import sys
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]

OUT = Path(__file__).resolve().parent


def _states(lib_name, kind, Y, mats, theta):
    import ctypes
    from oracle.truth import _lib
    from yfm_amd.params import state_dim
    D = ctypes.POINTER(ctypes.c_double)
    M = state_dim(kind)
    Y = np.asfortranarray(Y, dtype=np.float64)
    N, T = Y.shape
    th = np.ascontiguousarray(theta, dtype=np.float64)
    mats = np.ascontiguousarray(mats, dtype=np.float64)
    beta = np.zeros((M, T - 1), order="F")
    P = np.zeros((M, M, T - 1), order="F")
    ll = ctypes.c_double()
    fn = getattr(_lib(lib_name), f"{lib_name}_filter_states")
    fn(kind, 0, Y.ctypes.data_as(D), N, T, mats.ctypes.data_as(D), th.ctypes.data_as(D), beta.ctypes.data_as(D),
       P.ctypes.data_as(D), ctypes.byref(ll))
    return ll.value, beta, P


def one(args):
    """(ll, β, P_upper, A) from the truth and the oracle for one candidate."""
    kind, Y, mats, theta = args
    M = beta_dim = None
    out = {}
    pad = np.hstack([Y, np.full((Y.shape[0], 2), np.nan)])  # predict, horizon 1: hcat(Y, NaN) + final NaN step
    for tag, lib in (("truth", "yfm_truth"), ("oracle", "yfm_oracle")):
        ll, beta, P = _states(lib, kind, Y, mats, theta)
        M = beta.shape[0]
        iu = np.triu_indices(M)
        _, A, _ = _states(lib, kind, pad, mats, theta)
        out[tag] = (ll, beta, P[iu[0], iu[1], :], A)
    return out


def build(name, kind, Y, mats, Theta, note):
    B = Theta.shape[1]
    with ProcessPoolExecutor(max_workers=8) as ex:
        res = list(ex.map(one, [(kind, Y, mats, Theta[:, b]) for b in range(B)]))
    d = dict(kind=kind, Theta=np.asfortranarray(Theta), note=note, T=Y.shape[1], N=Y.shape[0])
    for tag in ("truth", "oracle"):
        d[f"ll_{tag}"] = np.array([r[tag][0] for r in res])
        d[f"beta_{tag}"] = np.stack([r[tag][1] for r in res], axis=-1)
        d[f"Pu_{tag}"] = np.stack([r[tag][2] for r in res], axis=-1)
        d[f"A_{tag}"] = np.stack([r[tag][3] for r in res], axis=-1)
    np.savez_compressed(OUT / f"{name}.npz", **d)
    e = np.abs(d["ll_oracle"] - d["ll_truth"]) / np.abs(d["ll_truth"])
    print(name, "ll oracle vs truth max rel", e.max(), flush=True)


def finite_picks(kind, Y, mats, Th, k):
    from oracle.truth import loglik_truth
    ll = loglik_truth(kind, Y, mats, Th)
    idx = np.flatnonzero(np.isfinite(ll))
    return idx[np.linspace(0, len(idx) - 1, k).astype(int)]


def main():
    from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL
    from yfm_amd import synthetic as S
    from yfm_amd.params import param_layout, untransform_params

    mats30 = S.maturities_30()
    # config 2: DNS
    Y = S.simulate_panel(KIND_DNS, 600)
    Thb = S.theta_batch(KIND_DNS, 65536)
    cand = np.asfortranarray(Thb[:, ::4096])  # 16 spread over the bench batch
    pick = finite_picks(KIND_DNS, Y, mats30, cand, 7)
    tc = S.theta0_constrained(KIND_DNS).copy()
    tc[param_layout(KIND_DNS).phi_offset] = 0.9995  # near-unit-root level factor
    Th = np.column_stack([cand[:, pick], untransform_params(KIND_DNS, tc)])
    build("dns_c2", KIND_DNS, Y, mats30, Th, "config 2 bench batch columns " + str(list(pick * 4096)) +
          " + theta0 with Phi11 = 0.9995")
    # config 5: GNS5
    Y5 = S.simulate_panel(KIND_GNS, 600)
    cand5 = np.column_stack([S.theta_range(KIND_GNS, i, i + 1, scale=0.1)[:, 0] for i in range(0, 1 << 20, 1 << 16)])
    pick5 = finite_picks(KIND_GNS, Y5, mats30, cand5, 8)
    build("gns5_c5", KIND_GNS, Y5, mats30, cand5[:, pick5], "config 5 global indices " + str(list(pick5 << 16)))
    # config 3: TVλ
    m360 = S.maturities_360()
    Y3 = S.simulate_panel(KIND_TVL, 600, maturities=m360)
    Th3 = np.asfortranarray(S.theta_batch(KIND_TVL, 16384, seed=S.BATCH_SEED, bad_frac=0.0, scale=0.02)[:, :8])
    build("tvl_c3", KIND_TVL, Y3, m360, Th3, "config 3 bench batch columns 0..7")


if __name__ == "__main__":
    main()
