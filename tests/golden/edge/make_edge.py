"""Generate tests/golden/edge/edge_cases.npz: the reference's numeric edge cases.

Each case stores its panel, maturities, Θ, param space and optional windows, with
  loglik_oracle — oracle/kalman_oracle.py (NumPy + LAPACK getrf/getri, the routines Julia calls),
  loglik_truth  — oracle/yfm_truth.c (binary128; where F is singular in exact arithmetic — σ² = 0
                  with N > M, or F = 0 — the exact answer is get_loss's −Inf).

  small_sigma_dns / _tvl / _gns  σ² ∈ {1e-6, 1e-8}: κ(F) = 1e8..1e11, the dense inverse loses
                                 digits (SURVEY §7 "Hard parts")
  sigma_underflow_dns            unconstrained θ[σ²] = −800 ⇒ σ² = exp(−800) = 0 in FP64
  sigma_zero_dns                 constrained σ² = 0
  F_zero_dns / F_zero_tvl        constrained σ² = 0 and U = 0 ⇒ Q = P₀ = 0 ⇒ F = 0: inv(F) throws —
                                 DNS sets F⁻¹ = Inf (filter.jl:149-155), TVλ leaves it stale
                                 (:51-56); both skip the update; T_use = 2 gives get_loss's 0.0

    python tests/golden/edge/make_edge.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]

from oracle import kalman_oracle as O  # noqa: E402
from oracle.truth import loglik_truth  # noqa: E402
from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402
from yfm_amd.params import param_layout, state_dim, transform_params  # noqa: E402


def oracle(kind, Y, mats, Th, space, T_use=None):
    out = []
    for b in range(Th.shape[1]):
        Yb = Y if T_use is None else Y[:, :T_use[b]]
        out.append(O.loglik(kind, mats, state_dim(kind), Yb, Th[:, b], space=space))
    return np.array(out)


def cases():
    m30 = S.maturities_30()
    Yd = S.simulate_panel(KIND_DNS, 600)
    Yg = S.simulate_panel(KIND_GNS, 300)
    Yt = S.simulate_panel(KIND_TVL, 200, maturities=m30)
    for kind, Y, name in ((KIND_DNS, Yd, "small_sigma_dns"), (KIND_TVL, Yt, "small_sigma_tvl"),
                          (KIND_GNS, Yg, "small_sigma_gns")):
        lay = param_layout(kind)
        Th = S.theta_batch(kind, 8, seed=101, bad_frac=0.0, scale=0.02 if kind == KIND_TVL else 0.05)
        Th[lay.base_offset, :4] = np.log(1e-6)
        Th[lay.base_offset, 4:] = np.log(1e-8)
        yield name, kind, Y, m30, Th, 0, None
    lay = param_layout(KIND_DNS)
    Th = S.theta_batch(KIND_DNS, 4, seed=103, bad_frac=0.0, scale=0.05)
    Th[lay.base_offset, :] = -800.0
    yield "sigma_underflow_dns", KIND_DNS, Yd[:, :120], m30, Th, 0, None
    Tc = transform_params(KIND_DNS, S.theta_batch(KIND_DNS, 4, seed=105, bad_frac=0.0, scale=0.05))
    Tc[lay.base_offset, :] = 0.0
    yield "sigma_zero_dns", KIND_DNS, Yd[:, :120], m30, Tc, 1, None
    for kind, Y, name in ((KIND_DNS, Yd[:, :60], "F_zero_dns"), (KIND_TVL, Yt[:, :60], "F_zero_tvl")):
        lay = param_layout(kind)
        M = state_dim(kind)
        Tc = np.repeat(S.theta0_constrained(kind)[:, None], 3, axis=1)
        Tc[lay.base_offset:lay.base_offset + 1 + M * (M + 1) // 2, :] = 0.0  # σ² = 0, U = 0
        yield name, kind, Y, m30, Tc, 1, np.array([60, 2, 3], dtype=np.int32)


def main():
    arrays = {}
    names = []
    for name, kind, Y, mats, Th, space, tu in cases():
        ora = oracle(kind, Y, mats, Th, space, tu)
        tru = loglik_truth(kind, Y, mats, Th, space=space, T_use=tu)
        names.append(name)
        arrays.update({f"{name}/kind": np.int32(kind), f"{name}/Y": Y, f"{name}/maturities": mats,
                       f"{name}/Theta": Th, f"{name}/space": np.int32(space), f"{name}/loglik_oracle": ora,
                       f"{name}/loglik_truth": tru})
        if tu is not None:
            arrays[f"{name}/T_use"] = tu
        fin = np.isfinite(tru) & np.isfinite(ora)
        e = np.abs(ora[fin] - tru[fin]) / np.abs(tru[fin]) if fin.any() else np.zeros(0)
        print(f"{name:22s} oracle {np.array2string(ora, precision=6)}\n{'':22s} truth  {np.array2string(tru, precision=6)}"
              f"  max rel {e.max() if e.size else 0:.2e}")
    arrays["names"] = np.array(names)
    np.savez_compressed(Path(__file__).parent / "edge_cases.npz", **arrays)


if __name__ == "__main__":
    main()
