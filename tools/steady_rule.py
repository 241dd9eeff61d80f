"""CPU model of the frozen-covariance steady state (yfm_fixedz.hpp FixedZFilter) and its freeze rule.

Runs the collapsed-form filter vectorised over a batch of candidates in numpy FP64
twice — the full recursion, and with each lane's P frozen by a freeze rule — and reports per regime:
the freeze step quantiles, the share of filter steps a 64-lane wave would run steady, the largest
loglik change against the full recursion, and the largest ratio of that change to the first-order
bound of DESIGN.md §3.1 (the bound must hold: ratio ≤ 1).

Rules:
  r3        round 3: d ≤ 2^-46 and d·ρ/(1−ρ) ≤ 2^-50, ρ = d_t/d_{t−1} (one ratio)
  contract  round 4: d = 0, or d ≤ 2^-46 and M·d·C ≤ 2^-50 with C = Σ_{k≥1} ‖A^k‖_F² bounded from
            A = Φ R S⁻¹ (the closed-loop matrix; exact Riccati difference identity
            P_{t+2} − P_{t+1} = A_{t+1} (P_{t+1} − P_t) A_t')
  gain      round 5 (the kernel's rule): contract at 2^-52, and the loglik's sensitivity
            max(1, C₁)·‖P‖_∞‖S⁻¹‖_∞ ≤ 512 with C₁ = Σ_{k≥1} ‖A^k‖_∞ (else only d = 0 freezes) — a frozen P's
            rounding-level error moves c'S⁻¹c by ‖ΔP‖‖S⁻¹‖ and the filtered mean by C₁‖ΔK‖
            (yfm_fixedz.hpp contraction_bound)

    python tools/steady_rule.py [--B 4096] [--T 600]
"""
from __future__ import annotations

import argparse
import math
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]
from yfm_amd import KIND_DNS, KIND_GNS  # noqa: E402
from yfm_amd import params as PR  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

LOG2PI = math.log(2 * math.pi)


def decode(kind, Thc):
    """constrained θ (P×B) → (γ (L×B), σ² (B), Q, δ, Φ)."""
    lay = PR.param_layout(kind)
    M, B = lay.M, Thc.shape[1]
    g = Thc[:lay.n_lead]
    s2 = Thc[lay.base_offset]
    U = np.zeros((B, M, M))
    k = lay.u_offset
    for j in range(M):
        for i in range(j + 1):
            U[:, i, j] = Thc[k]
            k += 1
    Q = np.einsum("bli,blj->bij", U, U)
    dl = Thc[lay.delta_offset:lay.delta_offset + M].T
    Phi = Thc[lay.phi_offset:lay.phi_offset + M * M].T.reshape(B, M, M)
    return g, s2, Q, dl, Phi


def loadings(g, mats):
    B = g.shape[1]
    cols = [np.ones((B, len(mats)))]
    for l in range(g.shape[0]):
        lam = (0.01 + np.exp(g[l]))[:, None]
        tau = lam * mats[None]
        z = np.exp(-tau)
        s = (1 - z) / tau
        cols += [s, s - z]
    return np.stack(cols, 2)  # B, N, M


def contraction_C(Phi, R, Sm, M, P=None, cap=None):
    """Upper bound of Σ_{k≥1} ‖A^k‖_∞² for A = Φ R S⁻¹ (inf where ‖A⁴‖_∞ ≥ 1), as the device's
    contraction_bound (yfm_fixedz.hpp) with its 1.01 rounding margin; with `cap`, also inf where the
    loglik sensitivity max(1, C₁)‖P‖_∞‖S⁻¹‖_∞ exceeds it (C₁ = Σ_{k≥1} ‖A^k‖_∞)."""
    A = Phi @ np.swapaxes(np.linalg.solve(Sm, R), 1, 2)  # R S⁻¹ = (S⁻¹R)'
    A2 = A @ A
    A3 = A2 @ A
    A4 = A2 @ A2
    r = [np.max(np.sum(np.abs(X), axis=2), axis=1) for X in (A, A2, A3, A4)]
    n = [x ** 2 for x in r]
    with np.errstate(divide="ignore", invalid="ignore"):
        C = np.where(n[3] < 1.0, 1.01 * (n[0] + n[1] + n[2] + n[3]) / (1.0 - n[3]), np.inf)
        if cap is not None:
            c1 = 1.01 * (r[0] + r[1] + r[2] + r[3]) / (1.0 - r[3])
            inf_norm = lambda X: np.max(np.sum(np.abs(X), axis=2), axis=1)  # noqa: E731
            gain = np.maximum(1.0, c1) * inf_norm(P) * inf_norm(np.linalg.inv(Sm))
            C = np.where(gain <= cap, C, np.inf)
    return C


def run(kind, Y, mats, Thc, rule=None, tau=2.0 ** -50):
    """Collapsed filter over every column of Y (loglik mode); rule None = full recursion."""
    M = PR.state_dim(kind)
    g, s2, Q, dl, Phi = decode(kind, Thc)
    B = Thc.shape[1]
    N, T = Y.shape
    Z = loadings(g, mats)
    G = np.einsum("bni,bnj->bij", Z, Z)
    # candidates whose Z'Z is ill-conditioned go to the kernel's double-double path, not the collapsed filter
    # modelled here (κ₁ ≥ 1e6, yfm_fixedz.hpp): their G is replaced by I and their results are NaN
    bad = ~(np.linalg.cond(G, 1) < 1e6)
    G = np.where(bad[:, None, None], np.eye(G.shape[1])[None], G)
    Gi = np.linalg.inv(G)
    R = s2[:, None, None] * Gi
    R = 0.5 * (R + np.swapaxes(R, 1, 2))
    beta = np.linalg.solve(np.eye(M)[None] - Phi, dl[:, :, None])[:, :, 0]
    K = np.eye(M * M)[None] - np.einsum("bij,bkl->bikjl", Phi, Phi).reshape(B, M * M, M * M)
    P = np.linalg.solve(K, Q.reshape(B, M * M, 1)).reshape(B, M, M)
    P = 0.5 * (P + np.swapaxes(P, 1, 2))
    frozen = np.zeros(B, bool)
    fstep = np.full(B, T, int)
    prevd = np.full(B, np.inf)
    ld = np.zeros(B)
    sq = np.zeros(B)
    ldG = np.linalg.slogdet(G)[1]
    drift_bound = np.zeros(B)  # M·d·C at the freeze (relative P drift bound)
    sens = np.zeros(B)  # Σ_t terms of the loglik bound
    for t in range(T - 1):
        y = Y[:, t]
        ZtY = np.einsum("bni,n->bi", Z, y)
        ch = np.einsum("bij,bj->bi", Gi, ZtY)
        rr = y @ y - np.einsum("bi,bi->b", ZtY, ch)
        c = ch - beta
        Sm = P + R
        x = np.linalg.solve(Sm, c[:, :, None])[:, :, 0]
        q = rr / s2 + np.einsum("bi,bi->b", c, x)
        if t >= 1:
            ld += np.linalg.slogdet(Sm)[1]
            sq += q
            if rule is not None:
                # loglik bound terms for frozen lanes: ½‖S⁻¹‖(M + q_t)‖δP‖ + β-path term (bounded below)
                Si = np.linalg.inv(Sm)
                ns = np.sqrt(np.sum(Si * Si, axis=(1, 2)))
                sens += np.where(frozen, 0.5 * ns * (M + np.einsum("bi,bi->b", c, x)), 0.0)
        bf = beta + np.einsum("bij,bj->bi", P, x)
        Pf = P @ np.linalg.solve(Sm, R)
        beta = dl + np.einsum("bij,bj->bi", Phi, bf)
        Pn = Phi @ Pf @ np.swapaxes(Phi, 1, 2) + Q
        Pn = 0.5 * (Pn + np.swapaxes(Pn, 1, 2))
        if rule is None:
            P = Pn
            continue
        nmax = np.max(np.abs(Pn), axis=(1, 2))
        d = np.max(np.abs(Pn - P), axis=(1, 2)) / nmax
        P = np.where(frozen[:, None, None], P, Pn)
        if rule == "r3":
            with np.errstate(divide="ignore", invalid="ignore"):
                rho = d / prevd
                ok = (d <= 2.0 ** -46) & (rho < 0.999) & (d * rho <= tau * (1 - rho))
            db = np.where(ok, d * rho / np.maximum(1 - rho, 1e-300), 0)
        else:
            cap = 512.0 if rule == "gain" else None
            C = 2.0 * contraction_C(Phi, R, P + R, M, P, cap)  # the device's 2C (first-order margin)
            ok = (d == 0) | ((d <= 2.0 ** -46) & (d * C <= tau))
            db = np.where(d == 0, 0.0, d * C)
        newf = ok & ~frozen
        drift_bound = np.where(newf, db, drift_bound)
        fstep[newf] = t + 1
        prevd = np.where(frozen, prevd, d)
        frozen |= ok
    nterms = T - 2
    per = (N - M) * np.log(s2) + ldG + N * LOG2PI
    ll = -0.5 * (nterms * per + ld + sq)
    ll = np.where(bad, np.nan, ll)  # deferred to the double-double kernel
    return ll, fstep, drift_bound, sens


def regimes(kind, B, rng):
    """name → constrained θ batch (P×B)."""
    lay = PR.param_layout(kind)
    M = lay.M
    out = {}
    base = S.theta_batch(kind, B, seed=S.BATCH_SEED, bad_frac=0.0)
    out["config (θ₀ ± 0.1)"] = PR.transform_params(kind, base)
    out["wide (θ₀ ± 0.3)"] = PR.transform_params(kind, S.theta_batch(kind, B, seed=11, bad_frac=0.0, scale=0.3))
    out["scale 1.0 (explosive Φ among them)"] = PR.transform_params(kind, S.theta_batch(kind, B, seed=15, bad_frac=0.02,
                                                                                         scale=1.0))
    th = PR.transform_params(kind, S.theta_batch(kind, B, seed=12, bad_frac=0.0))
    th[lay.base_offset] = 10.0 ** rng.uniform(-6, -3, B)
    out["small σ² (1e-6..1e-3)"] = th
    th = PR.transform_params(kind, S.theta_batch(kind, B, seed=13, bad_frac=0.0))
    ph = th[lay.phi_offset:lay.phi_offset + M * M].reshape(M, M, B)
    for i in range(M):
        ph[i, i] = 1.0 - 10.0 ** rng.uniform(-3.5, -2, B)
    th[lay.phi_offset:lay.phi_offset + M * M] = ph.reshape(M * M, B)
    th[lay.base_offset] = 10.0 ** rng.uniform(-2, 0.5, B)  # large σ²: slow gain convergence
    out["near unit root, large σ²"] = th
    th = PR.transform_params(kind, S.theta_batch(kind, B, seed=14, bad_frac=0.0))
    r = rng.uniform(0.8, 0.99, B)
    w = rng.uniform(0.2, 1.2, B)
    ph = np.zeros((M, M, B))
    for i in range(M):
        ph[i, i] = 0.9
    ph[0, 0] = ph[1, 1] = r * np.cos(w)
    ph[0, 1] = -r * np.sin(w)
    ph[1, 0] = r * np.sin(w)
    th[lay.phi_offset:lay.phi_offset + M * M] = ph.reshape(M * M, B)
    th[lay.base_offset] = 10.0 ** rng.uniform(-2, 0.5, B)
    out["complex-eigenvalue Φ"] = th
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--T", type=int, default=600)
    ap.add_argument("--kind", type=int, default=KIND_DNS)
    ap.add_argument("--rules", default="contract,gain")
    ap.add_argument("--taus", default="52", help="comma list of k: freeze when d·2C ≤ 2^-k (contract, gain rules)")
    a = ap.parse_args()
    kind = a.kind
    mats = S.maturities_30()
    Y = S.simulate_panel(kind, a.T, maturities=mats)
    rng = np.random.default_rng(3)
    for name, Thc in regimes(kind, a.B, rng).items():
        full, *_ = run(kind, Y, mats, Thc)
        fin = np.isfinite(full)
        print(f"== {name}: {fin.sum()} finite of {a.B}")
        for rule, k in [(r, k) for r in a.rules.split(",") for k in (a.taus.split(",") if r in ("contract", "gain") else ["50"])]:
            ll, fs, db, sens = run(kind, Y, mats, Thc, rule, 2.0 ** -int(k))
            rule = f"{rule}{k}" if rule in ("contract", "gain") else rule
            e = np.abs(ll[fin] - full[fin])
            rel = e / np.abs(full[fin])
            w = fs[: (a.B // 64) * 64].reshape(-1, 64).max(1)
            share = np.mean(np.maximum(a.T - 1 - w, 0)) / (a.T - 1)
            # first-order bound: Σ_t ½‖S⁻¹‖_F (M + q_t) ‖δP‖_F with ‖δP‖_F ≤ drift_bound·nmax — reported as
            # the bound's ratio to the measured change
            print(f"  {rule:8s} freeze step q50/q90/max {np.quantile(fs, 0.5):6.0f} {np.quantile(fs, 0.9):6.0f} "
                  f"{fs.max():5d}  wave steady share {share:.3f}  max rel vs full {rel.max():.2e}  "
                  f"max drift bound {db[fin].max():.2e}")


if __name__ == "__main__":
    main()
