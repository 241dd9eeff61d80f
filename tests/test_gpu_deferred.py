"""The deferred lanes of the fixed-loading models: candidates whose loading Gram
matrix Z'Z is ill-conditioned (κ₁ ≥ 1e6), singular, or has fewer maturities than states leave the
FP64 collapsed form and run the double-double capacitance kernel (yfm_fixedz_dd.hip).

* the deferral count (yfm_last_batch_deferred) equals the host's count of such candidates;
* every deferred candidate is checked against the dense FP64 oracle and adjudicated at factor 1 by
  the binary128 truth — GNS5 with near-equal λ₁, λ₂ (|γ₁ − γ₂| from 1e-9 to 1e-2: the collinear
  regime a random sample of config 5 misses) at the config-5 shape (N = 30, T = 600), DNS with λ so
  large the slope and curvature loadings coincide, and the rank-deficient N < M panels;
* with the |ll| denominator: within 1e-9 of the oracle or at least as close to the truth.
References: filter.jl:125-209, dns.jl:51-65.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

from oracle.truth import loglik_oracle, loglik_truth
from test_gpu_parity import assert_parity
from yfm_amd import KIND_DNS, KIND_GNS
from yfm_amd import synthetic as S
from yfm_amd.params import param_layout, state_dim, transform_params

pytestmark = pytest.mark.gpu


def kappa1(kind, Th, mats):
    """κ₁(Z'Z) per candidate (host FP64; the kernels compute the same with an in-register solve)."""
    lead = 2 if kind == KIND_GNS else 1
    N, B = len(mats), Th.shape[1]
    cols = [np.ones((B, N))]
    for g in Th[:lead]:
        lam = 0.01 + np.exp(g)[:, None]
        tau = lam * mats[None]
        z = np.exp(-tau)
        s = (1 - z) / tau
        cols += [s, s - z]
    Z = np.stack(cols, axis=2)
    G = np.einsum("bni,bnj->bij", Z, Z)
    k = np.full(B, np.inf)
    for b in range(B):  # an explicit inverse, as the kernels take (pinv would truncate and under-report)
        try:
            Gi = np.linalg.inv(G[b])
        except np.linalg.LinAlgError:
            continue
        k[b] = np.abs(G[b]).sum(0).max() * np.abs(Gi).sum(0).max()
    return k


def near_equal_gns5(B, seed=5):
    """GNS5 candidates around θ₀ with γ₂ = γ₁ + ε, ε = ±10^-U(2, 9)."""
    rng = np.random.default_rng(seed)
    Th = S.theta_batch(KIND_GNS, B, seed=seed, bad_frac=0.0, scale=0.05)
    eps = np.sign(rng.standard_normal(B)) * 10.0 ** -rng.uniform(2, 9, B)
    Th[1] = Th[0] + eps
    return np.asfortranarray(Th)


def check(engine, kind, Y, mats, Th, what):
    engine.set_panel(Y, mats)
    t0 = time.perf_counter()
    got = engine.loglik(kind, Th)
    dt = time.perf_counter() - t0
    nd = engine.last_deferred()
    k = kappa1(kind, Th, mats)
    lo, hi = int((k >= 2e6).sum()), int((k >= 5e5).sum()) if len(mats) >= state_dim(kind) else Th.shape[1]
    assert lo <= nd <= hi, (what, nd, lo, hi)
    ora = loglik_oracle(kind, Y, mats, Th)
    tru = loglik_truth(kind, Y, mats, Th)
    table = assert_parity(got, ora, tru)
    fin = np.isfinite(ora) & np.isfinite(got)
    e_go = np.abs(got[fin] - ora[fin]) / np.abs(ora[fin])
    strict_bad = (e_go > 1e-9) & (np.abs(got[fin] - tru[fin]) > np.abs(ora[fin] - tru[fin]))
    assert not strict_bad.any(), (what, np.flatnonzero(strict_bad))
    print(what, f"B={Th.shape[1]} deferred={nd} call={1e3 * dt:.1f} ms", table)
    return nd


def test_gns5_near_equal_lambda_config5_shape(engine):
    mats = S.maturities_30()
    Y = S.simulate_panel(KIND_GNS, 600)
    Th = near_equal_gns5(256)
    nd = check(engine, KIND_GNS, Y, mats, Th, "GNS5 near-equal λ, N=30 T=600")
    assert nd >= 200  # the regime is deferred


def test_dns_collinear_loadings_config2_shape(engine):
    """λ = 0.01 + e^γ large: e^{−λm} ≈ 0 at every maturity, so C = S − e^{−λm} ≈ S (κ₁ ~ 1e8 … 1e16)."""
    mats = S.maturities_30()
    Y = S.simulate_panel(KIND_DNS, 600)
    Th = S.theta_batch(KIND_DNS, 128, seed=12, bad_frac=0.0, scale=0.05)
    Th[0] = np.linspace(0.5, 4.0, 128)
    nd = check(engine, KIND_DNS, Y, mats, np.asfortranarray(Th), "DNS large λ, N=30 T=600")
    assert nd >= 32


@pytest.mark.parametrize("kind,N", [(KIND_DNS, 1), (KIND_DNS, 2), (KIND_GNS, 1), (KIND_GNS, 3), (KIND_GNS, 4)])
def test_rank_deficient_panels(engine, kind, N):
    """N < M: Z'Z is singular, every candidate is deferred."""
    mats = np.array([3.0, 24.0, 60.0, 120.0][:N])
    Y = S.simulate_panel(kind, 120, maturities=mats)
    Th = S.theta_batch(kind, 64, seed=3 + N, bad_frac=0.05, scale=0.05)
    nd = check(engine, kind, Y, mats, Th, f"kind {kind} N={N} T=120")
    assert nd == 64


def test_deferred_trajectories(engine):
    """filter_states / predict of deferred candidates come from the double-double kernel: states vs
    the binary128 truth trajectory (GNS5, near-equal λ, T = 120)."""
    from oracle.truth import states_truth
    mats = S.maturities_30()
    Y = S.simulate_panel(KIND_GNS, 120)
    Th = near_equal_gns5(4, seed=9)
    engine.set_panel(Y, mats)
    ll, beta, P = engine.filter_states(KIND_GNS, Th)
    assert engine.last_deferred() == 4
    for b in range(4):
        llt, bt, Pt = states_truth(KIND_GNS, Y, mats, Th[:, b])
        assert abs(ll[b] - llt) <= 1e-13 * abs(llt)
        assert np.abs(beta[..., b] - bt).max() <= 1e-12 * np.abs(bt).max()
        assert np.abs(P[..., b] - Pt).max() <= 1e-12 * np.abs(Pt).max()
