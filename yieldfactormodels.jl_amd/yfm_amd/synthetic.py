"""Seeded synthetic workloads for the benchmark configs.

The reference's data (``thread_id__<id>__data.csv``, N×T, read by
``src/utils/data_management.jl:1-5``) must be downloaded and is not in the
repository, so every panel here is simulated from the model itself.

Layout conventions follow the reference: a panel is N×T (rows = maturities,
columns = months), stored column-major (Fortran order) like Julia's
``Matrix{Float64}``; a parameter batch Θ is P×B column-major, i.e. one
candidate θ_b is contiguous (``Theta[:, b]``).
"""
from __future__ import annotations

import math

import numpy as np

from .params import (KIND_DNS, KIND_GNS, KIND_TVL, n_params, param_layout,
                     untransform_params)

PANEL_SEED = 20260227
BATCH_SEED = 20260228


def maturities_30() -> np.ndarray:
    """3,6,9,12,18,24,30,36, 48..240 step 12, 264..360 step 24 (months) — N = 30."""
    m = [3, 6, 9, 12, 18, 24, 30, 36] + list(range(48, 241, 12)) + [264, 288, 312, 336, 360]
    assert len(m) == 30
    return np.asarray(m, dtype=np.float64)


def maturities_360() -> np.ndarray:
    return np.arange(1, 361, dtype=np.float64)


def theta0_constrained(kind: int = KIND_DNS) -> np.ndarray:
    """θ₀ in the constrained space (as ``set_params!`` consumes it)."""
    if kind == KIND_DNS:
        M = 3
        lead = [math.log(0.0609 - 0.01)]
    elif kind == KIND_GNS:
        M = 5
        lead = [math.log(0.0609 - 0.01), math.log(0.30 - 0.01)]
    elif kind == KIND_TVL:
        M = 4
        lead = []
    else:
        raise ValueError(kind)
    sigma2 = 0.10 ** 2
    if M == 3:
        phi = np.array([[0.99, 0.02, -0.02],
                        [0.02, 0.95, 0.02],
                        [-0.02, 0.02, 0.90]])
        mu = np.array([5.0, -1.5, 0.5])
        udiag = [0.30, 0.40, 0.60]
    elif M == 4:  # TVλ: 4th state is a = log(λ - 0.01)
        phi = np.array([[0.99, 0.02, -0.02, 0.0],
                        [0.02, 0.95, 0.02, 0.0],
                        [-0.02, 0.02, 0.90, 0.0],
                        [0.0, 0.0, 0.0, 0.97]])
        mu = np.array([5.0, -1.5, 0.5, math.log(0.0509)])
        udiag = [0.30, 0.40, 0.60, 0.10]
    else:
        phi = np.diag([0.99, 0.95, 0.90, 0.93, 0.88])
        phi[0, 1] = phi[1, 0] = 0.02
        mu = np.array([5.0, -1.5, 0.5, 0.3, -0.2])
        udiag = [0.30, 0.40, 0.60, 0.50, 0.50]
    U = np.diag(udiag)
    for j in range(M):
        for i in range(j):
            U[i, j] = 0.05 if (i + j) % 2 else -0.03
    delta = (np.eye(M) - phi) @ mu
    ucol = [U[i, j] for j in range(M) for i in range(M) if i <= j]  # paramoperations.jl:18-33 order
    return np.asarray(lead + [sigma2] + ucol + list(delta) + list(phi.reshape(-1)), dtype=np.float64)


def theta0(kind: int = KIND_DNS) -> np.ndarray:
    """θ₀ in the unconstrained space (as ``compute_loss`` consumes it)."""
    return untransform_params(kind, theta0_constrained(kind))


def _decode(kind, tc, maturities):
    lay = param_layout(kind)
    M = lay.M
    U = np.zeros((M, M))
    k = lay.base_offset + 1
    for j in range(M):
        for i in range(j + 1):
            U[i, j] = tc[k]
            k += 1
    Q = U.T @ U
    delta = tc[k:k + M]
    k += M
    Phi = tc[k:k + M * M].reshape(M, M)
    sigma2 = tc[lay.base_offset]
    return M, sigma2, Q, delta, Phi


def _loadings(gammas, maturities, M):
    N = len(maturities)
    Z = np.ones((N, M))
    for b, g in enumerate(gammas):
        lam = 0.01 + math.exp(g)
        tau = lam * maturities
        z = np.exp(-tau)
        Z[:, 1 + 2 * b] = (1 - z) / tau
        Z[:, 2 + 2 * b] = Z[:, 1 + 2 * b] - z
    return Z


def simulate_panel(kind: int = KIND_DNS, T: int = 600, maturities=None, seed: int = PANEL_SEED) -> np.ndarray:
    """Simulate y_t = Z β_t + ε_t, β_{t+1} = δ + Φ β_t + η_t at θ₀ (yields in percent). Returns N×T (F-order)."""
    if maturities is None:
        maturities = maturities_360() if kind == KIND_TVL else maturities_30()
    maturities = np.asarray(maturities, dtype=np.float64)
    rng = np.random.Generator(np.random.PCG64(seed))
    tc = theta0_constrained(kind)
    M, sigma2, Q, delta, Phi = _decode(kind, tc, maturities)
    mu = np.linalg.solve(np.eye(M) - Phi, delta)
    Lq = np.linalg.cholesky(Q + 1e-14 * np.eye(M))
    N = len(maturities)
    Y = np.empty((N, T), order="F")
    beta = mu.copy()
    for t in range(T):
        if kind == KIND_TVL:
            Z = _loadings([beta[3]], maturities, 3)
            yhat = Z @ beta[:3]
        else:
            gam = tc[:2] if kind == KIND_GNS else tc[:1]
            Z = _loadings(gam, maturities, M)
            yhat = Z @ beta
        Y[:, t] = yhat + math.sqrt(sigma2) * rng.standard_normal(N)
        beta = delta + Phi @ beta + Lq @ rng.standard_normal(M)
    return Y


def theta_batch(kind: int = KIND_DNS, B: int = 65536, scale: float = 0.1, seed: int = BATCH_SEED,
                bad_frac: float = 0.01) -> np.ndarray:
    """Θ (P×B, F-order): θ_b = θ₀ + scale·N(0,I) in unconstrained space; `bad_frac` of columns get a
    non-stationary Φ to exercise the indefinite-P / -Inf paths: alternately Φ₁₂ = Φ₂₁ = 0.8 (real
    eigenvalue ≈ 1.8) and Φ₁₂ = 3, Φ₂₁ = -3 (complex pair of modulus ≈ 3)."""
    P = n_params(kind)
    rng = np.random.Generator(np.random.PCG64(seed))
    th0 = theta0(kind)
    Theta = np.asfortranarray(th0[:, None] + scale * rng.standard_normal((P, B)))
    nbad = int(round(bad_frac * B))
    if nbad:
        lay = param_layout(kind)
        idx = rng.choice(B, size=nbad, replace=False)
        a = np.where(np.arange(nbad) % 2 == 0, 0.8, 3.0)
        Theta[lay.phi_offset + 1, idx] = a  # Φ[1,2] (row-major)
        Theta[lay.phi_offset + lay.M, idx] = np.where(a == 0.8, 0.8, -3.0)  # Φ[2,1]
    return Theta


RANGE_BLOCK = 65536


def theta_range(kind: int, lo: int, hi: int, scale: float = 0.1, seed: int = BATCH_SEED) -> np.ndarray:
    """Columns [lo, hi) of a global candidate stream (P×(hi−lo), F-order) in which candidate b
    depends only on (seed, b): blocks of RANGE_BLOCK candidates each draw θ₀ + scale·N(0, I) from
    their own generator PCG64([seed, block]).  Any shard of a job (bench config 5 split over G
    GPUs) therefore evaluates exactly the candidates a single GPU would."""
    P = n_params(kind)
    th0 = theta0(kind)
    out = np.empty((P, max(hi - lo, 0)), order="F")
    b = lo
    while b < hi:
        k = b // RANGE_BLOCK
        rng = np.random.Generator(np.random.PCG64([seed, k]))
        blk = th0[:, None] + scale * rng.standard_normal((RANGE_BLOCK, P)).T
        a, e = b - k * RANGE_BLOCK, min(hi - k * RANGE_BLOCK, RANGE_BLOCK)
        out[:, b - lo:b - lo + (e - a)] = blk[:, a:e]
        b += e - a
    return out
