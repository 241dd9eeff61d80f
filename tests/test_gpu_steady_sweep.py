"""Randomised gate of the frozen-covariance steady state (FixedZFilter) — the path every
config-2/4/5 benchmark number runs.

48 seeded cases = {DNS, GNS5} × T ∈ {120, 300, 600} × 8 parameter regimes, each with 200 candidates
(three full waves and a partial fourth) and a data pattern cycling over {clean, NaN columns after the
freeze, ragged windows (candidate B−1 short), NaN columns + ragged windows}:
  scale 0.3 / scale 1.0 around θ₀; σ² = 1e-6; σ² log-uniform in [1e-6, 1]; near-unit-root Φ with a large
  σ² (slow, monotone Riccati convergence); complex-eigenvalue Φ (a rotation block: oscillating
  convergence) with a large and with a small σ²; a mix of all of them per candidate.
Every case is gated twice:
  * steady vs the full recursion (YFM_DNS_STEADY=0): every loglik within 1e-12 relative, same patterns;
  * factor-1 parity: within 1e-9 of the dense FP64 oracle, or at least as close to the binary128 truth.
The share of the launch's wave-steps that ran steady is printed per case (yfm_last_batch_steady / (waves·(T−1)))
and the sweep must exercise the path (steady > 0 in most cases; > 0 wherever the regime is the benchmark
class).  Reference: filter.jl:158-176 (the covariance recursion being frozen), :195 (the terms it feeds).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle.truth import loglik_oracle, loglik_truth
from test_gpu_parity import assert_parity
from yfm_amd import KIND_DNS, KIND_GNS
from yfm_amd import params as PR
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu

REGIMES = ["scale0.3", "scale1.0", "sigma1e-6", "sigma-range", "unit-root", "complex", "complex-small-sigma", "mixed"]
PATTERNS = ["clean", "nan", "windows", "nan+windows"]
B = 200  # 3 full waves + a partial one of 8 lanes
CASES = [(kind, T, reg) for kind in (KIND_DNS, KIND_GNS) for T in (120, 300, 600) for reg in REGIMES]


def full(fn):
    os.environ["YFM_DNS_STEADY"] = "0"
    try:
        return fn()
    finally:
        os.environ.pop("YFM_DNS_STEADY", None)


def parity_adjudicated(got, orc, tru):
    """assert_parity, with the −Inf pattern adjudicated by the truth where the dense FP64 oracle's
    determinant has the wrong sign (σ² = 1e-6: det F of the oracle's N×N LU flips; test_gpu_random's rule)."""
    flip = np.isneginf(got) != np.isneginf(orc)
    for b in np.flatnonzero(flip):
        assert np.isneginf(tru[b]) == np.isneginf(got[b]), (b, got[b], orc[b], tru[b])
        if np.isfinite(got[b]):
            assert abs(got[b] - tru[b]) <= 1e-9 * abs(tru[b]), (b, got[b], tru[b])
    keep = ~flip
    tab = assert_parity(got[keep], orc[keep], tru[keep])
    tab["oracle_sign_flips_adjudicated"] = int(flip.sum())
    return tab


def regime_theta(kind, reg, rng, n):
    """Constrained θ (P×n) of one regime."""
    lay = PR.param_layout(kind)
    M = lay.M
    scale = {"scale0.3": 0.3, "scale1.0": 1.0}.get(reg, 0.1)
    th = PR.transform_params(kind, S.theta_batch(kind, n, seed=int(rng.integers(1 << 30)), scale=scale,
                                                 bad_frac=0.02))
    phi = th[lay.phi_offset:lay.phi_offset + M * M].reshape(M, M, n)
    if reg == "sigma1e-6":
        th[lay.base_offset] = 1e-6
    elif reg == "sigma-range":
        th[lay.base_offset] = 10.0 ** rng.uniform(-6, 0, n)
    elif reg == "unit-root":
        phi[...] = rng.uniform(-0.01, 0.01, (M, M, n))
        for i in range(M):
            phi[i, i] = 1.0 - 10.0 ** rng.uniform(-3.5, -2, n)
        th[lay.base_offset] = 10.0 ** rng.uniform(-2, 0.5, n)
    elif reg in ("complex", "complex-small-sigma"):
        r = rng.uniform(0.8, 0.99, n)
        w = rng.uniform(0.2, 1.2, n)
        phi[...] = rng.uniform(-0.01, 0.01, (M, M, n))
        for i in range(M):
            phi[i, i] = 0.9
        blocks = [(0, 1)] if M == 3 else [(0, 1), (3, 4)]
        for a, b in blocks:
            phi[a, a] = phi[b, b] = r * np.cos(w)
            phi[a, b] = -r * np.sin(w)
            phi[b, a] = r * np.sin(w)
        th[lay.base_offset] = 10.0 ** rng.uniform(-2, 0.5, n) if reg == "complex" else 1e-4
    th[lay.phi_offset:lay.phi_offset + M * M] = phi.reshape(M * M, n)
    return th


def make_case(kind, T, reg, seed):
    rng = np.random.default_rng(seed)
    N = [30, 30, 20, 12, 32, 8][seed % 6]
    mats = S.maturities_30() if N == 30 else np.sort(rng.choice(np.arange(3, 361), N, replace=False)).astype(float)
    Y = S.simulate_panel(kind, T, maturities=mats, seed=int(rng.integers(1 << 30))).copy(order="F")
    if reg == "mixed":
        parts = [regime_theta(kind, r, rng, B) for r in REGIMES[:-1]]
        pick = rng.integers(len(parts), size=B)
        th = np.stack([parts[pick[b]][:, b] for b in range(B)], axis=1)
    else:
        th = regime_theta(kind, reg, rng, B)
    pattern = PATTERNS[seed % len(PATTERNS)]
    if "nan" in pattern:  # after the first blocks (the lanes have frozen), one of them straddling a block edge
        cols = [T // 3, T // 3 + 1, (2 * T) // 3, 16 * (T // 32) - 1]
        Y[:, cols] = np.nan
    T_use = None
    if "windows" in pattern:
        T_use = np.full(B, T, dtype=np.int32)
        T_use[B - 1] = T // 2          # the partial last wave's mirror candidate: short window
        T_use[70] = T // 3             # one lane of the second wave
        T_use[150:160] = rng.integers(T // 2, T + 1, 10)
    space = seed % 2  # constrained θ as set_params! takes it, or unconstrained as compute_loss does
    Th = np.asfortranarray(th if space == 1 else PR.untransform_params(kind, th))
    return N, mats, Y, Th, space, T_use, pattern


@pytest.mark.parametrize("case", range(len(CASES)))
def test_steady_sweep(engine, case):
    kind, T, reg = CASES[case]
    N, mats, Y, Th, space, T_use, pattern = make_case(kind, T, reg, 7000 + case)
    engine.set_panel(Y, mats)
    os.environ["YFM_GNS5_STEADY"] = "1"  # GNS5's steady state is opt-in: gate it here too
    try:
        got = engine.loglik(kind, Th, space=space, T_use=T_use)
        steady_ws = engine.last_steady()
    finally:
        os.environ.pop("YFM_GNS5_STEADY", None)
    ref = full(lambda: engine.loglik(kind, Th, space=space, T_use=T_use))
    assert engine.last_steady() == 0
    # wave-steps of the launch (the partial wave's lanes past B mirror candidate B − 1's window)
    tu = np.full(B, T) if T_use is None else T_use
    waves = -(-B // 64)
    share = steady_ws / float(waves * (max(tu) - 1))
    fin = np.isfinite(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isneginf(got), np.isneginf(ref))
    d = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    print(f"case {case}: kind {kind} T {T} N {N} {reg:20s} {pattern:12s} space {space}: steady share {share:.3f}, "
          f"finite {fin.sum()}/{B}, steady vs full max rel {d.max() if d.size else 0:.2e}, "
          f"bitwise {np.mean(got[fin] == ref[fin]) if d.size else 1:.3f}")
    assert d.size == 0 or d.max() <= 1e-12
    orc = loglik_oracle(kind, Y, mats, Th, space=space, T_use=T_use)
    tru = loglik_truth(kind, Y, mats, Th, space=space, T_use=T_use)
    tab = parity_adjudicated(got, orc, tru)
    print(f"   parity {tab}")
    if reg in ("scale0.3", "sigma1e-6", "complex-small-sigma") and fin.sum() > 150:
        assert share > 0.0  # the benchmark class and the fast-gain regimes must reach frozen waves


def test_partial_wave_short_mirror_nan_after_freeze(engine):
    """B not a multiple of 64, the partial wave's lanes past B mirror candidate B − 1,
    whose window is shorter than its wave-mates', and a NaN column after the freeze.  The lanes inside
    their windows thaw at the NaN column, the mirrors do not; the wave's frozen state must still be
    uniform (the next block must not run the steady loop on some lanes and the full one on others)."""
    mats = S.maturities_30()
    T = 400
    Y = S.simulate_panel(KIND_DNS, T, maturities=mats).copy(order="F")
    Y[:, [200, 201]] = np.nan
    engine.set_panel(Y, mats)
    Bp = 64 * 4 + 10
    Th = S.theta_batch(KIND_DNS, Bp, seed=41, bad_frac=0.0)
    tu = np.full(Bp, T, dtype=np.int32)
    tu[Bp - 1] = 150  # ends before the NaN columns: its mirrors never reach them
    got = engine.loglik(KIND_DNS, Th, T_use=tu)
    st = engine.last_steady()
    ref = full(lambda: engine.loglik(KIND_DNS, Th, T_use=tu))
    assert st > 0
    d = np.abs(got - ref) / np.abs(ref)
    print(f"steady wave-steps {st}, max rel vs full {d.max():.2e}")
    assert d.max() <= 1e-12
    # the same candidates in full waves (B a multiple of 64): bitwise the same logliks
    got2 = engine.loglik(KIND_DNS, np.asfortranarray(Th[:, :256]), T_use=tu[:256])
    np.testing.assert_array_equal(got2, got[:256])
