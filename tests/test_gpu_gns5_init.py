"""GNS5 initial state (initialize_filter, filter.jl:1-10, for the 5-factor extension): the cooperative kernel that
spreads each candidate's 15×15 Lyapunov system over 2 lanes (yfm_kernels.hip fixedz_init_coop_kernel,
YFM_GNS5_INIT_LANES) runs gauss_solve's arithmetic operation for operation, so every loglik — finite, −Inf or the
NaN of a singular system — is bitwise the per-lane kernel's (YFM_GNS5_INIT_LANES=1), and the throw / −Inf counters
agree."""
from __future__ import annotations

import os

import numpy as np
import pytest

from yfm_amd import KIND_GNS
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu


def _run(engine, Th, lanes):
    os.environ["YFM_GNS5_INIT_LANES"] = str(lanes)
    try:
        ll = engine.loglik(KIND_GNS, Th)
        flags = engine.last_flags()
    finally:
        os.environ.pop("YFM_GNS5_INIT_LANES", None)
    return ll, flags


@pytest.mark.parametrize("lanes", [2])
def test_gns5_coop_init_bitwise(engine, lanes):
    Y = S.simulate_panel(KIND_GNS, 240)
    engine.set_panel(Y, S.maturities_30())
    # config 5's candidate stream (90% explosive Φ), a wide one, and B not a multiple of the block's groups
    Th = np.asfortranarray(np.concatenate([S.theta_range(KIND_GNS, 0, 4096, scale=0.1),
                                           S.theta_range(KIND_GNS, 4096, 8189, scale=1.0)], axis=1))  # P × B
    ref, f_ref = _run(engine, Th, 1)
    got, f_got = _run(engine, Th, lanes)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), np.flatnonzero(got.view(np.int64) != ref.view(np.int64))[:8]
    assert f_got == f_ref
    print(lanes, "finite", int(np.isfinite(ref).sum()), "of", ref.size, "flags", f_ref)


def test_gns5_coop_init_singular_throws(engine):
    """Φ = I in constrained space: I − Φ and the Lyapunov system are exactly singular — NaN and the throw counter,
    as initialize_filter throwing in the reference (§8b)."""
    Y = S.simulate_panel(KIND_GNS, 120)
    engine.set_panel(Y, S.maturities_30())
    lay = S.param_layout(KIND_GNS)
    Th = np.asfortranarray(np.repeat(S.theta0_constrained(KIND_GNS).reshape(-1, 1), 5, axis=1))
    Th[lay.phi_offset:lay.phi_offset + 25, :] = np.eye(5).reshape(25, 1)
    for lanes in (1, 2):
        os.environ["YFM_GNS5_INIT_LANES"] = str(lanes)
        try:
            ll = engine.loglik(KIND_GNS, Th, space=1)
            n_throw, _ = engine.last_flags()
        finally:
            os.environ.pop("YFM_GNS5_INIT_LANES", None)
        assert np.isnan(ll).all() and n_throw == Th.shape[1], (lanes, ll, n_throw)
