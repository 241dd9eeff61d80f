"""GPU parity on the reference's numeric edge cases (tests/golden/edge/make_edge.py):
σ² ∈ {1e-6, 1e-8} (κ(F) = 1e8..1e11), σ² underflowing to 0 (unconstrained θ = −800 and constrained
σ² = 0: F singular in exact arithmetic ⇒ −Inf), and F = 0 (σ² = 0, U = 0: inv(F) throws — DNS sets
F⁻¹ = Inf, TVλ leaves it stale, filter.jl:149-155 / :51-56 — so get_loss returns −Inf, or 0.0 when
the window has two columns).  Rule: test_gpu_parity.assert_parity (1e-9 of the LAPACK oracle or
at least as close to the binary128 truth, −Inf / NaN patterns exact), in the default precision;
the TVλ FP64 mode is held to the patterns (its small-σ² EKF runs amplify rounding like the
reference's own: the oracle is up to 70% from exact arithmetic there)."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN
from test_gpu_parity import assert_parity, parity_table
from yfm_amd import KIND_TVL, _lib

pytestmark = pytest.mark.gpu

with np.load(GOLDEN / "edge" / "edge_cases.npz", allow_pickle=False) as _z:
    FX = {k: _z[k] for k in _z.files}
NAMES = [str(n) for n in FX["names"]]


def case(name):
    return {k.split("/", 1)[1]: v for k, v in FX.items() if k.startswith(name + "/")}


@pytest.mark.parametrize("name", NAMES)
def test_edge_case(engine, name):
    c = case(name)
    kind = int(c["kind"])
    engine.set_panel(c["Y"], c["maturities"])
    got = engine.loglik(kind, c["Theta"], space=int(c["space"]), T_use=c.get("T_use"))
    table = assert_parity(got, c["loglik_oracle"], c["loglik_truth"])
    print(name, table)
    if kind == KIND_TVL:
        engine.precision = _lib.PREC_FP64
        try:
            f = engine.loglik(kind, c["Theta"], space=int(c["space"]), T_use=c.get("T_use"))
        finally:
            engine.precision = _lib.PREC_CERTIFIED
        ora = c["loglik_oracle"]
        assert np.array_equal(np.isfinite(f), np.isfinite(ora)) and np.array_equal(np.isnan(f), np.isnan(ora))
        print(name, "fp64", parity_table(f, ora, c["loglik_truth"]))
