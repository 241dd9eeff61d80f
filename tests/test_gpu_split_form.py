"""Regression test of commit 7a42719: with the measurement update written as two functions
(collapsed_cov + collapsed_mean) instead of the one body of collapsed_update, the GNS5 NP = 48 per-lane
instantiation (N = 33, the kernel that spills ≈1.8 KB per lane) returned O(1)-wrong logliks on the
3,000-seed sweep's cases 292, 916 and 2431.  Both forms are the same arithmetic (explicit fma, FP
contraction off), so they must give the same bits.  The library keeps diagnostic instantiations of the
two-function form (YFM_FZ_SPLIT_FORM=1, GNS5 NP ∈ {30, 48}, full recursion); this test runs both
forms on those cases and at the config-5 shape: bitwise equal, and factor-1 parity against the dense
oracle / binary128 truth.  Reference: filter.jl:143-176 (the update both forms restate)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle.truth import loglik_oracle, loglik_truth
from test_gpu_parity import assert_parity
from test_gpu_random import random_case
from yfm_amd import KIND_GNS
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu

# the regression is fenced by a build flag (build_native.py): refuse to run on a library built
# without it, loudly (tools/agpr_spill_repro/ reproduces the miscompile on the last unfenced sources)
import build_native as _BN  # noqa: E402

if "-amdgpu-spill-vgpr-to-agpr=0" not in _BN.FLAGS or (_BN.STAMP.exists() and
                                                       "-amdgpu-spill-vgpr-to-agpr=0" not in _BN.STAMP.read_text()):
    raise RuntimeError("libyfm_hip.so must be built with -mllvm -amdgpu-spill-vgpr-to-agpr=0 (DESIGN.md §5)")


def both_forms(engine, kind, Th, space=0, T_use=None):
    os.environ["YFM_DNS_STEADY"] = "0"  # the diagnostic instantiations are the full recursion
    try:
        one = engine.loglik(kind, Th, space=space, T_use=T_use)
        os.environ["YFM_FZ_SPLIT_FORM"] = "1"
        two = engine.loglik(kind, Th, space=space, T_use=T_use)
    finally:
        os.environ.pop("YFM_FZ_SPLIT_FORM", None)
        os.environ.pop("YFM_DNS_STEADY", None)
    return one, two


@pytest.mark.parametrize("seed", [292, 916, 2431])
def test_split_form_regression_7a42719(engine, seed):
    rng = np.random.default_rng(1000 + seed)
    N, T, mats, Y, Th, space, T_use = random_case(rng, KIND_GNS)
    engine.set_panel(Y, mats)
    one, two = both_forms(engine, KIND_GNS, Th, space, T_use)
    print(f"seed {seed}: N {N} T {T} space {space} windows {T_use is not None}; forms differ at "
          f"{np.flatnonzero(~((one == two) | (np.isnan(one) & np.isnan(two))))}")
    np.testing.assert_array_equal(one, two)
    assert_parity(two, loglik_oracle(KIND_GNS, Y, mats, Th, space=space, T_use=T_use),
                  loglik_truth(KIND_GNS, Y, mats, Th, space=space, T_use=T_use))


@pytest.mark.parametrize("N", [30, 33, 40])
def test_split_form_config_shape(engine, N):
    """The same at T = 600 for NP = 30 (N = 30) and NP = 48 (N = 33, 40), 512 candidates."""
    mats = S.maturities_30() if N == 30 else np.sort(np.random.default_rng(N).choice(np.arange(3, 361), N,
                                                                                     replace=False)).astype(float)
    Y = S.simulate_panel(KIND_GNS, 600, maturities=mats)
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_GNS, 512, seed=N)
    one, two = both_forms(engine, KIND_GNS, Th)
    np.testing.assert_array_equal(one, two)
    sub = np.asfortranarray(Th[:, :64])
    assert_parity(two[:64], loglik_oracle(KIND_GNS, Y, mats, sub), loglik_truth(KIND_GNS, Y, mats, sub))
