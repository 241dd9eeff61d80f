"""GPU parity of the TVλ extended Kalman filter (yfm_tvl_dd.hip / yfm_tvl.hip) — SURVEY §8 a8, config 3.

Oracles: the C restatement of the reference's dense path (oracle/yfm_oracle.c: F = ZPZ' + σ²I
formed, getrf + getri and a logdet LU every step — filter.jl:12-80, :182-209) and the binary128
evaluation of the same recursion (oracle/yfm_truth.c, pinned to the 40-digit dense mpmath
restatement in tests/test_oracle.py).

Rule (north star, factor 1, no noise-floor allowance): within 1e-9 relative of the oracle, or at
least as close to the truth as the oracle is.  The default precision (YFM_PREC_CERTIFIED, the
double-double filter) must meet it on every candidate and is additionally checked to reproduce
the truth to ~1e-13.  YFM_PREC_FP64 is the reference's arithmetic class: on candidates whose EKF
amplifies rounding (config 3: a quarter of the batch) no FP64 evaluation — the oracle's included
— is within 1e-9 of exact arithmetic, so for it the tests assert reproducibility and report the
(within 1e-9, adjudicated, failing) table.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle.truth import loglik_oracle, loglik_truth, states_truth
from test_gpu_parity import assert_parity, parity_table
from yfm_amd import KIND_TVL
from yfm_amd import _lib
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu

EXACT = 1e-13  # the certified filter vs binary128 truth (measured: 0 on the config-3 sample)


class env:
    """Set environment overrides of the TVλ launcher (read per call): YFM_TVL_LANES, YFM_TVL_EXP."""

    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        os.environ.update(self.kv)

    def __exit__(self, *exc):
        for k in self.kv:
            os.environ.pop(k, None)


class precision:
    def __init__(self, engine, mode):
        self.engine, self.mode = engine, mode

    def __enter__(self):
        self.old = self.engine.precision
        self.engine.precision = self.mode

    def __exit__(self, *exc):
        self.engine.precision = self.old


def rel(a, b):
    fin = np.isfinite(b)
    return np.abs(a[fin] - b[fin]) / np.maximum(np.abs(b[fin]), 1e-300)


def test_default_precision_is_certified(engine):
    assert engine.precision == _lib.PREC_CERTIFIED


@pytest.mark.parametrize("L", [4, 8, 16, 32, 64])
def test_tvl_golden_certified_every_group_width(engine, L):
    g = load_golden("tvl_basic")
    truth = loglik_truth(KIND_TVL, g["Y"], g["maturities"], g["Theta"])
    engine.set_panel(g["Y"], g["maturities"])
    with env(YFM_TVL_LANES=L):
        got = engine.loglik(KIND_TVL, g["Theta"])
    assert_parity(got, g["loglik"], truth)
    assert rel(got, truth).max() <= EXACT


@pytest.mark.parametrize("L", [1, 2, 4, 8, 16, 32, 64])
def test_tvl_golden_fp64_every_group_width(engine, L):
    g = load_golden("tvl_basic")
    truth = loglik_truth(KIND_TVL, g["Y"], g["maturities"], g["Theta"])
    engine.set_panel(g["Y"], g["maturities"])
    with precision(engine, _lib.PREC_FP64), env(YFM_TVL_LANES=L):
        got = engine.loglik(KIND_TVL, g["Theta"])
    assert_parity(got, g["loglik"], truth)


@pytest.mark.parametrize("mode", [_lib.PREC_CERTIFIED, _lib.PREC_FP64])
def test_tvl_states_vs_truth(engine, mode):
    """β and P after every filter! call (filter.jl:12-80) vs the binary128 trajectories."""
    g = load_golden("tvl_basic")
    engine.set_panel(g["Y"], g["maturities"])
    with precision(engine, mode):
        ll, beta, P = engine.filter_states(KIND_TVL, g["Theta"][:, :2])
    for b in range(2):
        _, bt, Pt = states_truth(KIND_TVL, g["Y"], g["maturities"], g["Theta"][:, b], space=int(g["space"]))
        tol = EXACT if mode == _lib.PREC_CERTIFIED else 1e-10
        for got, tru in ((beta[..., b], bt), (P[..., b], Pt)):
            assert np.abs(got - tru).max() / np.abs(tru).max() <= tol


@pytest.fixture(scope="module")
def config3():
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    with np.load(GOLDEN / "config3" / "tvl_config3_sample.npz", allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    return Y, mats, fx


def test_tvl_config3_sample_certified(engine, config3):
    """Config 3's workload (N = 360, T = 600) on the first 64 candidates of the bench batch: every
    candidate within 1e-9 of the dense oracle or at least as close to the binary128 truth (factor
    1) — where the oracle itself is up to 3e-4 from exact arithmetic."""
    Y, mats, fx = config3
    engine.set_panel(Y, mats)
    got = engine.loglik(KIND_TVL, fx["Theta"])
    table = assert_parity(got, fx["loglik_oracle"], fx["loglik_truth"])
    print("certified", table)
    assert table["failing"] == 0 and table["within_1e-9"] + table["adjudicated"] == 64
    assert rel(got, fx["loglik_truth"]).max() <= EXACT


def test_tvl_config3_sample_fp64(engine, config3):
    """The FP64 filter on the same sample: bitwise reproducible, the oracle's −Inf / NaN pattern,
    and at least as accurate as the reference's dense FP64 path in the median; the (within 1e-9,
    adjudicated, failing) table is printed."""
    Y, mats, fx = config3
    engine.set_panel(Y, mats)
    with precision(engine, _lib.PREC_FP64):
        got = engine.loglik(KIND_TVL, fx["Theta"])
        np.testing.assert_array_equal(engine.loglik(KIND_TVL, fx["Theta"]), got)
    ora, tru = fx["loglik_oracle"], fx["loglik_truth"]
    assert np.array_equal(np.isfinite(got), np.isfinite(ora)) and np.array_equal(np.isnan(got), np.isnan(ora))
    print("fp64", parity_table(got, ora, tru))
    assert np.median(rel(got, tru)) <= max(np.median(rel(ora, tru)), 1e-13)


@pytest.fixture(scope="module")
def config3_1024():
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    with np.load(GOLDEN / "config3" / "tvl_config3_1024.npz", allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    return Y, mats, fx


def test_tvl_config3_1024_certified(engine, config3_1024):
    """The certified filter on 1,024 config-3 candidates: factor-1 parity on every one, and every
    candidate within 1e-9 of the binary128 truth — where the reference's dense FP64 path (the oracle)
    is up to 1.1e-2 from exact arithmetic on this sample (tests/golden/config3/make_tvl_config3_1024.py).
    (A few candidates amplify rounding by up to ~1e20, so even double-double lands up to ~1e-10 from
    the truth there — 5 of the 1,012 finite ones above 1e-13, for the round-2 kernel as for this one,
    profiles/r3/tvl_dd_ab; the rest reproduce it to ~1e-13.)"""
    Y, mats, fx = config3_1024
    engine.set_panel(Y, mats)
    got = engine.loglik(KIND_TVL, fx["Theta"])
    table = assert_parity(got, fx["loglik_oracle"], fx["loglik_truth"])
    e = rel(got, fx["loglik_truth"])
    print("certified 1024", table, "max rel vs truth %.2e, %d above 1e-13" % (e.max(), (e > EXACT).sum()))
    assert table["failing"] == 0
    # the measured count (5 on every build since round 3: profiles/r3/tvl_dd_ab*, profiles/r4/ab2, ab3)
    assert e.max() <= 1e-9 and (e > EXACT).sum() <= 5


def test_tvl_config3_1024_fp64_reference_class(engine, config3_1024):
    """FP64 mode is the reference's arithmetic class: on amplifying candidates every FP64 evaluation
    (the reference's dense path included) is rounding noise around the exact value.  On 1,024
    candidates its error against the binary128 truth must be no worse than the dense oracle's in the
    median and at the 99th percentile, and its largest error within 2× the oracle's largest; the
    patterns must match."""
    Y, mats, fx = config3_1024
    engine.set_panel(Y, mats)
    with precision(engine, _lib.PREC_FP64):
        got = engine.loglik(KIND_TVL, fx["Theta"])
    ora, tru = fx["loglik_oracle"], fx["loglik_truth"]
    assert np.array_equal(np.isfinite(got), np.isfinite(ora)) and np.array_equal(np.isnan(got), np.isnan(ora))
    eg, eo = rel(got, tru), rel(ora, tru)
    q = lambda e: (float(np.median(e)), float(np.quantile(e, 0.99)), float(e.max()))  # noqa: E731
    print("fp64 1024 (median, p99, max) gpu", q(eg), "oracle", q(eo), parity_table(got, ora, tru))
    assert np.median(eg) <= max(np.median(eo), 1e-13)
    assert np.quantile(eg, 0.99) <= np.quantile(eo, 0.99)
    assert eg.max() <= 2.0 * eo.max()


def test_tvl_windows_nan_and_edges(engine, config3):
    """T_use windows, NaN columns (prediction-only steps, stale F/v re-added), tiny T."""
    Y, mats, _ = config3
    sub = np.arange(0, 360, 9)  # N = 40
    Yn = np.asfortranarray(Y[sub, :90].copy())
    Yn[:, [5, 6, 50]] = np.nan
    Yn[7, 70] = np.nan
    m = mats[sub].copy()
    Th = S.theta_batch(KIND_TVL, 12, seed=37, bad_frac=0.0, scale=0.02)
    tu = np.array([1, 2, 3, 10, 40, 89, 90, 90, 64, 65, 33, 77], dtype=np.int32)
    ref = loglik_oracle(KIND_TVL, Yn, m, Th, T_use=tu)
    truth = loglik_truth(KIND_TVL, Yn, m, Th, T_use=tu)
    engine.set_panel(Yn, m)
    for L in (4, 64):
        with env(YFM_TVL_LANES=L):
            got = engine.loglik(KIND_TVL, Th, T_use=tu)
        assert_parity(got, ref, truth)
        assert rel(got, truth).max(initial=0.0) <= EXACT
    with precision(engine, _lib.PREC_FP64):
        for L in (1, 4, 64):
            with env(YFM_TVL_LANES=L):
                got = engine.loglik(KIND_TVL, Th, T_use=tu)
            assert np.array_equal(np.isfinite(got), np.isfinite(ref)) and np.array_equal(np.isnan(got), np.isnan(ref))


def test_tvl_full_batch_properties(engine, config3):
    """Config 3 at B = 16,384, T = 600, N = 360 in the default precision: deterministic, independent
    of batch position, flag counters consistent, exact (vs binary128) on a 48-candidate sample;
    the FP64 mode has the same −Inf / NaN pattern."""
    Y, mats, _ = config3
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_TVL, 16384, seed=41, bad_frac=0.01, scale=0.02)
    a = engine.loglik(KIND_TVL, Th)
    n_throw, n_neginf = engine.last_flags()
    assert n_throw == np.isnan(a).sum() and n_neginf == np.isneginf(a).sum()
    np.testing.assert_array_equal(engine.loglik(KIND_TVL, Th), a)
    perm = np.random.default_rng(5).permutation(16384)[:512]
    with env(YFM_TVL_LANES=4):  # the launcher's width at B = 16,384
        c = engine.loglik(KIND_TVL, np.asfortranarray(Th[:, perm]))
    np.testing.assert_array_equal(c, a[perm])  # same group width → bitwise position independent
    assert np.isfinite(a).mean() > 0.9
    sub = np.asfortranarray(Th[:, perm[:48]])
    truth = loglik_truth(KIND_TVL, Y, mats, sub)
    assert np.array_equal(np.isfinite(truth), np.isfinite(a[perm[:48]]))
    assert rel(a[perm[:48]], truth).max() <= EXACT
    with precision(engine, _lib.PREC_FP64):
        f = engine.loglik(KIND_TVL, Th)
    assert np.array_equal(np.isfinite(f), np.isfinite(a)) and np.array_equal(np.isnan(f), np.isnan(a))


@pytest.mark.parametrize("L", [4, 8, 16, 32])
def test_tvl_power_mode_wu30_t600(engine, L):
    """The certified kernel's power mode (the N = 30 grid has 12–13 distinct jumps at L ≥ 4, more than the exact
    jump table holds: e^{−λm} = (e^{−λΔ})^{m/Δ}, Δ = 3 months, one dd exp per step) against one dd exp per
    maturity (YFM_TVL_EXP=1), at T = 600 on 64 candidates: both at factor 1 against the dense oracle and the
    binary128 truth, and the power mode within 4× the per-maturity path's own distance from the truth (+1e-13)."""
    mats = S.maturities_30()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    Th = S.theta_batch(KIND_TVL, 64, seed=47, bad_frac=0.0, scale=0.02)
    engine.set_panel(Y, mats)
    with env(YFM_TVL_LANES=L):
        pw = engine.loglik(KIND_TVL, Th)
        with env(YFM_TVL_EXP=1):
            ex = engine.loglik(KIND_TVL, Th)
    ref = loglik_oracle(KIND_TVL, Y, mats, Th)
    truth = loglik_truth(KIND_TVL, Y, mats, Th)
    for got in (pw, ex):
        assert_parity(got, ref, truth)
    e_pw, e_ex = rel(pw, truth), rel(ex, truth)
    print(f"L {L}: power mode vs truth max {e_pw.max():.2e} (median {np.median(e_pw):.2e}); one exp per maturity "
          f"{e_ex.max():.2e}; above 1e-13: {int((e_pw > EXACT).sum())} / {int((e_ex > EXACT).sum())}")
    assert e_pw.max() <= 4.0 * e_ex.max() + EXACT
    assert int((e_pw > EXACT).sum()) <= int((e_ex > EXACT).sum()) + 1


@pytest.mark.parametrize("grid", ["wu30", "irregular", "quarters"])
def test_tvl_maturity_grids_and_exp_paths(engine, grid):
    """The exp recurrence over maturity jumps (≤ 8 distinct m_{i+L} − m_i) vs one exp per maturity
    (YFM_TVL_EXP=1, also the automatic fallback for irregular grids), both precisions; "quarters" (maturities k/4
    years: exact differences, not integers, one jump) takes the certified kernel's exact table with the jump factor
    read across the group by ds_bpermute."""
    if grid == "wu30":
        mats = S.maturities_30()
    elif grid == "quarters":
        mats = 0.25 * np.arange(1, 121, dtype=np.float64)
    else:
        mats = np.sort(np.random.default_rng(3).uniform(1.0, 360.0, 24)).round(3)
    Y = S.simulate_panel(KIND_TVL, 80, maturities=mats)
    Th = S.theta_batch(KIND_TVL, 16, seed=43, bad_frac=0.0, scale=0.02)
    ref = loglik_oracle(KIND_TVL, Y, mats, Th)
    truth = loglik_truth(KIND_TVL, Y, mats, Th)
    engine.set_panel(Y, mats)
    for L in (4, 16):
        with env(YFM_TVL_LANES=L):
            rec = engine.loglik(KIND_TVL, Th)
            with env(YFM_TVL_EXP=1):
                ex = engine.loglik(KIND_TVL, Th)
        for got in (rec, ex):
            assert_parity(got, ref, truth)
            assert rel(got, truth).max() <= EXACT
    with precision(engine, _lib.PREC_FP64):
        for L in (1, 4, 16):
            with env(YFM_TVL_LANES=L):
                rec = engine.loglik(KIND_TVL, Th)
                with env(YFM_TVL_EXP=1):
                    ex = engine.loglik(KIND_TVL, Th)
            for got in (rec, ex):
                assert np.array_equal(np.isfinite(got), np.isfinite(ref))
                print(grid, L, parity_table(got, ref, truth))
