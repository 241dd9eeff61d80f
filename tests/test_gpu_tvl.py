"""GPU parity of the TVλ extended Kalman filter kernel (yfm_tvl.hip) — SURVEY §8 a8, config 3.

Oracles: the committed golden fixture (NumPy restatement, tests/golden/tvl_basic.npz, with
a 40-digit truth for its first candidate) and the independent C restatement
(oracle/yfm_oracle.c: dense N×N getrf+getri per step, the reference's algorithm) at the
config-3 cross-section N = 360.  Tolerance: 1e-9 relative on the loglik (north star).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT, load_golden
from oracle.kalman_ld import loglik_ld_tvl
from test_gpu_parity import REL, assert_ll_close, assert_parity
from yfm_amd import KIND_TVL
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu

LANES = [1, 2, 4, 8, 16, 32, 64]


def engine_default_lanes(B):
    """The launcher's own choice (yfm_tvl.hip: tvl_lanes_for) for N = 360."""
    L = 1
    while L < min(64, -(-131072 // B)):
        L *= 2
    return L


class lanes_override:
    """Force the lanes-per-filter choice of the TVλ launcher (YFM_TVL_LANES, read per call)."""

    def __init__(self, L):
        self.L = L

    def __enter__(self):
        os.environ["YFM_TVL_LANES"] = str(self.L)

    def __exit__(self, *exc):
        os.environ.pop("YFM_TVL_LANES", None)


def c_oracle(Y, mats, Th, T_use=None, threads=16):
    lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
    D = ctypes.POINTER(ctypes.c_double)
    Yf = np.asfortranarray(Y)
    Thf = np.asfortranarray(Th)
    N, T = Yf.shape
    P, B = Thf.shape
    out = np.empty(B)
    tu = None
    if T_use is not None:
        tu = np.ascontiguousarray(T_use, dtype=np.int32)
    lib.yfm_oracle_loglik(KIND_TVL, 0, Yf.ctypes.data_as(D), N, T, np.ascontiguousarray(mats).ctypes.data_as(D),
                          Thf.ctypes.data_as(D), P, B,
                          None if tu is None else tu.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                          out.ctypes.data_as(D), threads)
    return out


@pytest.mark.parametrize("L", LANES)
def test_tvl_golden_every_group_width(engine, L):
    g = load_golden("tvl_basic")
    engine.set_panel(g["Y"], g["maturities"])
    with lanes_override(L):
        got = engine.loglik(KIND_TVL, g["Theta"])
    k = len(g["ll_truth"])
    assert_parity(got[:k], g["loglik"][:k], g["ll_truth"])
    assert_ll_close(got[k:], g["loglik"][k:])


@pytest.mark.parametrize("L", [1, 8, 64])
def test_tvl_states_vs_truth(engine, L):
    g = load_golden("tvl_basic")
    engine.set_panel(g["Y"], g["maturities"])
    with lanes_override(L):
        ll, beta, P = engine.filter_states(KIND_TVL, g["Theta"][:, :1])
    for got, ora, tru in ((beta[..., 0], g["beta_traj"][..., 0], g["beta_truth"][..., 0]),
                          (P[..., 0], g["P_traj"][..., 0], g["P_truth"][..., 0])):
        scale = np.abs(tru).max()
        oracle_err = np.abs(ora - tru).max() / scale
        assert np.abs(got - ora).max() / scale <= max(REL, 2 * oracle_err)
        assert np.abs(got - tru).max() / scale <= 1e-10


@pytest.fixture(scope="module")
def config3():
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    return Y, mats


def test_tvl_config3_cross_section_vs_c_oracle(engine, config3):
    """N = 360 maturities (config 3), T = 100, 32 candidates: the C restatement of the reference's dense
    360×360 path vs the kernel at its default group width and at L = 1 / 64."""
    Y, mats = config3
    Y = np.asfortranarray(Y[:, :100])
    Th = S.theta_batch(KIND_TVL, 32, seed=31, bad_frac=0.0, scale=0.02)
    Th[:, 0] = S.theta0(KIND_TVL)
    ref = c_oracle(Y, mats, Th)
    truth = loglik_ld_tvl(mats, Y, Th)
    alt = loglik_ld_tvl(mats, Y, Th, dtype=np.float64)
    engine.set_panel(Y, mats)
    got = engine.loglik(KIND_TVL, Th)
    assert_parity(got, ref, truth, alt=alt)
    for L in (1, 64):
        with lanes_override(L):
            assert_parity(engine.loglik(KIND_TVL, Th), ref, truth, alt=alt)


def test_tvl_windows_nan_and_edges(engine, config3):
    """T_use windows, NaN columns (prediction-only steps, stale F/v re-added), tiny T."""
    Y, mats = config3
    sub = np.arange(0, 360, 9)  # N = 40
    Yn = np.asfortranarray(Y[sub, :90].copy())
    Yn[:, [5, 6, 50]] = np.nan
    Yn[7, 70] = np.nan
    m = mats[sub].copy()
    Th = S.theta_batch(KIND_TVL, 12, seed=37, bad_frac=0.0, scale=0.02)
    tu = np.array([1, 2, 3, 10, 40, 89, 90, 90, 64, 65, 33, 77], dtype=np.int32)
    ref = c_oracle(Yn, m, Th, T_use=tu)
    truth = loglik_ld_tvl(m, Yn, Th, T_use=tu)
    alt = loglik_ld_tvl(m, Yn, Th, T_use=tu, dtype=np.float64)
    engine.set_panel(Yn, m)
    for L in (1, 4, 64):
        with lanes_override(L):
            assert_parity(engine.loglik(KIND_TVL, Th, T_use=tu), ref, truth, alt=alt)


def test_tvl_full_batch_properties(engine, config3):
    """Config 3 at B = 16,384, T = 600, N = 360: deterministic, independent of batch position, flags
    consistent; and independent of the group width up to rounding: on 48 candidates the default width
    and L = 64 are each within max(1e-9, 100 × the error of an FP64 NumPy run of the same algebra) of the
    long-double truth (the TVλ EKF is ill-conditioned for a sizeable share of candidates: FP64 rounding
    alone moves their loglik by 1e-8..1e-3, for the reference's dense path even more — DESIGN.md §5)."""
    Y, mats = config3
    engine.set_panel(Y, mats)
    Th = S.theta_batch(KIND_TVL, 16384, seed=41, bad_frac=0.01, scale=0.02)
    a = engine.loglik(KIND_TVL, Th)
    n_throw, n_neginf = engine.last_flags()
    assert n_throw == np.isnan(a).sum() and n_neginf == np.isneginf(a).sum()
    np.testing.assert_array_equal(engine.loglik(KIND_TVL, Th), a)
    perm = np.random.default_rng(5).permutation(16384)[:512]
    with lanes_override(engine_default_lanes(16384)):
        c = engine.loglik(KIND_TVL, np.asfortranarray(Th[:, perm]))
    np.testing.assert_array_equal(c, a[perm])  # same group width → bitwise position independent
    assert np.isfinite(a).mean() > 0.9
    sub = np.asfortranarray(Th[:, perm[:48]])
    truth = loglik_ld_tvl(mats, Y, sub)
    fp64 = loglik_ld_tvl(mats, Y, sub, dtype=np.float64)
    with lanes_override(64):
        w64 = engine.loglik(KIND_TVL, sub)
    fin = np.isfinite(truth)
    assert np.array_equal(fin, np.isfinite(a[perm[:48]])) and np.array_equal(fin, np.isfinite(w64))
    bound = np.maximum(1e-9, 100 * np.abs(fp64[fin] - truth[fin]) / np.abs(truth[fin]))
    for got in (a[perm[:48]], w64):
        assert np.all(np.abs(got[fin] - truth[fin]) / np.abs(truth[fin]) <= bound)


@pytest.mark.parametrize("grid", ["wu30", "irregular"])
def test_tvl_maturity_grids_and_exp_paths(engine, grid):
    """The exp recurrence over maturity jumps (≤ 8 distinct m_{i+L} − m_i) vs one exp per maturity
    (YFM_TVL_EXP=1, also the automatic fallback for irregular grids), against the C oracle + truth."""
    if grid == "wu30":
        mats = S.maturities_30()
    else:
        mats = np.sort(np.random.default_rng(3).uniform(1.0, 360.0, 24)).round(3)
    Y = S.simulate_panel(KIND_TVL, 80, maturities=mats)
    Th = S.theta_batch(KIND_TVL, 16, seed=43, bad_frac=0.0, scale=0.02)
    ref = c_oracle(Y, mats, Th)
    truth = loglik_ld_tvl(mats, Y, Th)
    alt = loglik_ld_tvl(mats, Y, Th, dtype=np.float64)
    engine.set_panel(Y, mats)
    for L in (1, 4, 16):
        with lanes_override(L):
            rec = engine.loglik(KIND_TVL, Th)
            os.environ["YFM_TVL_EXP"] = "1"
            try:
                ex = engine.loglik(KIND_TVL, Th)
            finally:
                os.environ.pop("YFM_TVL_EXP", None)
        assert_parity(rec, ref, truth, alt=alt)
        assert_parity(ex, ref, truth, alt=alt)
