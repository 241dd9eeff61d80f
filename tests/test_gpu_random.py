"""Randomised parity sweep (seeded): the HIP library through the C ABI vs the C restatement of the
reference filter (oracle/yfm_oracle.c: dense N×N getrf+getri + logdet LU per step) over random
shapes and inputs — every model kind, maturity counts from 1 (fewer than the state dimension:
the capacitance path) to 96 (the lane-group kernel), short and long panels, NaN columns
(leading, interior, all-NaN), ragged T_use windows, unconstrained and constrained θ.

Rule (tests/test_gpu_parity.py): within 1e-9 of the oracle, relative to the loglik's term scale
(max(|ll|, ½·nterms·N·log 2π): short random panels can sum to ≈ 0); where the two differ by more,
the binary128 restatement (oracle/yfm_truth.c, pinned to the 40-digit dense one) adjudicates: the
kernel must be at least as close to it as the oracle (factor 1, every model kind, TVλ in the
default certified precision).  −Inf / NaN patterns must match exactly.  The same rule with |ll|
alone as the denominator is gated too (round 3: 0 failures over the 62,787 finite candidates of
3,000 cases; 148 of them are within 1e-9 of the oracle only by the term-scale denominator and are
then closer to the truth than the oracle); YFM_SWEEP_REPORT=<file> appends one JSON line per case
(profiles/r3/random_sweep/).

The default suite runs seeds 0-11 plus every seed a 3,000-case sweep has ever failed (KNOWN_HARD:
GNS5 with N ∈ {1, 3, 7, 12, 33, 64} and DNS with N = 1 — ill-conditioned or rank-deficient Z'Z,
evaluated on the double-double capacitance path since round 3) and 4985 (round 6).  TVλ cases are run a second
time in the FP64 mode (`_check_tvl_fp64`: patterns exact, accuracy reported)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import kalman_ld as LD
from oracle.truth import loglik_truth, predict_states_truth, states_truth
from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL
from yfm_amd import synthetic as S
from yfm_amd.params import n_params, transform_params

pytestmark = pytest.mark.gpu

D = ctypes.POINTER(ctypes.c_double)


def c_oracle(kind, space, Y, mats, Th, T_use):
    lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
    Yf = np.asfortranarray(Y)
    Thf = np.asfortranarray(Th)
    N, T = Yf.shape
    P, B = Thf.shape
    out = np.empty(B)
    tu = None if T_use is None else np.ascontiguousarray(T_use, dtype=np.int32)
    lib.yfm_oracle_loglik(kind, space, Yf.ctypes.data_as(D), N, T, np.ascontiguousarray(mats).ctypes.data_as(D),
                          Thf.ctypes.data_as(D), P, B, None if tu is None else tu.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                          out.ctypes.data_as(D), 8)
    return out


def random_case(rng, kind):
    N = int(rng.choice([1, 2, 3, 7, 12, 30, 33, 64, 65, 96]))
    if kind == KIND_TVL:
        N = max(N, 1)
    T = int(rng.choice([1, 2, 3, 5, 17, 40, 90]))
    mats = np.sort(rng.choice(np.arange(1, 361), size=N, replace=False)).astype(np.float64)
    Y = S.simulate_panel(kind, T, maturities=mats, seed=int(rng.integers(1 << 30))).copy(order="F")
    pattern = rng.integers(4)
    if pattern == 1 and T > 3:
        Y[:, rng.choice(T, size=max(1, T // 8), replace=False)] = np.nan
    elif pattern == 2 and T > 1:
        Y[int(rng.integers(N)), 0] = np.nan  # leading partial-NaN column
    B = 24
    scale = 0.02 if kind == KIND_TVL else float(rng.choice([0.03, 0.1]))
    Th = S.theta_batch(kind, B, seed=int(rng.integers(1 << 30)), bad_frac=0.1 if kind != KIND_TVL else 0.0,
                       scale=scale)
    space = int(rng.integers(2))
    if space == 1:
        Th = transform_params(kind, Th)
    T_use = None
    if rng.integers(2) and T > 1:
        T_use = rng.integers(1, T + 1, size=B).astype(np.int32)
    return N, T, mats, Y, Th, space, T_use


# seeds a 3,000-case sweep failed in round 2 (profiles/r2/random_sweep/random3000_last_build.log), and 4985, the one
# failure of round 6's 10,000-case sweep (TVλ, λ ≈ 3.6e304 at the first step: c2·m overflowed, test_gpu_edge.py)
KNOWN_HARD = (244, 405, 1078, 1546, 1603, 1804, 2038, 2473, 2686, 4985)
_N_SEEDS = int(os.environ.get("YFM_RANDOM_SEEDS", "12"))  # a wider sweep on demand
SEEDS = sorted(set(range(_N_SEEDS)) | set(KNOWN_HARD))


@pytest.mark.parametrize("seed", SEEDS)
def test_random_cases_vs_c_oracle(engine, seed):
    rng = np.random.default_rng(1000 + seed)
    kind = [KIND_DNS, KIND_GNS, KIND_TVL][seed % 3]
    N, T, mats, Y, Th, space, T_use = random_case(rng, kind)
    assert Th.shape[0] == n_params(kind)
    engine.set_panel(Y, mats)
    got = engine.loglik(kind, Th, space=space, T_use=T_use)
    ref = c_oracle(kind, space, Y, mats, Th, T_use)
    what = dict(kind=kind, N=N, T=T, space=space, windows=T_use is not None)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), what
    assert not np.isposinf(got).any()
    truth = loglik_truth(kind, Y, mats, Th, space=space, T_use=T_use)
    # −Inf patterns: exact, unless the oracle's FP64 dense determinant has the wrong sign — then the
    # kernel must agree with the binary128 truth (factor-1 adjudication applied to the pattern)
    for b in np.flatnonzero(np.isneginf(got) != np.isneginf(ref)):
        assert np.isneginf(truth[b]) == np.isneginf(got[b]), (what, b, got[b], ref[b], truth[b])
        if np.isfinite(got[b]):
            assert abs(got[b] - truth[b]) <= 1e-9 * abs(truth[b]), (what, b, got[b], truth[b])
    fin = np.isfinite(ref) & np.isfinite(got)
    # error scale: the loglik is a sum of per-step terms −½(log det F + v'F⁻¹v + N log 2π); FP64
    # accuracy is relative to the terms' magnitude, not to a sum that may cancel to ≈ 0 (random
    # short panels do that): scale = max(|ll|, ½·nterms·N·log 2π)
    nobs = np.full(Th.shape[1], T) if T_use is None else T_use
    scale = np.maximum(np.abs(ref), 0.5 * np.maximum(nobs - 2, 0) * N * np.log(2 * np.pi))
    err = np.zeros_like(ref)
    err[fin] = np.abs(got[fin] - ref[fin]) / np.maximum(scale[fin], 1e-300)
    assert np.all((ref[fin] != 0.0) | (got[fin] == 0.0)), what  # loglik exactly 0 (T_use ≤ 2) is exact
    # the same rule with |ll| alone as the denominator
    err_ll = np.zeros_like(ref)
    err_ll[fin] = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    strict_fail = [int(b) for b in np.flatnonzero(fin & (err_ll > 1e-9))
                   if abs(got[b] - truth[b]) > abs(ref[b] - truth[b])]
    relaxed_only = [int(b) for b in np.flatnonzero(fin & (err_ll > 1e-9) & (err <= 1e-9))]
    rep = os.environ.get("YFM_SWEEP_REPORT")
    if rep:
        import json
        with open(rep, "a") as fh:
            fh.write(json.dumps(dict(seed=seed, kind=kind, N=N, T=T, n=int(fin.sum()), strict_fail=strict_fail,
                                     within_only_by_term_scale=relaxed_only, deferred=engine_deferred(engine))) + "\n")
    for b in np.flatnonzero(fin & (err > 1e-9)):
        e_gt = abs(got[b] - truth[b]) / max(abs(truth[b]), scale[b])
        e_or = abs(ref[b] - truth[b]) / max(abs(truth[b]), scale[b])
        assert e_gt <= e_or, (what, b, err[b], e_gt, e_or)
    assert not strict_fail, (what, strict_fail, got[strict_fail], ref[strict_fail], truth[strict_fail])
    if kind == KIND_TVL:
        _check_tvl_fp64(engine, Th, space, T_use, ref, truth, scale, what, seed)


def _check_tvl_fp64(engine, Th, space, T_use, ref, truth, scale, what, seed):
    """The TVλ FP64 mode (yfm_set_precision) on the same case: NaN pattern exact, and a −Inf that differs from the
    FP64 oracle's agrees with the binary128 truth.  Its finite logliks are reported, not gated (YFM_SWEEP_REPORT):
    the capacitance form's v'F⁻¹v = (v'v − u'Wu)/σ² cancels where the start is far from the data, so on such steps the
    FP64 mode is less accurate than the reference's dense FP64 — the certified default is
    the mode the factor-1 rule gates."""
    from yfm_amd import _lib
    old = engine.precision
    engine.precision = _lib.PREC_FP64
    try:
        f = engine.loglik(KIND_TVL, Th, space=space, T_use=T_use)
    finally:
        engine.precision = old
    assert np.array_equal(np.isnan(f), np.isnan(ref)), ("fp64", what)
    assert not np.isposinf(f).any(), ("fp64", what)
    for b in np.flatnonzero(np.isneginf(f) != np.isneginf(ref)):
        assert np.isneginf(truth[b]) == np.isneginf(f[b]), ("fp64", what, b, f[b], ref[b], truth[b])
    rep = os.environ.get("YFM_SWEEP_REPORT")
    if rep:
        import json
        both = np.isfinite(f) & np.isfinite(truth) & np.isfinite(ref)
        sc = np.maximum(np.abs(truth), np.where(np.isfinite(scale), scale, 0.0))
        e64 = np.abs(f[both] - truth[both]) / np.maximum(sc[both], 1e-300)
        eor = np.abs(ref[both] - truth[both]) / np.maximum(sc[both], 1e-300)
        with open(rep, "a") as fh:
            fh.write(json.dumps(dict(seed=seed, fp64=True, n=int(both.sum()), e64=[float(x) for x in e64],
                                     e_oracle=[float(x) for x in eor])) + "\n")


def engine_deferred(engine):
    return engine.last_deferred()


@pytest.mark.parametrize("seed", range(int(os.environ.get("YFM_TRAJ_SEEDS", "6"))))  # a wider sweep on demand
def test_random_trajectories_vs_oracle(engine, seed):
    """predict (NaN-padded horizon, ragged windows) and get_loss_array on random shapes vs the NumPy
    oracle (filter.jl:211-282): normwise 1e-9 per output array; NaN / −Inf patterns exact."""
    from oracle import kalman_oracle as O
    from yfm_amd.params import state_dim
    rng = np.random.default_rng(2000 + seed)
    kind = [KIND_DNS, KIND_GNS, KIND_TVL][seed % 3]
    N = int(rng.choice([1, 3, 7, 30, 65]))
    T = int(rng.choice([2, 5, 17, 40]))
    mats = np.sort(rng.choice(np.arange(1, 361), size=N, replace=False)).astype(np.float64)
    Y = S.simulate_panel(kind, T, maturities=mats, seed=int(rng.integers(1 << 30))).copy(order="F")
    if T > 4 and rng.integers(2):
        Y[:, int(rng.integers(1, T))] = np.nan
    B = 5
    Th = transform_params(kind, S.theta_batch(kind, B, seed=int(rng.integers(1 << 30)), bad_frac=0.0,
                                              scale=0.02 if kind == KIND_TVL else 0.05))
    h = int(rng.integers(1, 5))
    tu = rng.integers(1, T + 1, size=B).astype(np.int32)
    engine.set_panel(Y, mats)
    r = engine.predict(kind, Th, space=1, T_use=tu, horizon=h)
    la = engine.loss_array(kind, Th, space=1, T_use=tu)
    for b in range(B):
        s = O.KalmanState.fresh(kind, mats, state_dim(kind))
        O.set_params(s, Th[:, b])
        ref = O.predict(s, O.pad_nan(Y[:, :tu[b]], h))
        n = tu[b] + h - 1
        # factors and predictions: within 1e-9 of the FP64 oracle or at least as close to the binary128 trajectory
        # (tests/test_gpu_predict.py: assert_close_truth) — every kind: a 600-seed sweep found DNS / GNS5 cases
        # (N = 3 with M = 5, near-singular starts) where the FP64 oracle itself is more than 1e-9 off
        from test_gpu_predict import assert_close_truth
        A = predict_states_truth(kind, Y[:, :tu[b]], mats, Th[:, b], horizon=h)[:n + 1]
        if kind == KIND_TVL:
            tru = {"factors": A[1:].T, "preds": LD.fitted_tvl(mats, A[:n]).T}
        else:
            s = O.KalmanState.fresh(kind, mats, state_dim(kind))
            O.set_params(s, Th[:, b])
            tru = {"factors": A[1:].T, "preds": s.Z @ A[:n].T}
        fin_traj = np.isfinite(ref["factors"]).any()
        for k in ("factors", "preds"):
            if fin_traj:
                assert_close_truth(r[k][:, :n, b], ref[k], tru[k], what=(seed, k, b))
        for k, v in ref.items():
            got = r[k][:, :n, b]
            assert np.array_equal(np.isnan(got), np.isnan(v)), (seed, k, b)
            fin = np.isfinite(v)
            if fin.any() and kind != KIND_TVL and k not in ("factors", "preds"):  # γ and the fixed loadings
                sc = max(np.abs(v[fin]).max(), 1e-300)
                assert np.abs(got[fin] - v[fin]).max() / sc <= 1e-9, (seed, k, b, N, T)
            assert np.isnan(r[k][:, n:, b]).all()
        s = O.KalmanState.fresh(kind, mats, state_dim(kind))
        O.set_params(s, Th[:, b])
        ref_la = O.get_loss_array(s, Y[:, :tu[b]])
        got_la = la[:tu[b] - 1, b]
        if np.isscalar(ref_la):
            assert np.isneginf(got_la).all() or got_la.size == 0, (seed, b)
        elif kind != KIND_TVL and ref_la.size:
            # −v'v/N per step (filter.jl:211-247) from the binary128 states: v_t = y_t − Z β_{t|t−1}
            _, Bt, _ = states_truth(kind, Y[:, :tu[b]], mats, Th[:, b], space=1)
            tru_la = np.zeros(tu[b] - 1)
            for t in range(2, tu[b]):
                v = Y[:, t - 1] - s.Z @ Bt[:, t - 2]
                tru_la[t - 1] = -float(v @ v) / N
            sc = max(np.abs(tru_la).max(), 1e-300)
            e_go = np.abs(got_la - ref_la).max(initial=0.0) / sc
            e_gt = np.abs(got_la - tru_la).max(initial=0.0) / sc
            e_or = np.abs(ref_la - tru_la).max(initial=0.0) / sc
            assert e_go <= 1e-9 or e_gt <= e_or, (seed, b, e_go, e_gt, e_or)
