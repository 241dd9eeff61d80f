"""GPU parity of the trajectory outputs: predict, the forecast
blocks of the rolling-window driver, and get_loss_array — libyfm_hip.so through the C ABI
vs the committed fixtures (tests/golden/traj) and the live NumPy oracle.

Tolerance: 1e-9 relative, normwise per output array (scale = max |expected|); the NaN
pattern (columns beyond a window, init throws) and −Inf rows must match exactly.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import kalman_oracle as O
from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL
from yfm_amd import synthetic as S
from yfm_amd.params import gamma_dim, param_layout, state_dim, transform_params

pytestmark = pytest.mark.gpu

REL = 1e-9
KEYS = ("preds", "factors", "states", "factor_loadings_1", "factor_loadings_2")
TRAJ = sorted(p.stem for p in (GOLDEN / "traj").glob("*.npz"))


def load(name):
    with np.load(GOLDEN / "traj" / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def assert_close(got, ref, rel=REL, what=""):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    assert np.array_equal(np.isnan(got), np.isnan(ref)), what
    assert np.array_equal(np.isneginf(got), np.isneginf(ref)), what
    fin = np.isfinite(ref)
    if fin.any():
        scale = np.abs(ref[fin]).max()
        err = np.abs(got[fin] - ref[fin]).max() / (scale if scale > 0 else 1.0)
        assert err <= rel, (what, err)


def oracle_state(kind, mats, theta_c):
    s = O.KalmanState.fresh(kind, mats, state_dim(kind))
    O.set_params(s, theta_c)
    return s


@pytest.mark.parametrize("name", TRAJ)
def test_traj_golden(engine, name):
    g = load(name)
    kind, h = int(g["kind"]), int(g["horizon"])
    engine.set_panel(g["Y"], g["maturities"])
    r = engine.predict(kind, g["Theta"], space=1, T_use=g["T_use"], horizon=h)
    for k in KEYS:
        assert_close(r[k], g[f"predict_{k}"], what=k)
    assert_close(engine.forecast(kind, g["Theta"], space=1, T_use=g["T_use"], horizon=h), g["forecast"], what="fc")
    assert_close(engine.loss_array(kind, g["Theta"], space=1, T_use=g["T_use"]), g["loss_array_K1"], what="K1")
    assert_close(engine.loss_array(kind, g["Theta"], space=1, K=2), g["loss_array_K2"], what="K2")


@pytest.fixture(scope="module")
def panel():
    Y = S.simulate_panel(KIND_DNS, 600)[:, :150].copy(order="F")
    return Y, S.maturities_30()


def test_predict_headline_shape_vs_oracle(engine, panel):
    """N = 30, ragged expanding windows, 12-month forecast horizon (forecasting.jl:141), incl. a
    NaN column inside the data (prediction-only step)."""
    Y, mats = panel
    Y = Y.copy(order="F")
    Y[:, 70] = np.nan
    Th = transform_params(KIND_DNS, S.theta_batch(KIND_DNS, 6, seed=51, bad_frac=0.0, scale=0.05))
    tu = np.array([150, 149, 100, 71, 70, 12], dtype=np.int32)
    h = 12
    engine.set_panel(Y, mats)
    r = engine.predict(KIND_DNS, Th, space=1, T_use=tu, horizon=h)
    fc = engine.forecast(KIND_DNS, Th, space=1, T_use=tu, horizon=h)
    for b in range(6):
        ref = O.predict(oracle_state(KIND_DNS, mats, Th[:, b]), O.pad_nan(Y[:, :tu[b]], h))
        n = tu[b] + h - 1
        for k in KEYS:
            assert_close(r[k][:, :n, b], ref[k], what=(k, b))
            assert np.isnan(r[k][:, n:, b]).all()
        # the forecast block is predict's tail, bit for bit (same recursion, same arithmetic)
        tail = np.vstack([r["factors"][:, n - h:n, b], r["states"][:, n - h:n, b], r["preds"][:, n - h:n, b]])
        np.testing.assert_array_equal(fc[:, :, b], tail)


def test_predict_alignment_identity(engine, panel):
    """preds[:, j] = Z · factors[:, j−1] (both are the state after step j; filter.jl:264-279)."""
    Y, mats = panel
    th = S.theta0_constrained(KIND_DNS)
    engine.set_panel(Y[:, :60], mats)
    r = engine.predict(KIND_DNS, th, space=1)
    Z = np.ones((30, 3))
    O.dns_loadings(th[0], mats, Z)
    np.testing.assert_allclose(r["preds"][:, 1:, 0], Z @ r["factors"][:, :-1, 0], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(r["factor_loadings_1"][:, 5, 0], Z[:, 1], rtol=1e-15)
    assert (r["states"][0, :, 0] == th[0]).all()


def assert_close_truth(got, oracle, truth, what=""):
    """Trajectory parity (normwise per array, scale = max |truth|): within 1e-9 of the FP64 oracle,
    or at least as close to the binary128 truth (oracle/yfm_truth.c) as the oracle is."""
    assert np.array_equal(np.isnan(got), np.isnan(oracle)), what
    fin = np.isfinite(oracle)
    scale = np.abs(truth[fin]).max()
    e_go = np.abs(got[fin] - oracle[fin]).max() / scale
    e_gt = np.abs(got[fin] - truth[fin]).max() / scale
    e_or = np.abs(oracle[fin] - truth[fin]).max() / scale
    assert e_go <= REL or e_gt <= e_or, (what, e_go, e_gt, e_or)


def _tvl_loadings(mats, A):
    with np.errstate(all="ignore"):
        tau = (0.01 + np.exp(A[..., 3:4])) * mats
        z = np.exp(-tau)
        s = (1 - z) / tau
    return s, s - z


@pytest.mark.parametrize("kind", [KIND_GNS, KIND_TVL])
def test_predict_other_kinds_vs_oracle(engine, kind):
    from oracle import kalman_ld as LD
    from oracle.truth import predict_states_truth
    mats = S.maturities_30() if kind == KIND_GNS else np.arange(1, 31, dtype=np.float64) * 2.0
    Y = S.simulate_panel(kind, 50, maturities=mats)
    scale = 0.05 if kind == KIND_GNS else 0.02
    Th = transform_params(kind, S.theta_batch(kind, 4, seed=53, bad_frac=0.0, scale=scale))
    engine.set_panel(Y, mats)
    h = 6
    r = engine.predict(kind, Th, space=1, horizon=h)
    for b in range(4):
        ref = O.predict(oracle_state(kind, mats, Th[:, b]), O.pad_nan(Y, h))
        if kind == KIND_GNS:
            for k in KEYS:
                assert_close(r[k][..., b], ref[k], what=(kind, k, b))
            continue
        n = ref["factors"].shape[1]
        A = predict_states_truth(kind, Y, mats, Th[:, b], horizon=h)
        tru = {"factors": A[1:n + 1].T, "preds": LD.fitted_tvl(mats, A[:n]).T}
        (tru["factor_loadings_1"], tru["factor_loadings_2"]) = (x.T for x in _tvl_loadings(mats, A[:n]))
        for k in ("factors", "preds", "factor_loadings_1", "factor_loadings_2"):
            assert_close_truth(r[k][..., b], ref[k], tru[k], what=(k, b))
        np.testing.assert_array_equal(r["states"][..., b], 0.0)  # TVλ base.gamma is never set
    assert r["states"].shape[0] == gamma_dim(kind)


def test_loss_array_vs_oracle(engine, panel):
    Y, mats = panel
    Th = transform_params(KIND_DNS, S.theta_batch(KIND_DNS, 5, seed=57, bad_frac=0.0, scale=0.05))
    engine.set_panel(Y, mats)
    for K in (1, 3):
        got = engine.loss_array(KIND_DNS, Th, space=1, K=K)
        for b in range(5):
            assert_close(got[:, b], O.get_loss_array(oracle_state(KIND_DNS, mats, Th[:, b]), Y, K=K), what=(K, b))
    tu = np.array([150, 90, 2, 3, 149], dtype=np.int32)
    got = engine.loss_array(KIND_DNS, Th, space=1, T_use=tu)
    for b in range(5):
        ref = O.get_loss_array(oracle_state(KIND_DNS, mats, Th[:, b]), Y[:, :tu[b]])
        assert_close(got[:tu[b] - 1, b], ref, what=("win", b))
        assert np.isnan(got[tu[b] - 1:, b]).all()


def test_loss_array_neg_inf_and_init_throw(engine, panel):
    """A NaN data column at t > 1 makes the reference return the scalar −Inf (filter.jl:234-236);
    a singular I − Φ makes initialize_filter throw (NaN + flag)."""
    from yfm_amd import SingularException, create_model, get_loss_array, set_params_
    Y, mats = panel
    Yn = Y[:, :40].copy(order="F")
    Yn[:, 20] = np.nan
    Th = np.stack([S.theta0_constrained(KIND_DNS)] * 3, axis=1)
    lay = param_layout(KIND_DNS)
    Th[lay.phi_offset:lay.phi_offset + 9, 2] = np.eye(3).reshape(-1)  # Φ = I
    engine.set_panel(Yn, mats)
    got = engine.loss_array(KIND_DNS, Th, space=1)
    assert np.isneginf(got[:, :2]).all() and np.isnan(got[:, 2]).all()
    assert engine.last_flags() == (1, 2)
    assert O.get_loss_array(oracle_state(KIND_DNS, mats, Th[:, 0]), Yn) == -np.inf
    model, _ = create_model("1C", mats, 30)
    set_params_(model, Th[:, 0])
    assert get_loss_array(model, Yn) == -np.inf
    set_params_(model, Th[:, 2])
    with pytest.raises(SingularException):
        get_loss_array(model, Y[:, :40])
    r = engine.predict(KIND_DNS, Th, space=1, horizon=2)
    assert np.isnan(r["preds"][..., 2]).all() and np.isfinite(r["preds"][..., 0]).all()


def test_model_api_predict(engine, panel):
    """predict(model, data) returns the reference's named tuple for the model's parameters."""
    from yfm_amd import create_model, predict, set_params_
    Y, mats = panel
    model, _ = create_model("1C", mats, 30)
    th = S.theta0_constrained(KIND_DNS)
    set_params_(model, th)
    r = predict(model, Y[:, :80])
    ref = O.predict(oracle_state(KIND_DNS, mats, th), Y[:, :80])
    for k in KEYS:
        assert_close(r[k], ref[k], what=k)
    assert r["preds"].shape == (30, 80) and r["factors"].shape == (3, 80)


def test_trajectory_api_errors(engine, panel):
    """Invalid requests return the documented status and message (include/yfm.h), never a kernel."""
    import ctypes
    from yfm_amd import _lib
    Y, mats = panel
    engine.set_panel(Y[:, :30], mats)
    lib = engine.lib
    th = np.ascontiguousarray(np.tile(S.theta0_constrained(KIND_DNS)[:, None], (1, 2)).T)
    out = np.zeros(4096)
    D = _lib.dptr
    assert lib.yfm_predict(engine.ctx, 0, 1, D(th), 20, 2, None, 0, D(out), D(out), D(out), None, None) == -1
    assert b"horizon" in lib.yfm_last_error()
    assert lib.yfm_forecast(engine.ctx, 0, 1, D(th), 20, 2, None, 0, D(out)) == -1
    assert lib.yfm_loss_array(engine.ctx, 0, 1, D(th), 20, 2, None, 0, D(out)) == -1
    tu = np.array([10, 20], dtype=np.int32)
    assert lib.yfm_loss_array(engine.ctx, 0, 1, D(th), 20, 2, _lib.iptr(tu), 2, D(out)) == -4  # EUNSUPPORTED
    assert lib.yfm_predict(engine.ctx, 0, 1, D(th), 19, 2, None, 1, D(out), D(out), D(out), None, None) == -1
    bad = np.array([0, 5], dtype=np.int32)
    assert lib.yfm_forecast(engine.ctx, 0, 1, D(th), 20, 2, _lib.iptr(bad), 2, D(out)) == -1
    st = np.zeros(2, dtype=np.int32)
    ll = np.zeros(2)
    assert lib.yfm_estimate(engine.ctx, 0, 1, D(th), 20, 2, None, 10, 1e-6, 0, 1e-8, D(out), None, None, D(ll),
                            _lib.iptr(st), None) == -1  # max_group_iters < 1
    assert lib.yfm_estimate(engine.ctx, 0, 5, D(th), 20, 2, None, 10, 1e-6, 1, 1e-8, D(out), None, None, D(ll),
                            _lib.iptr(st), None) == -1  # param_space
    assert lib.yfm_gamma_dim(0) == 1 and lib.yfm_gamma_dim(1) == 1 and lib.yfm_gamma_dim(2) == 2
    assert lib.yfm_gamma_dim(7) == -1
    # B = 0 is a valid empty request
    assert lib.yfm_predict(engine.ctx, 0, 1, D(th), 20, 0, None, 1, D(out), D(out), D(out), None, None) == 0
