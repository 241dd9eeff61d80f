"""GPU parity of the batched estimation driver: yfm_estimate (R
estimate_steps! chains, Nelder–Mead per Optim.jl's published algorithm, every round of all
chains evaluated in one device launch) vs oracle/optim_nm.py (a sequential restatement of
estimate_steps! + Optim.NelderMead).

* Bit for bit when both drive the SAME objective values: the oracle's objective is the
  device loglik of one θ at a time, so any difference is a difference in the optimiser
  state machine (branching, ordering, simplex arithmetic, stopping rules, exceptions).
* Against the fully independent CPU path (oracle chain over the C restatement of the
  reference filter): the final loglik within 1e-9 relative.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import pytest

from conftest import ROOT
from oracle import optim_nm as NM
from yfm_amd import KIND_DNS
from yfm_amd import synthetic as S
from yfm_amd.params import param_layout, transform_params, untransform_params

pytestmark = pytest.mark.gpu


def device_objective(engine, kind, window):
    def f(theta):
        ll = engine.loglik(kind, np.asarray(theta)[:, None], space=0, T_use=None if window is None else [window])[0]
        if math.isnan(ll):
            raise NM.InitThrow()
        return -ll
    return f


@pytest.fixture(scope="module")
def panel():
    return S.simulate_panel(KIND_DNS, 600)[:, :80].copy(order="F"), S.maturities_30()


def test_estimate_bitwise_vs_oracle_chain(engine, panel):
    """Three windows, unconstrained starts, 150 Nelder–Mead iterations × up to 2 group iterations."""
    Y, mats = panel
    engine.set_panel(Y, mats)
    starts = S.theta_batch(KIND_DNS, 3, seed=61, bad_frac=0.0, scale=0.05)
    win = np.array([80, 60, 45], dtype=np.int32)
    got = engine.estimate(KIND_DNS, starts, space=0, T_use=win, iterations=150, max_group_iters=2)
    for r in range(3):
        ref = NM.estimate_steps(device_objective(engine, KIND_DNS, int(win[r])), starts[:, r],
                                transform=lambda x: transform_params(KIND_DNS, x), untransform=lambda x: x,
                                max_group_iters=2, iterations=150)
        assert got["status"][r] == ref.status == 0
        np.testing.assert_array_equal(got["p"][:, r], ref.p)
        assert got["ll"][r] == ref.ll
        np.testing.assert_allclose(got["theta_c"][:, r], ref.theta_c, rtol=1e-15)
        assert np.isfinite(ref.ll) and ref.ll > engine.loglik(KIND_DNS, starts[:, r], space=0, T_use=[win[r]])[0]


def test_estimate_rescaled_start_and_throw(engine, panel):
    """A start whose loglik is −Inf goes through the ×0.95 rescaling (optimization.jl:173-184); a
    constrained start with Φ = I makes compute_loss throw → status 1, NaN outputs."""
    Y, mats = panel
    engine.set_panel(Y, mats)
    cand = S.theta_batch(KIND_DNS, 4096, seed=63, bad_frac=0.05)
    ll = engine.loglik(KIND_DNS, cand, space=0)
    bad = cand[:, np.flatnonzero(np.isneginf(ll))[:1]]
    assert bad.shape[1] == 1
    got = engine.estimate(KIND_DNS, bad, space=0, iterations=60, max_group_iters=1)
    ref = NM.estimate_steps(device_objective(engine, KIND_DNS, None), bad[:, 0],
                            transform=lambda x: transform_params(KIND_DNS, x), untransform=lambda x: x,
                            max_group_iters=1, iterations=60)
    assert got["status"][0] == ref.status
    np.testing.assert_array_equal(got["p"][:, 0], ref.p)
    assert got["ll"][0] == ref.ll or (math.isinf(ref.ll) and got["ll"][0] == ref.ll)

    # constrained Φ = I untransforms to +Inf on the diagonal, which _sanitize_parameters zeroes
    # (optimization.jl:157-162, :422-432): no throw
    th = S.theta0_constrained(KIND_DNS)
    lay = param_layout(KIND_DNS)
    th[lay.phi_offset:lay.phi_offset + 9] = np.eye(3).reshape(-1)
    got = engine.estimate(KIND_DNS, th, space=1, iterations=10, max_group_iters=1)
    assert got["status"][0] == 0 and got["p"][lay.phi_offset, 0] != 0.0
    # an unconstrained start with Φ diagonal 40 decodes to exactly Φ = I: initialize_filter throws
    tu = S.theta0(KIND_DNS)
    tu[lay.phi_offset:lay.phi_offset + 9] = np.eye(3).reshape(-1) * 40.0
    got = engine.estimate(KIND_DNS, tu, space=0, iterations=10, max_group_iters=1)
    assert got["status"][0] == 1 and np.isnan(got["ll"][0]) and np.isnan(got["theta_c"]).all()


def test_estimate_vs_cpu_reference_path(engine, panel):
    """The whole chain on the independent CPU path (the C restatement of the reference filter,
    oracle/yfm_oracle.c, one θ per call) reaches the same optimum."""
    Y, mats = panel
    Y = Y[:, :50].copy(order="F")
    engine.set_panel(Y, mats)
    lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
    D = ctypes.POINTER(ctypes.c_double)

    def f(theta):
        th = np.ascontiguousarray(theta, dtype=np.float64)
        out = np.empty(1)
        lib.yfm_oracle_loglik(KIND_DNS, 0, Y.ctypes.data_as(D), 30, 50, mats.ctypes.data_as(D), th.ctypes.data_as(D),
                              20, 1, None, out.ctypes.data_as(D), 1)
        if math.isnan(out[0]):
            raise NM.InitThrow()
        return -out[0]

    th0 = S.theta0_constrained(KIND_DNS)
    ref = NM.estimate_steps(f, th0, transform=lambda x: transform_params(KIND_DNS, x),
                            untransform=lambda x: untransform_params(KIND_DNS, x), max_group_iters=1, iterations=80)
    got = engine.estimate(KIND_DNS, th0, space=1, iterations=80, max_group_iters=1)
    assert got["status"][0] == ref.status == 0
    assert abs(got["ll"][0] - ref.ll) <= 1e-9 * abs(ref.ll)
    np.testing.assert_allclose(got["theta_c"][:, 0], ref.theta_c, rtol=1e-7, atol=1e-9)


def test_estimate_steps_model_api(engine, panel):
    """estimate_steps!(model, data, all_params, param_groups) returns (init_p, ll, best_p, ir)."""
    from yfm_amd import create_model, estimate_steps_, get_loss, set_params_
    Y, mats = panel
    model, _ = create_model("1C", mats, 30)
    th0 = S.theta0_constrained(KIND_DNS)
    init_p, ll, best_p, ir = estimate_steps_(model, Y, th0[:, None], ["1"] * 20, max_group_iters=1)
    np.testing.assert_allclose(init_p, th0, rtol=1e-14)  # transform(untransform(th0)): rounding only
    set_params_(model, best_p)
    assert abs(get_loss(model, Y) - ll) <= 1e-12 * abs(ll)
    set_params_(model, th0)
    assert ll > get_loss(model, Y)


def test_estimate_init_is_the_rescaled_start(engine, panel):
    """A start whose loglik is not finite (unconstrained Φ₁₁ = 800: from_R_to_11 overflows to
    Inf/Inf = NaN) is multiplied by 0.95 in the unconstrained space until it is (three times here,
    optimization.jl:173-184); the chain's init_p is that start transformed back (:298-302)."""
    from yfm_amd.params import param_layout, transform_params
    Y, mats = panel
    lay = param_layout(KIND_DNS)
    p = S.theta0(KIND_DNS).copy()
    p[lay.phi_offset] = 800.0
    engine.set_panel(Y, mats)
    q = p.copy()
    k = 0
    while not np.isfinite(engine.loglik(KIND_DNS, q, space=0)[0]):
        q = q * 0.95
        k += 1
    assert k == 3
    r = engine.estimate(KIND_DNS, p[:, None], space=0, iterations=20, max_group_iters=1)
    assert r["status"][0] == 0 and np.isfinite(r["ll"][0])
    np.testing.assert_allclose(r["init_c"][:, 0], transform_params(KIND_DNS, q), rtol=1e-13)


def test_speculation_is_bitwise_neutral(engine, panel):
    """Speculation-tree budgets YFM_NM_SPEC = 1 (one iteration per round), 7, 16 (the default) and 32
    nodes: the same chains bit for bit and the same count of consumed evaluations, on 12 windows
    with rescaled and failing starts."""
    import os
    Y, mats = panel
    engine.set_panel(Y, mats)
    starts = S.theta_batch(KIND_DNS, 12, seed=67, bad_frac=0.2, scale=0.08)
    win = np.array([80, 79, 70, 66, 60, 55, 50, 45, 40, 33, 80, 72], dtype=np.int32)
    res = {}
    modes = ("1", "7", "16", "32")
    for mode in modes:
        os.environ["YFM_NM_SPEC"] = mode
        try:
            res[mode] = engine.estimate(KIND_DNS, starts, space=0, T_use=win, iterations=200, max_group_iters=3)
        finally:
            os.environ.pop("YFM_NM_SPEC", None)
    a = res["1"]
    for mode in modes[1:]:
        b = res[mode]
        for k in ("theta_c", "p", "init_c", "ll", "status"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"{k} at {mode} nodes")
        assert a["n_evals"] == b["n_evals"]


@pytest.mark.parametrize("switch", [{"YFM_EST_GROUPS": "1"}, {"YFM_EST_GROUPS": "3"}, {"YFM_EST_ZEROCOPY": "0"},
                                    {"YFM_EST_THREADS": "1"}, {"YFM_EST_STATS": "1"}])
def test_estimator_tuning_switches_are_bitwise_neutral(engine, panel, switch):
    """The estimator's tuning switches (csrc/yfm_estimate.hip: chain groups on their own streams, zero-copy
    page-locked rounds, host threads, the per-phase statistics print) change how a round is scheduled, never
    what a chain computes: 40 windows (two chain groups by default) give the same chains bit for bit and the
    same evaluation count as the defaults."""
    import os
    Y, mats = panel
    engine.set_panel(Y, mats)
    starts = S.theta_batch(KIND_DNS, 40, seed=73, bad_frac=0.1, scale=0.08)
    win = (80 - np.arange(40) % 30).astype(np.int32)
    a = engine.estimate(KIND_DNS, starts, space=0, T_use=win, iterations=60, max_group_iters=2)
    os.environ.update(switch)
    try:
        b = engine.estimate(KIND_DNS, starts, space=0, T_use=win, iterations=60, max_group_iters=2)
    finally:
        for k in switch:
            os.environ.pop(k, None)
    for k in ("theta_c", "p", "init_c", "ll", "status"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"{k} with {switch}")
    assert a["n_evals"] == b["n_evals"] > 0


@pytest.mark.parametrize("kind_name", ["GNS5", "TVL"])
def test_speculation_tree_other_models(engine, panel, kind_name):
    """The speculation tree on the larger simplices (GNS5: 48 parameters, TVλ: 31, certified
    precision): budgets 1 and 16 give the same chains bit for bit and the same evaluation count."""
    import os
    from yfm_amd import KIND_GNS, KIND_TVL
    kind = {"GNS5": KIND_GNS, "TVL": KIND_TVL}[kind_name]
    Y, mats = panel
    Y = Y[:, :40].copy(order="F")
    engine.set_panel(Y, mats)
    starts = S.theta_batch(kind, 3, seed=71, bad_frac=0.0, scale=0.05)
    win = np.array([40, 33, 25], dtype=np.int32)
    res = {}
    for mode in ("1", "16"):
        os.environ["YFM_NM_SPEC"] = mode
        try:
            res[mode] = engine.estimate(kind, starts, space=0, T_use=win, iterations=40, max_group_iters=2)
        finally:
            os.environ.pop("YFM_NM_SPEC", None)
    a, b = res["1"], res["16"]
    for k in ("theta_c", "p", "init_c", "ll", "status"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert a["n_evals"] == b["n_evals"] and a["n_evals"] > 0
    assert np.isfinite(a["ll"]).all()


def test_rolling_forecasts_driver(engine, tmp_path):
    """run_rolling_forecasts (forecasting.jl:16-51, :81-224) for "both" window types, single process:
    the batched per-task estimation equals each task's chain run alone, the forecast records equal
    the oracle's predict on hcat(window, NaN × (h−1)) rounded to 3 digits (databaseoperations.jl:
    251-255), and the six export CSVs per window type have the reference's names and layouts
    (databaseoperations.jl:391-661).  (tests/test_gpu_multirank.py checks that 2 ranks give the
    same files; this test pins those files to the reference's semantics.)"""
    from oracle import kalman_oracle as O
    from yfm_amd import create_model
    from yfm_amd import io as yio
    from yfm_amd.forecasting import run_rolling_forecasts
    mats = S.maturities_30()
    Y = S.simulate_panel(KIND_DNS, 600)[:, :56].copy(order="F")
    model, _ = create_model("1C", mats, 30, results_location=str(tmp_path) + "/")
    th0 = S.theta0_constrained(KIND_DNS)
    h = 3
    out = run_rolling_forecasts(model, Y, "9", 50, 11, h, th0[:, None], window_type="both", max_group_iters=1,
                                iterations=25)
    ex, mv = out["expanding"], out["moving"]
    tasks = np.arange(50, 57)
    np.testing.assert_array_equal(ex["tasks"], tasks)
    np.testing.assert_array_equal(ex["params"], mv["params"])  # both use the expanding sample (:165)
    engine.set_panel(Y, mats)  # the moving-window forecasts left a window panel on the engine
    one = engine.estimate(KIND_DNS, th0, space=1, T_use=[53], iterations=25, max_group_iters=1)
    np.testing.assert_array_equal(one["theta_c"][:, 0], ex["params"][:, 3])
    assert one["ll"][0] == ex["loss"][3]
    for i, task in enumerate(tasks):
        for wt, res, lo in (("expanding", ex, 0), ("moving", mv, task - 39 - 1)):
            s = O.KalmanState.fresh(KIND_DNS, mats, 3)
            O.set_params(s, res["params"][:, i])
            r = O.predict(s, O.pad_nan(Y[:, lo:task], h))
            for k in ("preds", "factors", "factor_loadings_1"):
                ref = yio.julia_round(r[k][:, -h:], 3)
                assert np.abs(res[k][:, :, i] - ref).max() <= 1.0001e-3, (wt, k, task)
                assert (res[k][:, :, i] == ref).mean() > 0.9
    for wt in ("expanding", "moving"):
        f = yio.readdlm(tmp_path / f"1C__thread_id__9__{wt}_window_forecasts.csv")
        assert f.shape == (len(tasks) * h, 2 + 30)
        np.testing.assert_array_equal(f[:4, :2], [[50, 51], [50, 52], [50, 53], [51, 52]])
        p = yio.readdlm(tmp_path / f"1C__thread_id__9__{wt}_window_fitted_params.csv")
        assert p.shape == (len(tasks), 21)
        np.testing.assert_array_equal(p[:, 0], tasks)
        for what, rows in (("fl1", 30), ("fl2", 30), ("factors", 3), ("states", 1)):
            t = yio.readdlm(tmp_path / f"1C__thread_id__9__{wt}_window_{what}.csv")
            assert t.shape == (len(tasks) * h, 2 + rows), (wt, what, t.shape)
