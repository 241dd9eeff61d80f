"""The reference's one-call driver end to end (yfm_amd.run ↔ YieldFactorModels.run, src/YieldFactorModels.jl:
221-347) on a small CSV panel in the reference's file layout: load_data → create_model →
load_initial_parameters! → estimate_steps! → save_results (in/out of sample) → get_loss_array →
run_rolling_forecasts.  The written files are checked against the oracle's predict / get_loss /
get_loss_array (oracle/kalman_oracle.py) for the parameters the run wrote, and the estimate against a
direct batched estimation call."""
from __future__ import annotations

import numpy as np
import pytest

from yfm_amd import KIND_DNS
from yfm_amd import io as yio
from yfm_amd import synthetic as S

pytestmark = pytest.mark.gpu


def _write_inputs(root, tid, Y, mats, th0):
    d = root / "YieldFactorModels.jl" / "data"
    d.mkdir(parents=True)
    yio.writedlm(d / f"thread_id__{tid}__data.csv", Y)
    yio.writedlm(d / f"thread_id__{tid}__maturities.csv", mats)
    i = root / "YieldFactorModels.jl" / "initializations" / "1C"
    i.mkdir(parents=True)
    yio.writedlm(i / "init_params_1C.csv", th0[:, None])


def test_run_end_to_end(engine, tmp_path, monkeypatch):
    from oracle import kalman_oracle as O
    import yfm_amd
    monkeypatch.chdir(tmp_path)
    mats = S.maturities_30()
    T, ise, h = 72, 60, 3
    Y = S.simulate_panel(KIND_DNS, 600)[:, :T].copy(order="F")
    th0 = S.theta0_constrained(KIND_DNS)
    _write_inputs(tmp_path, "7", Y, mats, th0)
    model = yfm_amd.run("7", ise, h, True, "1C", window_type="expanding", max_group_iters=1, iterations=40)
    info = model.last_run
    res = tmp_path / "YieldFactorModels.jl" / "results" / "thread_id__7" / "1C"
    pre = str(res / "1C__thread_id__7__")
    # estimation = the batched estimator on data[:, 1:in_sample_end] from the init file's start
    engine.set_panel(Y[:, :ise], mats)
    one = engine.estimate(KIND_DNS, th0, space=1, iterations=40, max_group_iters=1)
    np.testing.assert_array_equal(info["params"], one["theta_c"][:, 0])
    out_params = yio.readdlm(pre + "out_params.csv").reshape(-1)
    np.testing.assert_array_equal(out_params, info["params"])
    np.testing.assert_array_equal(model.base.flat_params, info["params"])
    # in-sample loglik (loss.csv of the out-of-sample save, io.jl:27) vs the oracle's get_loss
    s = O.KalmanState.fresh(KIND_DNS, mats, 3)
    O.set_params(s, out_params)
    ll = O.get_loss(s, Y[:, :ise])
    assert abs(yio.readdlm(pre + "loss.csv")[0, 0] - ll) <= 1e-9 * abs(ll)
    # filtered factors / fits of both saves vs the oracle's predict
    for dt, lo_hi in (("insample", ise), ("outofsample", T)):
        s = O.KalmanState.fresh(KIND_DNS, mats, 3)
        O.set_params(s, out_params)
        r = O.predict(s, Y[:, :lo_hi])
        fac = yio.readdlm(pre + f"factors_filtered_{dt}.csv")
        fit = yio.readdlm(pre + f"fit_filtered_{dt}.csv")
        assert fac.shape == (lo_hi, 3 + 1) and fit.shape == (lo_hi, 30)
        np.testing.assert_allclose(fac[:, :3], r["factors"].T, rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(fit, r["preds"].T, rtol=1e-9, atol=1e-12)
    # out-of-sample loss array means (loss_array[in_sample_end+1:end])
    s = O.KalmanState.fresh(KIND_DNS, mats, 3)
    O.set_params(s, out_params)
    la = O.get_loss_array(s, Y)
    np.testing.assert_allclose(info["loss_array"], la, rtol=1e-9)
    assert abs(info["oos_loss_means"]["full"] - la[ise:].mean()) <= 1e-9 * abs(la[ise:].mean())
    # rolling expanding-window forecasts: tasks in_sample_end..T, h rows each
    f = yio.readdlm(pre + "expanding_window_forecasts.csv")
    assert f.shape == ((T - ise + 1) * h, 2 + 30)
    np.testing.assert_array_equal(f[:h, :2], [[ise, ise + 1], [ise, ise + 2], [ise, ise + 3]])
    assert np.isfinite(f).all()
