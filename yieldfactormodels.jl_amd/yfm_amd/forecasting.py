"""Rolling-window re-estimation and forecasting — the caller of the hot path in
``src/forecasting.jl``, batched over the forecast origins.

Reference (paths relative to the reference root):

* ``run_rolling_forecasts`` forecasting.jl:16-51 → :func:`run_rolling_forecasts`
  (window types "expanding", "moving", "both", "no_windowing").
* ``run_forecast_window_database`` forecasting.jl:81-224 — per task (forecast origin)
  ``task_id ∈ in_sample_end:T``: re-estimate with ``run_estimation!`` on
  ``data[:, 1:task_id]`` (both window types: the "moving" branch also passes the expanding
  sample, :165), ``predict`` on ``hcat(window, NaN × (h−1))`` (expanding window
  ``1:task_id``, moving window ``span:task_id``, :141, :161), and store the last h columns,
  rounded to 3 digits (databaseoperations.jl:247-293).  Every task starts from the same
  ``init_params`` (:123, ``read_static_params_from_db`` is the identity for Kalman models).
  Here all tasks' estimation chains run as ONE batched ``yfm_estimate`` call (one device
  launch per optimiser round) and all expanding-window forecasts as ONE ``yfm_predict``
  call with per-task windows (``T_use``).
* ``run_forecast_no_window_database`` forecasting.jl:228-283 → :func:`run_forecast_no_window`.
* The merged-shard CSV exports ``export_all_csv`` (databaseoperations.jl:391-661) are
  written directly from the batched results (:func:`write_window_csvs`); the SQLite shard
  store, mkdir task locks and shuffled task order only coordinate independent processes
  and are replaced by the batch (out of scope).
"""
from __future__ import annotations

import os

import numpy as np

from . import io as _io
from .models import estimate_batch, _engine


def _tails(r: dict, T_b: np.ndarray, h: int) -> dict:
    """The last h columns of every candidate's predict output (columns T_b .. T_b + h − 1)."""
    out = {}
    for k, v in r.items():
        out[k] = np.stack([v[:, T_b[b] - 1:T_b[b] - 1 + h, b] for b in range(v.shape[2])], axis=-1)
    return out


def _estimate_tasks(model, data, tasks, init_params, max_group_iters, group_tol, iterations, group=None):
    start = np.asarray(init_params, dtype=np.float64)
    start = start[:, 0] if start.ndim == 2 else start
    Theta0 = np.repeat(start[:, None], len(tasks), axis=1)

    def estimate(Th, tu):
        return estimate_batch(model, data, Th, T_use=tu, space=1, iterations=iterations,
                              max_group_iters=max_group_iters, tol=group_tol)

    if group is not None:  # one process per GPU: windows split over the ranks, results all-gathered
        import torch
        from . import distributed as D
        r = D.sharded_estimate(Theta0, tasks, estimate, group=group,
                               device=torch.device("cuda", model.device) if torch.cuda.is_available() else None)
    else:
        r = estimate(Theta0, tasks)
    return r["theta_c"], r["ll"], r["status"]


def forecast_windows(model, data, in_sample_end: int, in_sample_start: int, forecast_horizon: int, window_type: str,
                     init_params, max_group_iters: int = 10, group_tol: float = 1e-8, reestimate: bool = True,
                     params=None, iterations: int = 500, estimates=None) -> dict:
    """run_forecast_window_database (forecasting.jl:81-224) for one window type, all tasks at once.
    Returns tasks, params (P × ntasks, constrained), loss (ntasks), status, and the rounded
    per-task records preds / factor_loadings_1 / factor_loadings_2 (N × h × ntasks), factors
    (M × h × ntasks), states (L × h × ntasks)."""
    data = np.asarray(data, dtype=np.float64)
    T = data.shape[1]
    h = int(forecast_horizon)
    tasks = np.arange(in_sample_end, T + 1, dtype=np.int32)
    if estimates is not None:
        th_c, loss, status = estimates
    elif reestimate:
        th_c, loss, status = _estimate_tasks(model, data, tasks, init_params, max_group_iters, group_tol, iterations)
    else:  # params read back per task in the reference (read_params_from_db); given here
        p = np.asarray(params if params is not None else init_params, dtype=np.float64)
        th_c = np.repeat(p.reshape(-1, 1), len(tasks), axis=1) if p.ndim == 1 or p.shape[1] == 1 else p
        loss, status = np.full(len(tasks), np.nan), np.zeros(len(tasks), dtype=np.int32)
    if window_type == "expanding":
        eng = _engine(model, data)
        r = eng.predict(model.kind, th_c, space=1, T_use=tasks, horizon=h)
        rec = _tails(r, tasks, h)
    elif window_type == "moving":
        width = in_sample_end - in_sample_start
        parts = []
        for i, task in enumerate(tasks):
            span = int(task) - width  # forecasting.jl:160 (1-based)
            eng = _engine(model, data[:, span - 1:task])
            parts.append(_tails(eng.predict(model.kind, th_c[:, i:i + 1], space=1, horizon=h),
                                np.array([task - span + 1]), h))
        rec = {k: np.concatenate([p[k] for p in parts], axis=-1) for k in parts[0]}
    else:
        raise ValueError(f"Invalid window type: {window_type}")
    rec = {k: _io.julia_round(v, 3) for k, v in rec.items()}  # databaseoperations.jl:251-255
    return dict(window_type=window_type, tasks=tasks, params=th_c, loss=loss, status=status, **rec)


def _rows(tasks, A):
    """_append_array_rows! (databaseoperations.jl:585-600): rows (task, task + h, A[:, h]...)."""
    K, H, B = A.shape
    out = np.empty((B * H, 2 + K))
    for b in range(B):
        for j in range(H):
            out[b * H + j] = np.concatenate([[tasks[b], tasks[b] + j + 1], A[:, j, b]])
    return out


def write_window_csvs(model, thread_id: str, res: dict) -> dict:
    """export_all_csv (databaseoperations.jl:654-661): forecasts, fitted_params, fl1, fl2, factors, states."""
    os.makedirs(model.base.results_folder or ".", exist_ok=True)
    wt = res["window_type"]
    tasks = res["tasks"].astype(np.float64)

    def path(what):
        return _io.result_path(model, thread_id, f"{wt}_window_{what}.csv")

    def sort_task_target(tbl):  # sortperm by column 2, then (stable) by column 1
        tbl = tbl[np.argsort(tbl[:, 1], kind="stable")]
        return tbl[np.argsort(tbl[:, 0], kind="stable")]

    files = {}
    files["forecasts"] = path("forecasts")
    _io.writedlm(files["forecasts"], sort_task_target(_rows(tasks, res["preds"])))
    files["fitted_params"] = path("fitted_params")
    _io.writedlm(files["fitted_params"], np.column_stack([tasks, res["params"].T]))
    for key, what in (("factor_loadings_1", "fl1"), ("factor_loadings_2", "fl2"), ("factors", "factors"),
                      ("states", "states")):
        files[what] = path(what)
        tbl = _rows(tasks, res[key])
        _io.writedlm(files[what], tbl[np.argsort(tbl[:, 0], kind="stable")])
    return files


def run_forecast_no_window(model, data, thread_id: str, in_sample_end: int, forecast_horizon: int, init_params,
                           max_group_iters: int = 10, group_tol: float = 1e-8, iterations: int = 500,
                           write_csv: bool = True) -> dict:
    """run_forecast_no_window_database (forecasting.jl:228-283): estimate once on data[:, 1:in_sample_end],
    forecast every origin with those parameters; all_results (2+M+L+N) × (h · ntasks), rounded to 3 digits."""
    data = np.asarray(data, dtype=np.float64)
    T = data.shape[1]
    h = int(forecast_horizon)
    start = np.asarray(init_params, dtype=np.float64)
    start = start[:, 0] if start.ndim == 2 else start
    est = estimate_batch(model, data[:, :in_sample_end], start[:, None], space=1, iterations=iterations,
                         max_group_iters=max_group_iters, tol=group_tol)
    params = est["theta_c"][:, 0]
    tasks = np.arange(in_sample_end, T + 1, dtype=np.int32)
    eng = _engine(model, data)
    th = np.repeat(params[:, None], len(tasks), axis=1)
    fc = eng.forecast(model.kind, th, space=1, T_use=tasks, horizon=h)  # (M+L+N) × h × ntasks
    R = fc.shape[0]
    all_results = np.empty((2 + R, h * len(tasks)))
    for i, task in enumerate(tasks):
        sl = slice(i * h, (i + 1) * h)
        all_results[0, sl] = task
        all_results[1, sl] = np.arange(1, h + 1) + task
        all_results[2:, sl] = fc[:, :, i]
    all_results = all_results[:, np.argsort(all_results[1], kind="stable")]
    all_results = all_results[:, np.argsort(all_results[0], kind="stable")]
    all_results = _io.julia_round(all_results, 3)
    full = eng.predict(model.kind, params, space=1, horizon=1)
    filt = _io.julia_round(np.vstack([full["factors"][:, :, 0], full["states"][:, :, 0]]), 3)
    out = dict(params=params, loss=est["ll"][0], status=est["status"][0], all_results=all_results,
               factors_filtered_outofsample=filt)
    if write_csv:
        os.makedirs(model.base.results_folder or ".", exist_ok=True)
        _io.writedlm(_io.result_path(model, thread_id, "expanding_window_forecasts.csv"), all_results.T)
        _io.writedlm(_io.result_path(model, thread_id, "out_params.csv"), params)
        _io.writedlm(_io.result_path(model, thread_id, "factors_filtered_outofsample.csv"), filt)
    return out


def run_rolling_forecasts(model, data, thread_id: str, in_sample_end: int, in_sample_start: int,
                          forecast_horizon: int, init_params, window_type: str = "both", max_group_iters: int = 10,
                          group_tol: float = 1e-8, reestimate: bool = True, params=None, iterations: int = 500,
                          write_csv: bool = True, group=None) -> dict:
    """forecasting.jl:16-51.  Returns {window_type: result dict} (on rank 0 of `group`; {} on the
    other ranks); writes the reference's CSVs when write_csv.  With window_type "both" the per-task estimation (identical for both window types,
    both use the expanding sample) runs once and is shared.  `group`: a torch.distributed process
    group (one process per GPU) over which the per-task estimation chains are split (the
    reference's multi-process task claiming, forecasting.jl:54-79, done as one sharded batch)."""
    if window_type in ("no_windowing", "simulation"):
        return {"expanding": run_forecast_no_window(model, data, thread_id, in_sample_end, forecast_horizon,
                                                    init_params, max_group_iters, group_tol, iterations, write_csv)}
    kinds = {"both": ("expanding", "moving"), "expanding": ("expanding",), "moving": ("moving",)}.get(window_type)
    if kinds is None:
        raise ValueError("Invalid window type")
    data = np.asarray(data, dtype=np.float64)
    tasks = np.arange(in_sample_end, data.shape[1] + 1, dtype=np.int32)
    est = None
    if reestimate:
        est = _estimate_tasks(model, data, tasks, init_params, max_group_iters, group_tol, iterations, group)
    # with a group, every rank holds every task's estimate after the all-gather; the predict pass
    # and the CSV files (one set of paths per model / thread_id) belong to rank 0 alone, so ranks
    # never truncate-and-write the same files concurrently
    lead = group is None or _rank(group) == 0
    out = {}
    if not lead:
        return out
    for wt in kinds:
        res = forecast_windows(model, data, in_sample_end, in_sample_start, forecast_horizon, wt, init_params,
                               max_group_iters, group_tol, reestimate, params, iterations, estimates=est)
        if write_csv:
            res["files"] = write_window_csvs(model, thread_id, res)
        out[wt] = res
    return out


def _rank(group) -> int:
    import torch.distributed as dist
    return dist.get_rank(group)
