"""The reference's one-call driver, `YieldFactorModels.run` (src/YieldFactorModels.jl:221-347), for the
Kalman models, on the reference's file layout.

    run(thread_id, in_sample_end, forecast_horizon, run_rolling, model_type, float_type; …) → model

chains, exactly as the reference does (line numbers of src/YieldFactorModels.jl):
  setup_data_paths (:88-98) → load_data (:261, data_management.jl:1-5) → create_model (:268,
  results folder "<results_location><model_type>/") → get_param_groups (:273, kalmanbasemodel.jl:150-159)
  → load_initial_parameters! (:131-155: init_params_<model_type>.csv from the model's init folder, or a
  random start written there) → set_params! (:275) → load_static_parameters! (:105-119) →
  run_estimation! (:162-186 → estimate_steps!) → save_results "insample" / get_loss / save_results
  "outofsample" / get_loss_array (:304-328) → run_rolling_forecasts (:333-344).
Every loglik, predict, loss array and estimation round runs in libyfm_hip.so (the batched boundary);
this module is file plumbing and control flow only.

Differences, stated: the computation is Float64 only (the reference's `float_type` default is Float32,
which the MI355X path does not offer: `create_model` rejects it); a missing init file is replaced by
`rand(P, 1)` from numpy's generator seeded with `seed` (Julia's MersenneTwister stream is not
reproduced); the printed progress lines follow the reference's wording.
"""
from __future__ import annotations

import os

import numpy as np

from . import io as _io
from .forecasting import run_rolling_forecasts
from .models import (AbstractKalmanModel, DNSModel, TVLambdaDNSModel, create_model, estimate_steps_, get_loss,
                     get_loss_array, get_params, predict, set_params_)


def setup_data_paths(model_type: str, simulation: bool, scratch_dir: str, thread_id: str):
    """YieldFactorModels.jl:88-98 → (data_folder, results_location)."""
    if simulation:
        return (f"{scratch_dir}YieldFactorModels.jl/data_simulation/",
                f"{scratch_dir}YieldFactorModels.jl/results_simulation/thread_id__{thread_id}/")
    return (f"{scratch_dir}YieldFactorModels.jl/data/",
            f"{scratch_dir}YieldFactorModels.jl/results/thread_id__{thread_id}/")


def init_folder(model: AbstractKalmanModel) -> str:
    """kalmanbasemodel.jl:122 — relative to the working directory, as in the reference."""
    return f"YieldFactorModels.jl/initializations/{model.base.model_string}/"


def get_param_groups(model: AbstractKalmanModel, param_groups) -> list[str]:
    """kalmanbasemodel.jl:150-159: the given groups if there is one per parameter, else all "1"."""
    n = len(get_params(model))
    groups = list(param_groups or [])
    if len(groups) == n:
        return groups
    print("Default param groups assigned.")
    return ["1"] * n


def load_initial_parameters_(model: AbstractKalmanModel, model_type: str, float_type=np.float64,
                             simulation: bool = False, rng: np.random.Generator | None = None) -> np.ndarray:
    """YieldFactorModels.jl:131-155: init_params_<model_type>[_simulation].csv from the model's init folder
    (P × n_starts, constrained), or — when it cannot be read — a random P×1 start in [0, 1), written there."""
    folder = init_folder(model)
    path = os.path.join(folder, f"init_params_{model_type}.csv")
    sim = os.path.join(folder, f"init_params_{model_type}_simulation.csv")
    try:
        return _io.readdlm(sim if simulation and os.path.isfile(sim) else path)
    except (OSError, ValueError):
        print(f"Initial parameters for {model_type} not found in {folder}. Writing file with random initial "
              "parameters...")
        n = len(get_params(model))
        print(f"Number of parameters: {n}")
        rng = rng if rng is not None else np.random.default_rng()
        all_params = rng.random((n, 1)).astype(float_type)
        os.makedirs(folder, exist_ok=True)
        _io.writedlm(path, all_params)
        return all_params


def static_model_type(model: AbstractKalmanModel) -> str | None:
    """get_static_model_type: dns.jl:46-48 ("DNS"), tvλdns.jl:48-50 ("1C")."""
    if isinstance(model, DNSModel):
        return "DNS"
    if isinstance(model, TVLambdaDNSModel):
        return "1C"
    return None


def initialize_with_static_params(model: AbstractKalmanModel, params: np.ndarray, static: np.ndarray) -> np.ndarray:
    """paramoperations.jl:78-90 (TVλ from a fitted 3-factor DNS): σ², the 3×3 block of U, δ[1:3] and the
    3×3 block of Φ taken from the DNS parameter vector (1-based: params[1] = static[2], params[2:7] =
    static[end-17:end-12], params[12:14] = static[end-11:end-9], Φ rows at 16:18, 20:22, 24:26)."""
    s = np.asarray(static, dtype=np.float64).reshape(-1)
    p = np.array(params, dtype=np.float64, copy=True)
    n = s.size
    p[0:1] = s[1:2]
    p[1:7] = s[n - 18:n - 12]
    p[11:14] = s[n - 12:n - 9]
    p[15:18] = s[n - 9:n - 6]
    p[19:22] = s[n - 6:n - 3]
    p[23:26] = s[n - 3:n]
    return p


def load_static_parameters_(model: AbstractKalmanModel, model_type: str, results_location: str, thread_id: str,
                            params: np.ndarray) -> np.ndarray:
    """YieldFactorModels.jl:105-119: the static model's fitted parameters
    (<results_location><static>/<static>__thread_id__<id>__out_params.csv) mapped into this model's start.
    The reference defines the mapping only for TVλ (paramoperations.jl:78); for DNS the call ends in its
    catch (a warning, the parameters unchanged) whether or not the file exists."""
    name = static_model_type(model)
    path = f"{results_location}{name}/{name}__thread_id__{thread_id}__out_params.csv"
    try:
        static = _io.readdlm(path)
        if not isinstance(model, TVLambdaDNSModel):
            raise NotImplementedError("initialize_with_static_params has no method for this model")
        return initialize_with_static_params(model, params, static)
    except (OSError, ValueError, NotImplementedError):
        print(f"Warning: Static parameters for {model_type} not found, using default initialization.")
        return params


def run_estimation_(model: AbstractKalmanModel, data, in_sample_end: int, all_params, param_groups,
                    max_group_iters: int, group_tol: float, printing: bool = True, iterations: int = 500):
    """YieldFactorModels.jl:162-186 (Kalman models: grouped estimation, estimate_steps! on
    data[:, 1:in_sample_end]).  Like the reference's last compute_loss call, the model is left holding
    the estimated parameters."""
    if not param_groups:
        raise NotImplementedError("estimate! (LBFGS, ungrouped) is not used by the Kalman models")
    if any(g != "1" for g in param_groups):
        raise NotImplementedError("Kalman models estimate every parameter in group \"1\"")
    init_p, ll, best_p, ir = estimate_steps_(model, data[:, :in_sample_end], np.asarray(all_params, dtype=np.float64),
                                             param_groups, max_group_iters=max_group_iters, tol=group_tol,
                                             printing=printing, iterations=iterations)
    set_params_(model, best_p)
    return init_p, ll, best_p, ir


def _rank(group) -> int:
    import torch.distributed as dist
    return dist.get_rank(group)


def _broadcast_obj(obj, group):
    """Rank 0's object on every rank of `group` (a pickled object broadcast; a few hundred bytes)."""
    import torch.distributed as dist
    box = [obj]
    dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return box[0]


def _broadcast_from_lead(arr, group) -> np.ndarray:
    """Rank 0's array on every rank of `group`."""
    return np.array(_broadcast_obj(arr, group), dtype=np.float64)


def run(thread_id: str = "1", in_sample_end: int = 100, forecast_horizon: int = 12, run_rolling: bool = True,
        model_type: str = "1C", float_type=np.float64, *, window_type: str = "both", in_sample_start: int = 1,
        param_groups=(), max_group_iters: int = 10, group_tol: float = 1e-8, run_optimization: bool = True,
        save_results_bool: bool = True, simulation: bool = False, reestimate: bool = True, scratch_dir: str = "",
        seed: int = 43, iterations: int = 500, group=None):
    """YieldFactorModels.run (src/YieldFactorModels.jl:221-347) for the Kalman model codes ("1C"/"0",
    "TVλ"/"1", and this build's "GNS5").  Returns the model; `model.last_run` holds the numbers the
    reference prints (estimation loss, in-sample loglik, out-of-sample loss-array means) and the paths
    written.  `iterations` is the NelderMead budget per group (the reference's opt1: 500); `group` a
    torch.distributed group over which the rolling re-estimation chains are split (one process per GPU)."""
    if simulation:  # :245-250
        window_type = "simulation"
        run_optimization = False
        run_rolling = True
        save_results_bool = False
    rng = np.random.default_rng(seed)  # Random.seed!(seed), :252
    data_folder, results_location = setup_data_paths(model_type, simulation, scratch_dir, thread_id)
    data, maturities = _io.load_data(data_folder, thread_id)
    data = np.asarray(data, dtype=float_type)
    maturities = np.asarray(maturities, dtype=float_type).reshape(-1)
    N, M = len(maturities), 3  # :266-267
    model, model_type = create_model(model_type, maturities, N, M, float_type,
                                     results_location=f"{results_location}{model_type}/")
    param_groups = get_param_groups(model, param_groups)
    # With a group, rank 0 alone reads (or writes) the init file and every file below; the start is then
    # broadcast, so no rank reads a file another one is still writing; the in-sample estimation runs on rank 0
    # and its result is broadcast too.
    lead = group is None or _rank(group) == 0
    all_params = None
    if lead:
        all_params = np.array(load_initial_parameters_(model, model_type, float_type, simulation, rng),
                              dtype=np.float64)
        if all_params.ndim == 1:
            all_params = all_params[:, None]
    if group is not None:
        all_params = _broadcast_from_lead(all_params, group)
    save_results_bool = save_results_bool and lead
    set_params_(model, all_params[:, 0])
    all_params[:, 0] = load_static_parameters_(model, model_type, results_location, thread_id, all_params[:, 0])
    info = {"files": []}
    if run_optimization:
        # the in-sample estimation runs on the lead rank only; the other ranks take its result (every
        # rank used to run the whole NelderMead and discard it, relying on bitwise-equal results across devices)
        est = None
        if lead:
            print("The param groups are : ", param_groups)
            est = run_estimation_(model, data, in_sample_end, all_params, param_groups, max_group_iters, group_tol,
                                  iterations=iterations)
            est = (np.asarray(est[0], dtype=np.float64), float(est[1]), np.asarray(est[2], dtype=np.float64),
                   est[3])
        if group is not None:
            est = _broadcast_obj(est, group)
        init_params, loss, params, ir = est
        set_params_(model, params)  # as run_estimation_ leaves the lead's model
    else:
        init_params = params = all_params[:, 0].copy()
        loss, ir = 0.0, 0.0
    info.update(init_params=init_params, params=params, estimation_loss=loss)
    if save_results_bool:
        results = predict(model, data[:, :in_sample_end])  # the model's current parameters (:308)
        set_params_(model, params)
        _io.save_results(model, results, loss, thread_id, "insample")
        loss = get_loss(model, data[:, :in_sample_end])
        print(f"In-sample loss: {loss}")
        info["insample_loglik"] = loss
        results = predict(model, data)
        _io.save_results(model, results, loss, thread_id, "outofsample")
        loss_array = get_loss_array(model, data, K=1)
        oos = np.atleast_1d(loss_array)[in_sample_end:]  # loss_array[in_sample_end+1:end]
        means = {}
        for lab, frac in (("first 10%", 0.1), ("first 25%", 0.25), ("first 50%", 0.5), ("first 75%", 0.75),
                          ("full", None)):
            part = oos if frac is None else oos[:int(np.floor(frac * len(oos)))]
            means[lab] = float(np.mean(part)) if part.size else float("nan")
            print(f"Out-of-sample loss array ({lab}): {means[lab]}")
        info.update(loss_array=loss_array, oos_loss_means=means)
        for dt in ("insample", "outofsample"):
            for what in ("factors_filtered", "fit_filtered", "factor_loadings_1_filtered", "factor_loadings_2_filtered"):
                info["files"].append(_io.result_path(model, thread_id, f"{what}_{dt}.csv"))
    if run_rolling:
        print("Forecasting...")
        info["rolling"] = run_rolling_forecasts(model, data, thread_id, in_sample_end, in_sample_start,
                                                forecast_horizon, all_params, window_type=window_type,
                                                max_group_iters=max_group_iters, group_tol=group_tol,
                                                reestimate=reestimate, iterations=iterations, group=group)
    model.last_run = info
    return model
