"""Host-side mirror of the reference's Kalman model API (the drop-in surface).

Reference interface mirrored (paths relative to the reference root):

=======================================  =================================================
reference                                 here
=======================================  =================================================
``create_model`` model_dictionary.jl:7-16  :func:`create_model` (codes "1C"/"0", "TVλ"/"1";
                                            "GNS5" is this build's extension)
``DNSModel`` dns.jl:3-37                    :class:`DNSModel`
``TVλDNSModel`` tvλdns.jl:3-35              :class:`TVLambdaDNSModel`
``get_params`` paramoperations.jl:1-4       :func:`get_params`
``set_params!`` paramoperations.jl:45-68    :func:`set_params_` (Julia ``!`` → trailing ``_``)
``transform_params`` parameteroperations.jl:22-32    :func:`transform_params`
``untransform_params`` parameteroperations.jl:34-60  :func:`untransform_params`
``get_loss`` kalman/filter.jl:182-209       :func:`get_loss`
``compute_loss`` optimization.jl:10-23      :func:`compute_loss`
``predict`` kalman/filter.jl:250-282        :func:`predict` (``horizon`` = NaN padding of
                                            forecasting.jl:141)
``get_loss_array`` kalman/filter.jl:211-247 :func:`get_loss_array`
forecast blocks forecasting.jl:236-250      :func:`forecast_batch`
``estimate_steps!`` optimization.jl:137-312 :func:`estimate_steps_` (+ batched
                                            :func:`estimate_batch`)
=======================================  =================================================

plus the batched forms the device boundary exists for: :func:`get_loss_batch` and
:func:`compute_loss_batch` (one call evaluates B parameter vectors).

All numerics run in libyfm_hip.so on the GPU; this module only holds parameters,
validates shapes and forwards pointers.  Errors mirror the reference: a batch
entry is ``-inf`` where ``get_loss`` returns ``-Inf`` and ``nan`` where the
reference would throw (singular ``I-Φ`` / ``I-Φ⊗Φ``); :func:`get_loss` raises
:class:`SingularException` in that case, as Julia does.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import params as _p
from .engine import get_engine


class SingularException(ArithmeticError):
    """Raised where the reference's initialize_filter throws (filter.jl:4, :7)."""


@dataclass
class KalmanBaseModel:
    """kalmanbasemodel.jl:6-41 — the fields the hot path reads."""
    maturities: np.ndarray
    N: int
    M: int
    L: int
    kind: int
    model_string: str
    results_folder: str = "results/"
    flat_params: np.ndarray = field(default=None)

    def __post_init__(self):
        if self.flat_params is None:
            self.flat_params = np.zeros(_p.n_params(self.kind))

    @property
    def transformations(self):
        return _p.transform_codes(self.kind)


class AbstractKalmanModel:
    base: KalmanBaseModel
    device: int = 0

    @property
    def kind(self) -> int:
        return self.base.kind


class DNSModel(AbstractKalmanModel):
    """dns.jl:3-37: fixed-λ dynamic Nelson–Siegel, M = 3, P = 20."""

    def __init__(self, maturities, N: int, M: int = 3, model_string: str = "1C", results_location: str = "results/",
                 device: int = 0):
        if M != 3:
            raise ValueError("DNSModel is a 3-factor model (M = 3)")
        self.base = KalmanBaseModel(np.asarray(maturities, dtype=np.float64), N, 3, 1, _p.KIND_DNS, model_string,
                                    results_location)
        self.device = device


class TVLambdaDNSModel(AbstractKalmanModel):
    """tvλdns.jl:3-35: time-varying λ (EKF), state dimension M + 1 = 4, P = 31."""

    def __init__(self, maturities, N: int, M: int = 3, model_string: str = "TVλ", results_location: str = "results/",
                 device: int = 0):
        self.base = KalmanBaseModel(np.asarray(maturities, dtype=np.float64), N, M + 1, 1, _p.KIND_TVL, model_string,
                                    results_location)
        self.device = device


class GNS5Model(AbstractKalmanModel):
    """Extension (not in the reference): 5-factor generalised NS, loadings
    [1, S(λ₁), C(λ₁), S(λ₂), C(λ₂)], P = 48 ([γ₁, γ₂, base block])."""

    def __init__(self, maturities, N: int, M: int = 5, model_string: str = "GNS5", results_location: str = "results/",
                 device: int = 0):
        self.base = KalmanBaseModel(np.asarray(maturities, dtype=np.float64), N, 5, 2, _p.KIND_GNS, model_string,
                                    results_location)
        self.device = device


_CODES = {
    "1C": ("1C", DNSModel), "0": ("1C", DNSModel),
    "TVλ": ("TVλ", TVLambdaDNSModel), "1": ("TVλ", TVLambdaDNSModel),
    "GNS5": ("GNS5", GNS5Model),
}


def create_model(model_type: str, maturities, N: int, M: int = 3, float_type=np.float64,
                 results_location: str = "results/", device: int = 0):
    """model_dictionary.jl:7-16 for the Kalman codes; returns (model, standardized model_type)."""
    if np.dtype(float_type) != np.float64:
        raise ValueError("the MI355X path computes in Float64 only (the reference's Float64 path, test.jl:25)")
    if model_type not in _CODES:
        raise ValueError(f"Invalid model type: {model_type} (Kalman codes: {sorted(_CODES)})")
    std, cls = _CODES[model_type]
    mats = np.asarray(maturities, dtype=np.float64)
    if len(mats) != N:
        raise ValueError("len(maturities) != N")
    return cls(mats, N, M, model_string=model_type, results_location=results_location, device=device), std


def get_params(model: AbstractKalmanModel) -> np.ndarray:
    return model.base.flat_params


def set_params_(model: AbstractKalmanModel, params) -> None:
    """set_params! — stores the constrained parameter vector the filter will use."""
    params = np.asarray(params, dtype=np.float64).reshape(-1)
    if params.shape[0] != _p.n_params(model.kind):
        raise ValueError(f"expected {_p.n_params(model.kind)} parameters, got {params.shape[0]}")
    model.base.flat_params = params.copy()


def transform_params(model: AbstractKalmanModel, params) -> np.ndarray:
    return _p.transform_params(model.kind, params)


def untransform_params(model: AbstractKalmanModel, params) -> np.ndarray:
    return _p.untransform_params(model.kind, params)


def _engine(model, data):
    eng = get_engine(model.device)
    eng.set_panel(data, model.base.maturities)
    return eng


def get_loss(model: AbstractKalmanModel, data) -> float:
    """filter.jl:182-209 for the model's current (constrained) parameters."""
    eng = _engine(model, data)
    ll = float(eng.loglik(model.kind, model.base.flat_params, space=_p.SPACE_CONSTRAINED)[0])
    if np.isnan(ll):
        raise SingularException("initialize_filter: singular I - Φ or I - Φ⊗Φ")
    return ll


def compute_loss(model: AbstractKalmanModel, data, params) -> float:
    """optimization.jl:10-23: transform, set_params!, return -get_loss."""
    set_params_(model, transform_params(model, params))
    return -get_loss(model, data)


def get_loss_batch(model: AbstractKalmanModel, data, Theta, space: int = 1, T_use=None) -> np.ndarray:
    """Batched get_loss over the columns of Θ (P×B).  ``space`` 1 = constrained θ_c
    (set_params! input), 0 = unconstrained θ (compute_loss input).  ``T_use[b]``
    evaluates ``get_loss(model, data[:, :T_use[b]])``."""
    eng = _engine(model, data)
    return eng.loglik(model.kind, Theta, space=space, T_use=T_use)


def compute_loss_batch(model: AbstractKalmanModel, data, Theta, T_use=None) -> np.ndarray:
    """Batched compute_loss: −loglik for every unconstrained θ_b (column of Θ)."""
    return -get_loss_batch(model, data, Theta, space=_p.SPACE_UNCONSTRAINED, T_use=T_use)


def filter_states(model: AbstractKalmanModel, data, Theta=None, space: int = 1, T_use=None):
    """(loglik[B], beta[M,T-1,B], P[M,M,T-1,B]): the predicted state after every filter! call."""
    eng = _engine(model, data)
    if Theta is None:
        Theta = model.base.flat_params
    return eng.filter_states(model.kind, Theta, space=space, T_use=T_use)


def predict(model: AbstractKalmanModel, data, horizon: int = 1, Theta=None, space: int = 1, T_use=None):
    """filter.jl:250-282 — ``predict(model, data)`` for the model's parameters (horizon = 1), or
    ``predict(model, hcat(data[:, 1:T_b], NaN × (horizon − 1)))`` as the forecasting driver calls it
    (forecasting.jl:141, :181-183).  With ``Theta`` (P×B) the call is batched and every array gets a
    trailing batch axis; otherwise returns the reference's named tuple of N×n / M×n / L×n arrays,
    n = T + horizon − 1."""
    eng = _engine(model, data)
    single = Theta is None
    if single:
        Theta = model.base.flat_params
    out = eng.predict(model.kind, Theta, space=space, T_use=T_use, horizon=horizon)
    if single:
        out = {k: v[:, :, 0] for k, v in out.items()}
        if np.isnan(out["factors"]).all():
            raise SingularException("initialize_filter: singular I - Φ or I - Φ⊗Φ")
    return out


def get_loss_array(model: AbstractKalmanModel, data, K: int = 1, Theta=None, space: int = 1, T_use=None):
    """filter.jl:211-247: the per-step −‖y_t − ŷ_t‖²/N/K (length T−1), or the scalar −Inf where the
    reference returns it.  With ``Theta`` (P×B): a (T−1)×B array, −Inf rows for −Inf candidates."""
    eng = _engine(model, data)
    single = Theta is None
    out = eng.loss_array(model.kind, model.base.flat_params if single else Theta, space=space, T_use=T_use, K=K)
    if single:
        row = out[:, 0]
        if np.isnan(row).all() and row.size:
            raise SingularException("initialize_filter: singular I - Φ or I - Φ⊗Φ")
        if row.size and np.isneginf(row).all():
            return -np.inf
        return row
    return out


def forecast_batch(model: AbstractKalmanModel, data, Theta, T_use, horizon: int, space: int = 1) -> np.ndarray:
    """The rolling-window driver's per-task record (forecasting.jl:236-250): for window b,
    ``vcat(factors, states, preds)[:, end-h+1:end]`` of predict on hcat(data[:, 1:T_use[b]], NaN × (h−1)).
    Returns (M + L + N, h, B)."""
    eng = _engine(model, data)
    return eng.forecast(model.kind, Theta, space=space, T_use=T_use, horizon=horizon)


class EstimationError(RuntimeError):
    """estimate_steps! rethrows from the first group iteration (optimization.jl:249-253)."""


def estimate_steps_(model: AbstractKalmanModel, data, all_params, param_groups=None, max_group_iters: int = 10,
                    tol: float = 1e-8, printing: bool = False, iterations: int = 500):
    """estimate_steps! (optimization.jl:137-312) for a Kalman model: all_params (P×n, constrained; Kalman
    models use column 1 only, :153) → (init_p, ll, best_p, ir), init_p and best_p constrained like the
    reference: init_p = transform_params of the untransformed, sanitised and ×0.95-rescaled start
    (:157-184, :298-302).
    Parameter groups other than all-"1" are not supported (the Kalman default, kalmanbasemodel.jl:150-159).
    `iterations`: the NelderMead budget per group (opt1, optimization.jl:442-451: 500)."""
    A = np.asarray(all_params, dtype=np.float64)
    start = A[:, 0] if A.ndim == 2 else A
    if param_groups is not None and any(g != "1" for g in param_groups):
        raise NotImplementedError("Kalman models estimate every parameter in group \"1\"")
    r = estimate_batch(model, data, start[:, None], max_group_iters=max_group_iters, tol=tol, iterations=iterations)
    if r["status"][0] == 1:
        raise EstimationError("compute_loss threw on the first group iteration (singular initialize_filter)")
    if printing:
        print(f"✓ Best overall LL = {r['ll'][0]} from start 1")
    return r["init_c"][:, 0].copy(), float(r["ll"][0]), r["theta_c"][:, 0].copy(), 0


def estimate_batch(model: AbstractKalmanModel, data, Theta0, T_use=None, space: int = 1, iterations: int = 500,
                   g_tol: float = 1e-6, max_group_iters: int = 10, tol: float = 1e-8) -> dict:
    """R independent estimate_steps! chains (windows × starts) whose objective evaluations share one device
    launch per round (libyfm_hip.so: yfm_estimate).  Θ₀: P×R starts (constrained by default, as all_params)."""
    eng = _engine(model, data)
    return eng.estimate(model.kind, Theta0, space=space, T_use=T_use, iterations=iterations, g_tol=g_tol,
                        max_group_iters=max_group_iters, tol=tol)
