"""yfm_amd — MI355X-native batched Kalman log-likelihood for YieldFactorModels.jl.

The numerics live in ``libyfm_hip.so`` (HIP, gfx950) behind the C ABI of
``include/yfm.h``; this package is the host-side mirror of the reference's
model / objective API (see :mod:`yfm_amd.models`).
"""
from .params import (KIND_DNS, KIND_GNS, KIND_TVL, SPACE_CONSTRAINED, SPACE_UNCONSTRAINED, gamma_dim, n_params,
                     param_layout, state_dim)
from .models import (DNSModel, GNS5Model, SingularException, TVLambdaDNSModel, compute_loss, compute_loss_batch,
                     create_model, estimate_batch, estimate_steps_, filter_states, forecast_batch, get_loss, get_loss_array, get_loss_batch,
                     get_params, predict, set_params_, transform_params, untransform_params)
from .engine import Engine, get_engine
from .driver import load_initial_parameters_, run

__all__ = [
    "KIND_DNS", "KIND_TVL", "KIND_GNS", "SPACE_CONSTRAINED", "SPACE_UNCONSTRAINED", "n_params", "param_layout",
    "state_dim", "DNSModel", "TVLambdaDNSModel", "GNS5Model", "SingularException", "create_model", "get_params",
    "set_params_", "transform_params", "untransform_params", "get_loss", "compute_loss", "get_loss_batch",
    "compute_loss_batch", "filter_states", "estimate_steps_", "estimate_batch", "predict", "get_loss_array", "forecast_batch", "gamma_dim", "Engine",
    "get_engine", "run", "load_initial_parameters_",
]
