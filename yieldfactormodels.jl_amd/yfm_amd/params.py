"""Parameter layout and the unconstrained<->constrained maps (host side).

Mirrors the reference's per-parameter transform vectors:

* ``src/models/kalman/kalmanbasemodel.jl:74-120`` — base block
  ``[σ² (exp), U upper-triangular by column (exp on the diagonal), δ (id),
  Φ row-major (2eˣ/(1+eˣ)−1 on the diagonal)]``;
* ``src/models/kalman/dns.jl:15-22`` — DNS prepends one identity (γ);
* ``src/models/kalman/tvλdns.jl:12-35`` — TVλ prepends nothing and uses a
  4-dimensional state;
* ``src/utils/transformations.jl:2-26`` and
  ``src/models/parameteroperations.jl:22-60`` — the elementwise maps.

The device kernels decode θ themselves (``csrc/yfm_device.hpp``); this module
is the host API surface (``transform_params`` / ``untransform_params``) and
the single source of the layout offsets the host code uses.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

KIND_DNS, KIND_TVL, KIND_GNS = 0, 1, 2
KIND_NAMES = {KIND_DNS: "1C", KIND_TVL: "TVλ", KIND_GNS: "GNS5"}

ID, POS, R11 = 0, 1, 2


@dataclass(frozen=True)
class ParamLayout:
    kind: int
    M: int  # state dimension
    n_lead: int  # γ entries before the base block
    P: int

    @property
    def base_offset(self):  # index of σ²
        return self.n_lead

    @property
    def u_offset(self):
        return self.n_lead + 1

    @property
    def delta_offset(self):
        return self.u_offset + self.M * (self.M + 1) // 2

    @property
    def phi_offset(self):
        return self.delta_offset + self.M


def state_dim(kind: int) -> int:
    return {KIND_DNS: 3, KIND_TVL: 4, KIND_GNS: 5}[kind]


def gamma_dim(kind: int) -> int:
    """L = length of base.gamma (kalmanbasemodel.jl:58), reported by predict as `states`."""
    return {KIND_DNS: 1, KIND_TVL: 1, KIND_GNS: 2}[kind]


def param_layout(kind: int) -> ParamLayout:
    M = state_dim(kind)
    n_lead = {KIND_DNS: 1, KIND_TVL: 0, KIND_GNS: 2}[kind]
    P = n_lead + 1 + M * (M + 1) // 2 + M + M * M
    return ParamLayout(kind, M, n_lead, P)


def n_params(kind: int) -> int:
    return param_layout(kind).P


def transform_codes(kind: int) -> np.ndarray:
    lay = param_layout(kind)
    M = lay.M
    cov = []
    for i in range(M):  # kalmanbasemodel.jl:76-89
        for j in range(i + 1):
            cov.append(POS if i == j else ID)
    phi = [R11 if i == j else ID for i in range(M) for j in range(M)]
    return np.asarray([ID] * lay.n_lead + [POS] + cov + [ID] * M + phi, dtype=np.int8)


def transform_params(kind: int, theta) -> np.ndarray:
    """parameteroperations.jl:22-32 (works on a vector or a P×B matrix)."""
    theta = np.asarray(theta, dtype=np.float64)
    codes = transform_codes(kind)
    out = theta.copy()
    with np.errstate(over="ignore", invalid="ignore"):
        pos = codes == POS
        out[pos] = np.exp(theta[pos])
        r = codes == R11
        y = np.exp(theta[r])
        out[r] = 2.0 * y / (1.0 + y) - 1.0  # transformations.jl:21-26, evaluated as written
    return out


def untransform_params(kind: int, theta_c) -> np.ndarray:
    """parameteroperations.jl:34-60."""
    theta_c = np.asarray(theta_c, dtype=np.float64)
    codes = transform_codes(kind)
    out = theta_c.copy()
    with np.errstate(divide="ignore", invalid="ignore"):
        pos = codes == POS
        out[pos] = np.log(theta_c[pos])
        r = codes == R11
        out[r] = np.log1p(theta_c[r]) - np.log1p(-theta_c[r])
    return out

SPACE_UNCONSTRAINED, SPACE_CONSTRAINED = 0, 1
