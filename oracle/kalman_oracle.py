"""CPU oracle: a line-by-line NumPy/LAPACK restatement of the reference Kalman path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker.  The product path (``yieldfactormodels.jl_amd``) never imports it.

Parity status: **parity unpinned** against the reference itself.  The reference
is Julia 1.11 (``/root/reference``); no ``julia`` binary exists in this image or
on the GPU box, and the reference ships no tests, fixtures or golden vectors
(SURVEY.md §4, §8c).  This oracle is instead pinned by

  * known-answer tests that use no filter code at all (Φ = 0 makes the
    innovations iid N(0, ZQZ' + σ²I); the loglik is then a sum of
    ``scipy.stats.multivariate_normal.logpdf`` values), and
  * an independent C restatement (``oracle/yfm_oracle.c``) with its own
    getrf/getri, which must agree to 1e-11 relative.

Every function cites the reference file:line it restates (paths relative to
the reference root).  LAPACK is reached through ``scipy.linalg.lapack`` —
``dgetrf``/``dgetri``/``dgetrs``/``dtrtrs``/``dtrtri`` — the routines Julia's
LinearAlgebra calls for ``lu``, ``inv``, ``\\`` and ``logdet``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
from scipy.linalg import lapack

LOG2PI = math.log(2.0 * math.pi)

# transform codes: 0 identity, 1 from_R_to_pos, 2 from_R_to_11
ID, POS, R11 = 0, 1, 2

KIND_DNS, KIND_TVL, KIND_GNS = 0, 1, 2


def exp_ieee(x):
    """math.exp with Julia's IEEE overflow (Inf) instead of Python's OverflowError."""
    x = float(x)
    try:
        return math.exp(x)
    except OverflowError:
        return math.inf


class SingularException(Exception):
    """Julia's LinearAlgebra.SingularException (thrown by `\\` / `inv`)."""


# --------------------------------------------------------------------------
# transformations  (src/utils/transformations.jl:2-26)
# --------------------------------------------------------------------------
def from_R_to_pos(x):  # transformations.jl:2-4
    return np.exp(x)


def from_pos_to_R(x):  # transformations.jl:6-8
    return np.log(x)


def from_R_to_11(x):  # transformations.jl:21-26  (evaluated exactly as 2y/(1+y)-1)
    with np.errstate(over="ignore", invalid="ignore"):
        y = np.exp(x)
        return 2.0 * y / (1.0 + y) - 1.0


def from_11_to_R(x):  # transformations.jl:10-12
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.log1p(x) - np.log1p(-x)


def base_transform_codes(M: int) -> list[int]:
    """kalmanbasemodel.jl:74-120: [σ² pos, U (col-major upper, diag pos), δ id, Φ row-major (diag 11)]."""
    cov = []
    for i in range(M):  # kalmanbasemodel.jl:76-89 (i outer, j inner, keep j <= i)
        for j in range(M):
            if i == j:
                cov.append(POS)
            elif j < i:
                cov.append(ID)
    phi = [R11 if i == j else ID for i in range(M) for j in range(M)]  # :92-104
    return [POS] + cov + [ID] * M + phi


def transform_codes(kind: int, M: int) -> list[int]:
    """dns.jl:15-22 prepends one identity (γ); TVλ (tvλdns.jl:12-35) prepends nothing, base M+1."""
    if kind == KIND_DNS:
        return [ID] + base_transform_codes(M)
    if kind == KIND_GNS:
        return [ID, ID] + base_transform_codes(M)
    if kind == KIND_TVL:
        return base_transform_codes(M)  # M here is the state dim (= 4)
    raise ValueError(kind)


def transform_params(codes, theta):
    """parameteroperations.jl:22-32: θ_c[i] = f_i(θ[i])."""
    theta = np.asarray(theta, dtype=np.float64)
    out = np.empty_like(theta)
    for i, c in enumerate(codes):
        if c == ID:
            out[i] = theta[i]
        elif c == POS:
            with np.errstate(over="ignore"):
                out[i] = from_R_to_pos(theta[i])
        else:
            out[i] = from_R_to_11(theta[i])
    return out


def untransform_params(codes, theta_c):
    """parameteroperations.jl:34-60."""
    theta_c = np.asarray(theta_c, dtype=np.float64)
    out = np.empty_like(theta_c)
    for i, c in enumerate(codes):
        if c == ID:
            out[i] = theta_c[i]
        elif c == POS:
            with np.errstate(divide="ignore", invalid="ignore"):
                out[i] = from_pos_to_R(theta_c[i])
        else:
            out[i] = from_11_to_R(theta_c[i])
    return out


# --------------------------------------------------------------------------
# Julia LinearAlgebra dispatch for `\`, `inv`, `logdet` on dense matrices
# --------------------------------------------------------------------------
def _istriu(A):
    return bool(np.all(np.tril(A, -1) == 0.0))


def _istril(A):
    return bool(np.all(np.triu(A, 1) == 0.0))


def jl_ldiv(A, b):
    """Julia `A \\ b` for square A: Diagonal / triangular / LU dispatch (LinearAlgebra generic.jl)."""
    A = np.array(A, dtype=np.float64, order="F")
    b = np.array(b, dtype=np.float64)
    if _istril(A):
        if _istriu(A):
            d = np.diag(A)
            if np.any(d == 0.0):
                raise SingularException()
            return b / d
        x, info = lapack.dtrtrs(A, b, lower=1)
        if info > 0:
            raise SingularException()
        return x
    if _istriu(A):
        x, info = lapack.dtrtrs(A, b, lower=0)
        if info > 0:
            raise SingularException()
        return x
    lu, piv, info = lapack.dgetrf(A)
    if info > 0:
        raise SingularException()
    x, info = lapack.dgetrs(lu, piv, b)
    return x


def jl_inv(A):
    """Julia `inv(A::StridedMatrix)`: triangular inverse if triangular, else getrf+getri."""
    A = np.array(A, dtype=np.float64, order="F")
    if _istriu(A):
        Ai, info = lapack.dtrtri(A, lower=0)
        if info > 0:
            raise SingularException()
        return np.triu(Ai)
    if _istril(A):
        Ai, info = lapack.dtrtri(A, lower=1)
        if info > 0:
            raise SingularException()
        return np.tril(Ai)
    lu, piv, info = lapack.dgetrf(A)
    if info > 0:
        raise SingularException()
    Ai, info = lapack.dgetri(lu, piv)
    return Ai


class DomainError(Exception):
    pass


def jl_logdet(A):
    """Julia `logdet(A)` = logabsdet(lu(A, check=false)) then d + log(s); log(-1) throws DomainError."""
    A = np.array(A, dtype=np.float64, order="F")
    lu, piv, info = lapack.dgetrf(A)
    if info > 0:  # issuccess false: (log(0), log(1)) -> -Inf + log(0.0)... = -Inf
        return -math.inf
    d = np.diag(lu)
    s = 1.0
    acc = 0.0
    for i in range(len(d)):
        s *= math.copysign(1.0, d[i]) if d[i] == d[i] else math.nan
        if piv[i] != i:
            s = -s
        acc += math.log(abs(d[i])) if d[i] == d[i] else math.nan
    if s < 0:
        raise DomainError()
    return acc + (math.log(s) if s == s else math.nan)


# --------------------------------------------------------------------------
# model state (kalmanbasemodel.jl:6-41) and parameter decoding
# --------------------------------------------------------------------------
@dataclass
class KalmanState:
    kind: int
    maturities: np.ndarray
    N: int
    M: int  # state dimension (3 DNS, 4 TVλ, 5 GNS)
    Z: np.ndarray = None
    beta: np.ndarray = None
    Phi: np.ndarray = None
    delta: np.ndarray = None
    gamma: np.ndarray = None
    Omega_state: np.ndarray = None
    Omega_obs: np.ndarray = None
    P: np.ndarray = None
    y_pred: np.ndarray = None
    v: np.ndarray = None
    F: np.ndarray = None
    F_inv: np.ndarray = None
    lam: float = 0.0  # TVλ model.lambda
    z_i: np.ndarray = None
    extra: dict = field(default_factory=dict)

    @classmethod
    def fresh(cls, kind, maturities, M):
        mats = np.asarray(maturities, dtype=np.float64)
        N = len(mats)
        s = cls(kind=kind, maturities=mats, N=N, M=M)
        s.Z = np.ones((N, M))  # kalmanbasemodel.jl:53
        s.beta = np.zeros(M)
        s.Phi = np.zeros((M, M))
        s.delta = np.zeros(M)
        s.gamma = np.zeros(1)
        s.Omega_state = np.eye(M)
        s.Omega_obs = np.eye(N)
        s.P = np.eye(M)
        s.y_pred = np.zeros(N)
        s.v = np.zeros(N)
        s.F = np.zeros((N, N))  # :66  (fresh model: zero F, F_inv, v)
        s.F_inv = np.zeros((N, N))
        s.z_i = np.zeros(N)
        return s


def set_params_base(s: KalmanState, params):
    """paramoperations.jl:6-41."""
    M = s.M
    k = 0
    s.Omega_obs = np.eye(s.N) * params[k]
    k += 1
    U = np.zeros((M, M))
    for j in range(M):  # column j, then row i <= j
        for i in range(M):
            if i <= j:
                U[i, j] = params[k]
                k += 1
    s.Omega_state = U.T @ U  # :35
    s.delta = np.array(params[k:k + M], dtype=np.float64)
    k += M
    s.Phi = np.array(params[k:k + M * M], dtype=np.float64).reshape(M, M)  # reshape(.,M,M)' == row-major
    k += M * M


def dns_loadings(gamma, maturities, Z):
    """dns.jl:51-65: λ = 0.01 + e^γ; z = e^{-λτ}; Z = [1, (1-z)/(λτ), (1-z)/(λτ) - z]."""
    lam = 1e-2 + exp_ieee(gamma)
    with np.errstate(all="ignore"):
        tau = lam * maturities
        z = np.exp(-tau)
    Z[:, 0] = 1.0
    Z[:, 1] = (1.0 - z) / tau
    Z[:, 2] = Z[:, 1] - z


def gns_loadings(gammas, maturities, Z):
    """5-factor generalised NS extension (not in the reference): [1, S(λ1), C(λ1), S(λ2), C(λ2)]."""
    Z[:, 0] = 1.0
    for b, g in enumerate(gammas):
        lam = 1e-2 + exp_ieee(g)
        with np.errstate(all="ignore"):
            tau = lam * maturities
            z = np.exp(-tau)
        Z[:, 1 + 2 * b] = (1.0 - z) / tau
        Z[:, 2 + 2 * b] = Z[:, 1 + 2 * b] - z


def tvl_loadings(s: KalmanState, beta4):
    """tvλdns.jl:53-64 (columns 2 and 3 only; column 1 stays ones)."""
    s.lam = 1e-2 + exp_ieee(beta4)
    with np.errstate(all="ignore"):
        tau = s.lam * s.maturities
        s.z_i = np.exp(-tau)
    s.extra["tau"] = tau
    s.Z[:, 1] = (1.0 - s.z_i) / tau
    s.Z[:, 2] = s.Z[:, 1] - s.z_i


def set_params(s: KalmanState, params):
    """paramoperations.jl:45-59 (DNS), :61-68 (TVλ); GNS extension takes two γ."""
    params = np.asarray(params, dtype=np.float64)
    if s.kind == KIND_DNS:
        s.gamma = np.array([params[0]])
        set_params_base(s, params[1:])
        dns_loadings(params[0], s.maturities, s.Z)
    elif s.kind == KIND_GNS:
        s.gamma = np.array(params[0:2])  # L = 2 (both γ) for the extension
        set_params_base(s, params[2:])
        gns_loadings(params[0:2], s.maturities, s.Z)
    elif s.kind == KIND_TVL:
        set_params_base(s, params)
    else:
        raise ValueError(s.kind)


def n_params(kind, M):
    base = 1 + M * (M + 1) // 2 + M + M * M
    return base + (1 if kind == KIND_DNS else 2 if kind == KIND_GNS else 0)


# --------------------------------------------------------------------------
# filter  (src/models/kalman/filter.jl)
# --------------------------------------------------------------------------
def initialize_filter(s: KalmanState):
    """filter.jl:1-10 — both solves throw on singularity (outside get_loss's try)."""
    M = s.M
    s.beta = jl_ldiv(np.eye(M) - s.Phi, s.delta)
    A = np.eye(M * M) - np.kron(s.Phi, s.Phi)
    vecP = jl_inv(A) @ s.Omega_state.reshape(-1, order="F")
    s.P = vecP.reshape((M, M), order="F")


def filter_step_generic(s: KalmanState, y):
    """filter.jl:125-179 (DNS / fixed-Z Kalman step). Returns False iff inv(F) threw."""
    if np.any(np.isnan(y)):  # :126-140
        s.y_pred = s.Z @ s.beta
        s.beta = s.delta + s.Phi @ s.beta
        s.P = (s.Phi @ s.P) @ s.Phi.T + s.Omega_state
        return True
    s.y_pred = s.Z @ s.beta  # :143
    s.v = y - s.y_pred  # :144
    s.F = (s.Z @ s.P) @ s.Z.T + s.Omega_obs  # :147
    try:
        s.F_inv = jl_inv(s.F)  # :150
    except SingularException:
        s.F_inv = np.full_like(s.F, np.inf)  # :153
        return False
    K = (s.Z @ s.P.T).T @ s.F_inv  # :158  (M×N)
    s.beta = s.beta + K @ s.v  # :162
    s.beta = s.delta + s.Phi @ s.beta  # :163-165
    KZ = K @ s.Z  # :169
    IKZ = np.eye(s.M) - KZ  # :171
    tmp = IKZ @ s.P  # :173
    KZ = s.Phi @ tmp  # :174
    s.P = KZ @ s.Phi.T + s.Omega_state  # :175-176
    return True


def filter_step_tvl(s: KalmanState, y):
    """filter.jl:12-80 — EKF for TVλ with the reference's dZ1 formula reproduced as written (:43)."""
    if np.any(np.isnan(y)):  # :13-29
        tvl_loadings(s, s.beta[3])
        s.y_pred = s.Z[:, :3] @ s.beta[:3]
        s.beta = s.delta + s.Phi @ s.beta
        s.P = (s.Phi @ s.P) @ s.Phi.T + s.Omega_state
        return True
    tvl_loadings(s, s.beta[3])  # :32
    s.y_pred = s.Z[:, :3] @ s.beta[:3]  # :33
    s.v = y - s.y_pred  # :34
    dlam = s.lam - 1e-2  # :38
    m = s.maturities
    dZ1 = s.z_i / s.lam - s.z_i / ((s.lam * s.lam) * m)  # :43 (quirk kept; λ^2 = λ*λ, Inf on overflow)
    dZ2 = m * s.z_i  # :44
    s.Z[:, 3] = ((s.beta[1] + s.beta[2]) * dZ1 + s.beta[2] * dZ2) * dlam  # :46
    s.F = (s.Z @ s.P) @ s.Z.T + s.Omega_obs  # :49
    try:
        s.F_inv = jl_inv(s.F)  # :52
    except SingularException:
        return False  # :53-55 (F_inv left stale, no update)
    K = (s.Z @ s.P.T).T @ s.F_inv  # :59
    s.beta = s.beta + K @ s.v  # :63
    s.beta = s.delta + s.Phi @ s.beta  # :64-66
    KZ = K @ s.Z
    IKZ = np.eye(s.M) - KZ
    tmp = IKZ @ s.P
    KZ = s.Phi @ tmp
    s.P = KZ @ s.Phi.T + s.Omega_state  # :69-77
    return True


def filter_step(s, y):
    if s.kind == KIND_TVL:
        return filter_step_tvl(s, y)
    return filter_step_generic(s, y)


class InitThrow(Exception):
    """initialize_filter threw (singular I-Φ or I-Φ⊗Φ); the batched API maps this to NaN."""


def get_loss(s: KalmanState, data, record=None):
    """filter.jl:182-209.  `record` (list) receives (beta, P) after every filter! call."""
    data = np.asarray(data, dtype=np.float64)
    nobs = data.shape[1]
    try:
        initialize_filter(s)
    except SingularException as e:
        raise InitThrow() from e
    loglik = 0.0
    logdet_2pi = s.N * LOG2PI  # :188
    with np.errstate(all="ignore"):
        for t in range(1, nobs):  # Julia t = 1 .. nobs-1
            filter_step(s, data[:, t - 1].copy())
            if record is not None:
                record.append((s.beta.copy(), s.P.copy()))
            try:
                if t > 1:
                    ld = jl_logdet(s.F)
                    quad = float((s.v @ s.F_inv) @ s.v)
                    loglik -= 0.5 * (ld + quad + logdet_2pi)
            except DomainError:
                return -math.inf
            if math.isinf(loglik) or math.isnan(loglik):
                return -math.inf
    return loglik


def compute_loss(kind, maturities, M, data, theta):
    """optimization.jl:10-23: -get_loss(set_params!(transform_params(θ)))."""
    s = KalmanState.fresh(kind, maturities, M)
    tc = transform_params(transform_codes(kind, M if kind != KIND_TVL else M), theta)
    set_params(s, tc)
    return -get_loss(s, data)


def loglik(kind, maturities, M, data, theta, space=0, record=None):
    """Convenience for tests: +loglik of one candidate; NaN where the reference would throw."""
    s = KalmanState.fresh(kind, maturities, M)
    codes = transform_codes(kind, M)
    tc = transform_params(codes, theta) if space == 0 else np.asarray(theta, dtype=np.float64)
    set_params(s, tc)
    try:
        return get_loss(s, data, record=record)
    except InitThrow:
        return math.nan


def get_loss_array(s: KalmanState, data, K: int = 1):
    """filter.jl:211-247.  The K passes continue the filter state (initialize_filter runs once,
    :214); the set_params!(catched_params) of passes k > 1 (:223-225) re-sets the same flat
    parameters of a Kalman model (get_params returns flat_params, paramoperations.jl:1-4), so it
    changes nothing and is omitted.  Returns the scalar -Inf where the reference does (:234-236)."""
    data = np.asarray(data, dtype=np.float64)
    nobs = data.shape[1]
    initialize_filter(s)
    mse = np.zeros(nobs - 1)
    with np.errstate(all="ignore"):
        for _k in range(K):
            for t in range(1, nobs):
                filter_step(s, data[:, t - 1].copy())
                s.v = data[:, t - 1] - s.y_pred
                if t > 1:
                    mse[t - 1] -= float(s.v @ s.v)
                if not np.isfinite(mse[t - 1]):
                    return -math.inf
    return mse / s.N / K


def predict(s: KalmanState, data):
    """filter.jl:250-282: outputs are stored at column t-1 for t > 1, plus one NaN-step forecast."""
    data = np.asarray(data, dtype=np.float64)
    N, nobs = data.shape
    initialize_filter(s)
    preds = np.empty((N, nobs))
    factors = np.empty((s.M, nobs))
    states = np.empty((len(s.gamma), nobs))
    fl1 = np.empty((N, nobs))
    fl2 = np.empty((N, nobs))
    with np.errstate(all="ignore"):
        for t in range(1, nobs + 1):
            filter_step(s, data[:, t - 1].copy())
            if t > 1:
                preds[:, t - 2] = s.y_pred
                factors[:, t - 2] = s.beta
                states[:, t - 2] = s.gamma
                fl1[:, t - 2] = s.Z[:, 1]
                fl2[:, t - 2] = s.Z[:, 2]
        filter_step(s, np.full(N, np.nan))
    preds[:, -1] = s.y_pred
    factors[:, -1] = s.beta
    states[:, -1] = s.gamma
    fl1[:, -1] = s.Z[:, 1]
    fl2[:, -1] = s.Z[:, 2]
    return dict(preds=preds, factors=factors, states=states,
                factor_loadings_1=fl1, factor_loadings_2=fl2)


def pad_nan(data, horizon: int):
    """hcat(data, fill(NaN, N, horizon-1)) — the forecast padding of forecasting.jl:141, :161, :242."""
    data = np.asarray(data, dtype=np.float64)
    return np.hstack([data, np.full((data.shape[0], horizon - 1), np.nan)])


def forecast_block(s: KalmanState, data, horizon: int):
    """forecasting.jl:242-247: vcat(factors, states, preds)[:, end-h+1:end] of predict on the padded data."""
    r = predict(s, pad_nan(data, horizon))
    return np.vstack([r["factors"][:, -horizon:], r["states"][:, -horizon:], r["preds"][:, -horizon:]])
