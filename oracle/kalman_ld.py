"""Extended-precision (x87 long double, 64-bit mantissa) batched truth proxy.

TEST INFRASTRUCTURE ONLY (see kalman_oracle.py).  Vectorised over candidates so a
test can adjudicate thousands of T = 600 evaluations in seconds — where the
40-digit kalman_mp.py would take minutes per candidate.

It restates get_loss (filter.jl:182-209) for the fixed-loading models in the
CAPACITANCE form — B̃ = σ²I + P·Z'Z, pivoted Gaussian elimination — i.e. an
algebra independent of the HIP kernel's collapsed form, carried out with ~11
more bits than FP64, so its own error is ~κ·5e-20.  tests/test_oracle.py pins it
to the 40-digit mpmath truth.  Initialisation follows filter.jl:1-10 (the
M²×M² Lyapunov system, solved by pivoted elimination).  NaN columns are not
supported here (use kalman_oracle.py / kalman_mp.py for those).
"""
from __future__ import annotations

import numpy as np

LD = np.longdouble


def _gesv(A, Bm):
    """Batched Gaussian elimination with partial pivoting. A: b×n×n, Bm: b×n×r (any float dtype)."""
    A = A.copy()
    X = Bm.copy()
    b, n, _ = A.shape
    ar = np.arange(b)
    sign = np.ones(b, dtype=A.dtype)
    for k in range(n):
        p = k + np.argmax(np.abs(A[:, k:, k]), axis=1)
        sw = p != k
        sign[sw] = -sign[sw]
        rk = A[ar, k].copy()
        A[ar, k] = A[ar, p]
        A[ar, p] = rk
        xk = X[ar, k].copy()
        X[ar, k] = X[ar, p]
        X[ar, p] = xk
        for i in range(k + 1, n):
            with np.errstate(all="ignore"):
                l = A[:, i, k] / A[:, k, k]
            A[:, i, k:] -= l[:, None] * A[:, k, k:]
            X[:, i] -= l[:, None] * X[:, k]
    for k in range(n - 1, -1, -1):
        s = X[:, k] - np.einsum("bj,bjr->br", A[:, k, k + 1:], X[:, k + 1:])
        with np.errstate(all="ignore"):
            X[:, k] = s / A[:, k, k][:, None]
    det = sign * np.prod(np.diagonal(A, axis1=1, axis2=2), axis=1)
    return X, det


def _transform(codes, theta):
    th = theta.astype(LD)
    out = th.copy()
    with np.errstate(all="ignore"):
        pos = codes == 1
        out[pos] = np.exp(th[pos])
        r = codes == 2
        y = np.exp(th[r])
        out[r] = 2 * y / (1 + y) - 1
    return out


def loglik_ld(kind: int, maturities, Y, Theta, space: int = 0) -> np.ndarray:
    """+loglik for every column of Θ (P×B) on panel Y (N×T, no NaN); NaN where the reference throws."""
    from .kalman_oracle import KIND_DNS, KIND_GNS, transform_codes
    M = 3 if kind == KIND_DNS else 5
    lead = 1 if kind == KIND_DNS else 2
    if kind not in (KIND_DNS, KIND_GNS):
        raise ValueError("fixed-loading kinds only")
    codes = np.asarray(transform_codes(kind, M))
    Theta = np.asarray(Theta, dtype=np.float64)
    B = Theta.shape[1]
    tc = _transform(codes[:, None].repeat(B, 1), Theta) if space == 0 else Theta.astype(LD)
    k = lead
    sig2 = tc[k]
    k += 1
    U = np.zeros((B, M, M), LD)
    for j in range(M):
        for i in range(j + 1):
            U[:, i, j] = tc[k]
            k += 1
    Q = np.einsum("bli,blj->bij", U, U)
    d = tc[k:k + M].T.copy()
    k += M
    Phi = tc[k:k + M * M].T.reshape(B, M, M).copy()
    mats = np.asarray(maturities, dtype=np.float64).astype(LD)
    N = len(mats)
    Z = np.ones((B, N, M), LD)
    for l in range(lead):
        lam = LD(0.01) + np.exp(tc[l])
        tau = lam[:, None] * mats[None, :]
        z = np.exp(-tau)
        Z[:, :, 1 + 2 * l] = (1 - z) / tau
        Z[:, :, 2 + 2 * l] = Z[:, :, 1 + 2 * l] - z
    G = np.einsum("bni,bnj->bij", Z, Z)
    I = np.eye(M, dtype=LD)
    beta, det0 = _gesv(I - Phi, d[..., None])
    beta = beta[..., 0]
    K2 = np.eye(M * M, dtype=LD)[None] - np.einsum("bij,bkl->bikjl", Phi, Phi).reshape(B, M * M, M * M)
    vq = np.transpose(Q, (0, 2, 1)).reshape(B, M * M)
    vp, det1 = _gesv(K2, vq[..., None])
    P = np.transpose(vp[..., 0].reshape(B, M, M), (0, 2, 1))
    throws = (det0 == 0) | (det1 == 0)
    Y = np.asarray(Y, dtype=np.float64).astype(LD)
    T = Y.shape[1]
    lsum = np.zeros(B, LD)
    qsum = np.zeros(B, LD)
    neg = np.zeros(B, bool)
    with np.errstate(all="ignore"):
        for t in range(T - 1):
            y = Y[:, t]
            zy = np.einsum("bni,n->bi", Z, y)
            u = zy - np.einsum("bij,bj->bi", G, beta)
            r = y[None, :] - np.einsum("bni,bi->bn", Z, beta)
            vv = np.einsum("bn,bn->b", r, r)
            Bt = sig2[:, None, None] * I + P @ G
            W, det = _gesv(Bt, P)
            W = (W + np.transpose(W, (0, 2, 1))) / 2
            kv = np.einsum("bij,bj->bi", W, u)
            q = (vv - np.einsum("bi,bi->b", u, kv)) / sig2
            beta = d + np.einsum("bij,bj->bi", Phi, beta + kv)
            P = sig2[:, None, None] * (Phi @ W @ np.transpose(Phi, (0, 2, 1))) + Q
            if t >= 1:
                lsum += np.log(np.abs(det))
                qsum += q
                neg |= det < 0
        const = (N - M) * np.log(sig2) + N * np.log(2 * LD(np.pi))
        ll = (-((T - 2) * const + lsum + qsum) / 2).astype(np.float64)
    ll[neg | ~np.isfinite(ll)] = -np.inf
    ll[throws] = np.nan
    return ll


def loglik_ld_tvl(maturities, Y, Theta, space: int = 0, T_use=None, dtype=LD) -> np.ndarray:
    """TVλ EKF (filter.jl:12-80, tvλdns.jl:53-64) in extended precision, capacitance form,
    batched over the columns of Θ (P×B); NaN where the reference throws.  NaN columns are
    prediction-only steps whose loglik term repeats the previous one (stale F, v:
    filter.jl:13-29, :195); T_use[b] restricts candidate b to data[:, 1:T_use[b]].
    The Jacobian column keeps the reference's dZ1 = z/λ − z/(λ²m) (filter.jl:43)."""
    from .kalman_oracle import KIND_TVL, transform_codes
    M = 4
    codes = np.asarray(transform_codes(KIND_TVL, M))
    Theta = np.asarray(Theta, dtype=np.float64)
    B = Theta.shape[1]
    tc = _transform(codes[:, None].repeat(B, 1), Theta).astype(dtype) if space == 0 else Theta.astype(dtype)
    sig2 = tc[0]
    k = 1
    U = np.zeros((B, M, M), dtype)
    for j in range(M):
        for i in range(j + 1):
            U[:, i, j] = tc[k]
            k += 1
    Q = np.einsum("bli,blj->bij", U, U)
    d = tc[k:k + M].T.copy()
    k += M
    Phi = tc[k:k + M * M].T.reshape(B, M, M).copy()
    mats = np.asarray(maturities, dtype=np.float64).astype(dtype)
    N = len(mats)
    I = np.eye(M, dtype=dtype)
    beta, det0 = _gesv(I - Phi, d[..., None])
    beta = beta[..., 0]
    K2 = np.eye(M * M, dtype=dtype)[None] - np.einsum("bij,bkl->bikjl", Phi, Phi).reshape(B, M * M, M * M)
    vq = np.transpose(Q, (0, 2, 1)).reshape(B, M * M)
    vp, det1 = _gesv(K2, vq[..., None])
    P = np.transpose(vp[..., 0].reshape(B, M, M), (0, 2, 1))
    throws = (det0 == 0) | (det1 == 0)
    Y = np.asarray(Y, dtype=np.float64).astype(dtype)
    T = Y.shape[1]
    lsum = np.zeros(B, dtype)
    qsum = np.zeros(B, dtype)
    neg = np.zeros(B, bool)
    Z = np.ones((B, N, M), dtype)
    nobs = np.full(B, T) if T_use is None else np.asarray(T_use)
    last_det = np.zeros(B, dtype)
    last_q = np.zeros(B, dtype)
    with np.errstate(all="ignore"):
        for t in range(int(nobs.max()) - 1):
            act = t < nobs - 1
            if np.isnan(Y[:, t]).any():
                beta_n = d + np.einsum("bij,bj->bi", Phi, beta)
                P_n = Phi @ P @ np.transpose(Phi, (0, 2, 1)) + Q
                beta = np.where(act[:, None], beta_n, beta)
                P = np.where(act[:, None, None], P_n, P)
                if t >= 1:
                    lsum += np.where(act, np.log(np.abs(last_det)), 0)
                    qsum += np.where(act, last_q, 0)
                    neg |= act & (last_det < 0)
                continue
            lam = dtype(0.01) + np.exp(beta[:, 3])
            tau = lam[:, None] * mats[None, :]
            z = np.exp(-tau)
            Z[:, :, 1] = (1 - z) / tau
            Z[:, :, 2] = Z[:, :, 1] - z
            dl = lam - dtype(0.01)
            dz1 = z / lam[:, None] - z / (lam[:, None] ** 2 * mats[None, :])
            dz2 = mats[None, :] * z
            Z[:, :, 3] = ((beta[:, 1] + beta[:, 2])[:, None] * dz1 + beta[:, 2][:, None] * dz2) * dl[:, None]
            r = Y[:, t][None, :] - np.einsum("bni,bi->bn", Z[:, :, :3], beta[:, :3])
            u = np.einsum("bni,bn->bi", Z, r)
            vv = np.einsum("bn,bn->b", r, r)
            G = np.einsum("bni,bnj->bij", Z, Z)
            Bt = sig2[:, None, None] * I + P @ G
            W, det = _gesv(Bt, P)
            W = (W + np.transpose(W, (0, 2, 1))) / 2
            kv = np.einsum("bij,bj->bi", W, u)
            q = (vv - np.einsum("bi,bi->b", u, kv)) / sig2
            beta = np.where(act[:, None], d + np.einsum("bij,bj->bi", Phi, beta + kv), beta)
            P = np.where(act[:, None, None], sig2[:, None, None] * (Phi @ W @ np.transpose(Phi, (0, 2, 1))) + Q, P)
            last_det = np.where(act, det, last_det)
            last_q = np.where(act, q, last_q)
            if t >= 1:
                lsum += np.where(act, np.log(np.abs(det)), 0)
                qsum += np.where(act, q, 0)
                neg |= act & (det < 0)
        const = (N - M) * np.log(sig2) + N * np.log(2 * dtype(np.pi))
        nterms = np.maximum(nobs - 2, 0)
        ll = np.where(nterms > 0, -(nterms * const + lsum + qsum) / 2, 0).astype(np.float64)
    ll[neg | ~np.isfinite(ll)] = -np.inf
    ll[throws] = np.nan
    return ll


def predict_traj_tvl(maturities, Y, Theta_c, horizon: int = 1, T_use=None, dtype=LD) -> np.ndarray:
    """TVλ state trajectory of predict (filter.jl:250-282) on hcat(Y[:, 1:T_b], NaN × (horizon−1))
    in `dtype` arithmetic (capacitance form, as loglik_ld_tvl): returns A (B, T + horizon, 4),
    A[b, j] = β after filter! step j + 1 (the final NaN step included), NaN past candidate b's
    T_b + horizon steps.  Used as the truth proxy (long double) and as a second FP64 restatement
    (dtype = float64) for the noise floor of ill-conditioned EKF runs."""
    from .kalman_oracle import KIND_TVL, transform_codes  # noqa: F401
    M = 4
    Theta_c = np.asarray(Theta_c, dtype=np.float64)
    B = Theta_c.shape[1]
    tc = Theta_c.astype(dtype)
    sig2 = tc[0]
    k = 1
    U = np.zeros((B, M, M), dtype)
    for j in range(M):
        for i in range(j + 1):
            U[:, i, j] = tc[k]
            k += 1
    Q = np.einsum("bli,blj->bij", U, U)
    d = tc[k:k + M].T.copy()
    k += M
    Phi = tc[k:k + M * M].T.reshape(B, M, M).copy()
    mats = np.asarray(maturities, dtype=np.float64).astype(dtype)
    N = len(mats)
    I = np.eye(M, dtype=dtype)
    beta, _ = _gesv(I - Phi, d[..., None])
    beta = beta[..., 0]
    K2 = np.eye(M * M, dtype=dtype)[None] - np.einsum("bij,bkl->bikjl", Phi, Phi).reshape(B, M * M, M * M)
    vq = np.transpose(Q, (0, 2, 1)).reshape(B, M * M)
    vp, _ = _gesv(K2, vq[..., None])
    P = np.transpose(vp[..., 0].reshape(B, M, M), (0, 2, 1))
    Y = np.asarray(Y, dtype=np.float64).astype(dtype)
    T = Y.shape[1]
    nobs = np.full(B, T) if T_use is None else np.asarray(T_use)
    steps = nobs + horizon
    A = np.full((B, T + horizon, M), np.nan)
    Z = np.ones((B, N, M), dtype)
    with np.errstate(all="ignore"):
        for t in range(int(steps.max())):
            act = t < steps
            col = Y[:, t] if t < T else np.full(N, np.nan, dtype)
            nan = (t >= nobs) | bool(np.isnan(col).any())
            beta_p = d + np.einsum("bij,bj->bi", Phi, beta)
            P_p = Phi @ P @ np.transpose(Phi, (0, 2, 1)) + Q
            lam = dtype(0.01) + np.exp(beta[:, 3])
            tau = lam[:, None] * mats[None, :]
            z = np.exp(-tau)
            Z[:, :, 1] = (1 - z) / tau
            Z[:, :, 2] = Z[:, :, 1] - z
            dl = lam - dtype(0.01)
            dz1 = z / lam[:, None] - z / (lam[:, None] ** 2 * mats[None, :])
            dz2 = mats[None, :] * z
            Z[:, :, 3] = ((beta[:, 1] + beta[:, 2])[:, None] * dz1 + beta[:, 2][:, None] * dz2) * dl[:, None]
            r = np.nan_to_num(col)[None, :] - np.einsum("bni,bi->bn", Z[:, :, :3], beta[:, :3])
            u = np.einsum("bni,bn->bi", Z, r)
            G = np.einsum("bni,bnj->bij", Z, Z)
            W, det = _gesv(sig2[:, None, None] * I + P @ G, P)
            W = (W + np.transpose(W, (0, 2, 1))) / 2
            kv = np.einsum("bij,bj->bi", W, u)
            beta_u = d + np.einsum("bij,bj->bi", Phi, beta + kv)
            P_u = sig2[:, None, None] * (Phi @ W @ np.transpose(Phi, (0, 2, 1))) + Q
            upd = act & ~nan & (det != 0)
            prd = act & nan
            beta = np.where(upd[:, None], beta_u, np.where(prd[:, None], beta_p, beta))
            P = np.where(upd[:, None, None], P_u, np.where(prd[:, None, None], P_p, P))
            A[act, t] = beta[act].astype(np.float64)
    return A


def fitted_tvl(maturities, A):
    """ŷ = Z(β₄)[:, 1:3] β[1:3] for states A (..., 4) (filter.jl:15/:33, tvλdns.jl:53-64): (..., N)."""
    m = np.asarray(maturities, dtype=A.dtype)
    with np.errstate(all="ignore"):
        lam = 0.01 + np.exp(A[..., 3:4])
        tau = lam * m
        z = np.exp(-tau)
        s = (1 - z) / tau
        return A[..., 0:1] + s * A[..., 1:2] + (s - z) * A[..., 2:3]
