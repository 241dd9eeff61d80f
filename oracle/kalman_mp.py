"""High-precision (mpmath, 40 digits) ground truth of the reference Kalman recursion.

TEST INFRASTRUCTURE ONLY (see kalman_oracle.py).  Same recursion and quirks as
kalman_oracle.py — filter.jl:1-10, :12-80, :125-209 — but in exact-enough
arithmetic on the same FP64 inputs, so a test can tell whether a difference
between the HIP kernel and the FP64 oracle is the kernel's error or the
reference algorithm's own rounding (the dense path's ``I − KZ`` cancels badly
when P is large relative to σ²/‖Z'Z‖).
"""
from __future__ import annotations

import math

import mpmath as mp
import numpy as np

from .kalman_oracle import KIND_DNS, KIND_GNS, KIND_TVL, transform_codes, transform_params

mp.mp.dps = 40


def _decode(kind, theta, space):
    M = {KIND_DNS: 3, KIND_TVL: 4, KIND_GNS: 5}[kind]
    th = [mp.mpf(float(x)) for x in theta]
    codes = transform_codes(kind, M)
    if space == 0:
        for i, c in enumerate(codes):
            if c == 1:
                th[i] = mp.exp(th[i])
            elif c == 2:
                y = mp.exp(th[i])
                th[i] = 2 * y / (1 + y) - 1
    lead = {KIND_DNS: 1, KIND_TVL: 0, KIND_GNS: 2}[kind]
    gam = th[:lead]
    k = lead
    sig2 = th[k]
    k += 1
    U = mp.zeros(M, M)
    for j in range(M):
        for i in range(j + 1):
            U[i, j] = th[k]
            k += 1
    Q = U.T * U
    d = mp.matrix(th[k:k + M])
    k += M
    Phi = mp.matrix(M, M)
    for i in range(M):
        for j in range(M):
            Phi[i, j] = th[k]
            k += 1
    return M, gam, sig2, Q, d, Phi


def _pair(lam, m):
    tau = lam * m
    z = mp.exp(-tau)
    s = (1 - z) / tau
    return s, s - z, z


def loglik_mp(kind, maturities, Y, theta, space=0, T_use=None):
    """Returns (loglik as float, beta traj M×(T-1), P traj M×M×(T-1)) in high precision."""
    M, gam, sig2, Q, d, Phi = _decode(kind, theta, space)
    mats = [mp.mpf(float(x)) for x in maturities]
    N = len(mats)
    Y = np.asarray(Y, dtype=np.float64)
    nobs = Y.shape[1] if T_use is None else int(T_use)
    Z = mp.matrix(N, M)
    for i in range(N):
        for j in range(M):
            Z[i, j] = 1
    if kind in (KIND_DNS, KIND_GNS):
        for l, g in enumerate(gam):
            lam = mp.mpf("0.01") + mp.exp(g)
            for i in range(N):
                s, c, _ = _pair(lam, mats[i])
                Z[i, 1 + 2 * l] = s
                Z[i, 2 + 2 * l] = c
    I = mp.eye(M)
    beta = mp.lu_solve(I - Phi, d)
    K2 = mp.matrix(M * M, M * M)
    for i1 in range(M):
        for i2 in range(M):
            for j1 in range(M):
                for j2 in range(M):
                    r, c = i1 * M + i2, j1 * M + j2
                    K2[r, c] = (1 if r == c else 0) - Phi[i1, j1] * Phi[i2, j2]
    vq = mp.matrix([Q[r % M, r // M] for r in range(M * M)])
    vp = mp.lu_solve(K2, vq)
    P = mp.matrix(M, M)
    for r in range(M * M):
        P[r % M, r // M] = vp[r]
    F = mp.zeros(N, N)
    Fi = mp.zeros(N, N)
    v = mp.zeros(N, 1)
    ll = mp.mpf(0)
    c2pi = N * mp.log(2 * mp.pi)
    bt, Pt = [], []
    dead = False
    for t in range(1, nobs):
        y = Y[:, t - 1]
        if kind == KIND_TVL:
            lam = mp.mpf("0.01") + mp.exp(beta[3])
            zi = []
            for i in range(N):
                s, c, z = _pair(lam, mats[i])
                Z[i, 1], Z[i, 2] = s, c
                zi.append(z)
        Zo = Z[:, :3] if kind == KIND_TVL else Z
        bo = mp.matrix([beta[i] for i in range(3)]) if kind == KIND_TVL else beta
        if np.any(np.isnan(y)):
            beta = d + Phi * beta
            P = Phi * P * Phi.T + Q
        else:
            v = mp.matrix(y.tolist()) - Zo * bo
            if kind == KIND_TVL:
                dl = lam - mp.mpf("0.01")
                for i in range(N):
                    dz1 = zi[i] / lam - zi[i] / (lam ** 2 * mats[i])  # filter.jl:43 as written
                    dz2 = mats[i] * zi[i]
                    Z[i, 3] = ((beta[1] + beta[2]) * dz1 + beta[2] * dz2) * dl
            F = Z * P * Z.T + sig2 * mp.eye(N)
            Fi = mp.inverse(F)
            K = P * Z.T * Fi
            beta = d + Phi * (beta + K * v)
            P = Phi * (I - K * Z) * P * Phi.T + Q
        bt.append([float(beta[i]) for i in range(M)])
        Pt.append([[float(P[i, j]) for j in range(M)] for i in range(M)])
        if t > 1 and not dead:
            det = mp.det(F)
            if det < 0:
                dead = True
            elif det == 0:
                dead = True
            else:
                q = (v.T * Fi * v)[0]
                ll -= (mp.log(det) + q + c2pi) / 2
    llf = -math.inf if dead else float(ll)
    return llf, np.asarray(bt).T, np.transpose(np.asarray(Pt), (1, 2, 0))
