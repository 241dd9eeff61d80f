"""CPU restatement of the estimation driver for Kalman models — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module,
as the checker; the product path (libyfm_hip.so: yfm_estimate_nm) never calls it.

Restates, per chain (one window / one start):

* ``estimate_steps!`` — src/optimization.jl:137-312, for a Kalman model whose parameters
  all sit in group "1" (kalmanbasemodel.jl:150-159): untransform + sanitize the start
  (:157-162, :422-432), the ×0.95 rescaling of a non-finite start (:173-184), the outer
  block-coordinate loop (max_group_iters, |ΔLL| < tol, :218-281), the exception rules
  (rethrow on iteration 1, abort later, :249-257), transform of the result (:301).
* the optimiser it calls for group "1" — ``Optim.NelderMead()`` with ``opt1`` (500
  iterations, g_tol 1e-6; optimization.jl:442-451, :479).  Optim.jl (pinned by the
  reference's compat bound ``Optim = "1.13.2"``, Project.toml:42) is a third-party
  dependency absent from /root/reference; its published algorithm is restated here:
    - AdaptiveParameters (Gao & Han 2012): α = 1, β = 1 + 2/n, γ = 0.75 − 1/(2n), δ = 1 − 1/n;
    - AffineSimplexer(a = 0.025, b = 0.5): vertex j+1 = x0 with x_j ← (1 + b)·x_j + a;
    - each iteration: centroid of all vertices but the worst (storage order sum × 1/n),
      reflection; expansion if better than the best (then the new vertex becomes the
      lowest without re-sorting); reflection accepted if better than the second worst;
      else outside / inside contraction, or a shrink towards the best vertex;
      stable sortperm of the vertex values after every non-expansion step;
    - stop when the population std of the vertex values ≤ g_tol ("nm_x", the
      g_converged hijack of NelderMead) or after `iterations` iterations;
    - minimizer: the best vertex, or the centroid of all but the worst if that is lower.
  Parity is "unpinned" against Optim.jl itself (no Julia here); the GPU path is checked
  against this restatement bit for bit when both are driven by the same objective values.

The objective is injected: ``f(θ) -> −loglik`` (compute_loss, optimization.jl:10-23), raising
:class:`InitThrow` where the reference's initialize_filter throws.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


class InitThrow(Exception):
    """compute_loss threw (singular I − Φ or I − Φ⊗Φ in initialize_filter, filter.jl:4/:7)."""


def nm_parameters(n: int):
    """Optim.AdaptiveParameters(α=1, β=1, γ=0.75, δ=1) → (α, β + 2/n, γ − 1/2n, δ − 1/n)."""
    return 1.0, 1.0 + 2.0 / n, 0.75 - 1.0 / (2 * n), 1.0 - 1.0 / n


def affine_simplex(x0, a=0.025, b=0.5):
    n = len(x0)
    S = [np.array(x0, dtype=np.float64) for _ in range(n + 1)]
    for j in range(n):
        S[j + 1][j] = (1.0 + b) * S[j + 1][j] + a
    return S


def centroid(S, h):
    n = len(S) - 1
    c = np.zeros_like(S[0])
    for i in range(n + 1):
        if i != h:
            c = c + S[i]
    return c * (1.0 / n)


def nm_x(fs):
    """sqrt(var(y) · n/(n+1)) = population standard deviation of the vertex values."""
    y = np.asarray(fs, dtype=np.float64)
    m = len(y)
    with np.errstate(all="ignore"):
        mu = sum(y) / m
        q = 0.0
        for v in y:
            d = v - mu
            q = q + d * d
        return math.sqrt(q / (m - 1) * ((m - 1) / m))


def sortperm(fs):
    return sorted(range(len(fs)), key=lambda i: (math.isnan(fs[i]), fs[i]))  # stable, NaN last


@dataclass
class NMResult:
    x: np.ndarray
    f: float
    iterations: int
    f_calls: int


def nelder_mead(f, x0, iterations=500, g_tol=1e-6) -> NMResult:
    """Optim.optimize(f, x0, NelderMead(), Options(iterations, g_tol)) — minimizer and minimum."""
    n = len(x0)
    m = n + 1
    al, be, ga, de = nm_parameters(n)
    calls = [0]

    def val(x):
        calls[0] += 1
        return float(f(x))

    S = affine_simplex(x0)
    fs = [val(x) for x in S]
    order = sortperm(fs)
    it = 0
    converged = False
    while not converged and it < iterations:
        it += 1
        shrink = False
        xc = centroid(S, order[m - 1])
        xl = S[order[0]].copy()
        xh = S[order[m - 1]].copy()
        fl, fsh, fh = fs[order[0]], fs[order[n - 1]], fs[order[m - 1]]
        xr = xc + al * (xc - xh)
        fr = val(xr)
        if fr < fl:
            xe = xc + be * (xr - xc)
            fe = val(xe)
            ih = order[m - 1]
            if fe < fr:
                S[ih], fs[ih] = xe, fe
            else:
                S[ih], fs[ih] = xr, fr
            order = [ih] + order[:m - 1]
        elif fr < fsh:
            S[order[m - 1]], fs[order[m - 1]] = xr, fr
            order = sortperm(fs)
        else:
            if fr < fh:
                xo = xc + ga * (xr - xc)
                fo = val(xo)
                if fo < fr:
                    S[order[m - 1]], fs[order[m - 1]] = xo, fo
                    order = sortperm(fs)
                else:
                    shrink = True
            else:
                xi = xc - ga * (xr - xc)
                fi = val(xi)
                if fi < fh:
                    S[order[m - 1]], fs[order[m - 1]] = xi, fi
                    order = sortperm(fs)
                else:
                    shrink = True
        if shrink:
            for i in range(1, m):
                o = order[i]
                S[o] = xl + de * (S[o] - xl)
                fs[o] = val(S[o])
            order = sortperm(fs)
        converged = nm_x(fs) <= g_tol
    # after_while!: best vertex vs the centroid of all but the worst
    order = sortperm(fs)
    xcm = centroid(S, order[m - 1])
    fcm = val(xcm)
    i_min = min(range(m), key=lambda i: (fs[i], i)) if not any(map(math.isnan, fs)) else \
        next(i for i in range(m) if math.isnan(fs[i]))
    x_min, f_min = S[i_min], fs[i_min]
    if fcm < f_min:
        x_min, f_min = xcm, fcm
    return NMResult(np.array(x_min), f_min, it, calls[0])


@dataclass
class EstimateResult:
    theta_c: np.ndarray      # transform_params(best_p)
    ll: float                # prev_ll of estimate_steps!
    p: np.ndarray            # unconstrained optimum
    status: int              # 0 ok; 1 the reference throws; 2 aborted after iteration 1
    outer_iterations: int
    f_calls: int


def estimate_steps(f, theta0_c, transform, untransform, max_group_iters=10, tol=1e-8, iterations=500,
                   g_tol=1e-6) -> EstimateResult:
    """optimization.jl:137-312 for one start (try_initializations returns the start unchanged for
    Kalman models, :33-35, so n_starts = 1) with every parameter in group "1"."""
    p = np.asarray(untransform(np.asarray(theta0_c, dtype=np.float64)), dtype=np.float64)
    p = np.where(np.isfinite(p), p, 0.0)  # _sanitize_parameters
    calls = 0

    def loss(x):
        nonlocal calls
        calls += 1
        return float(f(x))

    try:
        ll = -loss(p)
        for _ in range(10):  # :173-184
            if not math.isfinite(ll):
                p = p * 0.95
                ll = -loss(p)
            else:
                break
    except InitThrow:
        return EstimateResult(np.full_like(p, np.nan), math.nan, p, 1, 0, calls)
    prev_ll = -math.inf
    outer = 0
    status = 0
    for it in range(1, max_group_iters + 1):
        outer = it
        try:
            res = nelder_mead(f, p.copy(), iterations=iterations, g_tol=g_tol)
            calls += res.f_calls
        except InitThrow:
            if it == 1:
                return EstimateResult(np.full_like(p, np.nan), math.nan, p, 1, it, calls)
            status = 2
            break
        p = res.x.copy()
        ll = -loss(p)
        d = ll - prev_ll
        if abs(d) < tol:
            prev_ll = ll
            break
        prev_ll = ll
    return EstimateResult(np.asarray(transform(p)), prev_ll, p, status, outer, calls)
