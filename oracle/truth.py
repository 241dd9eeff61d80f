"""ctypes wrappers of the quad-precision truth (oracle/yfm_truth.c) and the C dense oracle.

TEST INFRASTRUCTURE ONLY (see kalman_oracle.py): tests/, smoke() and bench.py's
cpu_baseline / parity leg use these as checkers; the product never imports them.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)
_libs: dict = {}


def _lib(name: str):
    if name not in _libs:
        path = HERE / f"lib{name}.so"
        if not path.exists():
            subprocess.run(["make", "-C", str(HERE), "-s"], check=True)
        _libs[name] = ctypes.CDLL(str(path))
    return _libs[name]


def _threads(n):
    """n, else every CPU this process may use: its affinity mask, capped by the cgroup CPU quota."""
    if n:
        return n
    aff = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, min(aff, int(float(q) / float(p))))
    except (OSError, ValueError):
        pass
    return aff


def _batched(fn, kind, Y, mats, Theta, space, T_use, nthreads):
    Y = np.asfortranarray(Y, dtype=np.float64)
    Th = np.asfortranarray(Theta, dtype=np.float64)
    mats = np.ascontiguousarray(mats, dtype=np.float64)
    B = Th.shape[1]
    out = np.empty(B)
    tu = None if T_use is None else np.ascontiguousarray(T_use, dtype=np.int32)
    if B:
        fn(kind, space, Y.ctypes.data_as(_D), Y.shape[0], Y.shape[1], mats.ctypes.data_as(_D),
           Th.ctypes.data_as(_D), Th.shape[0], B, None if tu is None else tu.ctypes.data_as(_I),
           out.ctypes.data_as(_D), _threads(nthreads))
    return out


def loglik_truth(kind, Y, mats, Theta, space=0, T_use=None, nthreads=0) -> np.ndarray:
    """+loglik of every column of Θ in binary128 arithmetic (the exact-arithmetic value of the
    reference recursion to ~1e-20 relative); NaN where the reference throws."""
    return _batched(_lib("yfm_truth").yfm_truth_loglik, kind, Y, mats, Theta, space, T_use, nthreads)


def loglik_oracle(kind, Y, mats, Theta, space=0, T_use=None, nthreads=0) -> np.ndarray:
    """The C dense FP64 restatement of the reference (oracle/yfm_oracle.c)."""
    return _batched(_lib("yfm_oracle").yfm_oracle_loglik, kind, Y, mats, Theta, space, T_use, nthreads)


def states_truth(kind, Y, mats, theta, space=0):
    """(loglik, β M×(T−1), P M×M×(T−1)) of one candidate in binary128 arithmetic."""
    from .kalman_oracle import KIND_DNS, KIND_TVL
    M = 3 if kind == KIND_DNS else 4 if kind == KIND_TVL else 5
    Y = np.asfortranarray(Y, dtype=np.float64)
    N, T = Y.shape
    th = np.ascontiguousarray(theta, dtype=np.float64)
    mats = np.ascontiguousarray(mats, dtype=np.float64)
    beta = np.zeros((M, max(T - 1, 0)), order="F")
    P = np.zeros((M, M, max(T - 1, 0)), order="F")
    ll = ctypes.c_double()
    _lib("yfm_truth").yfm_truth_filter_states(kind, space, Y.ctypes.data_as(_D), N, T, mats.ctypes.data_as(_D),
                                              th.ctypes.data_as(_D), beta.ctypes.data_as(_D), P.ctypes.data_as(_D),
                                              ctypes.byref(ll))
    return ll.value, beta, P


def predict_states_truth(kind, Y, mats, theta, horizon=1, space=1):
    """State trajectory of predict (filter.jl:250-282) on hcat(Y, NaN × (horizon − 1)) in binary128:
    A (T + horizon, M), A[j] = β after filter! step j + 1 (the final NaN step included) — the
    layout of kalman_ld.predict_traj_tvl for one candidate."""
    Y = np.asarray(Y, dtype=np.float64)
    pad = np.hstack([Y, np.full((Y.shape[0], horizon + 1), np.nan)])
    _, beta, _ = states_truth(kind, pad, mats, theta, space)
    return beta.T
