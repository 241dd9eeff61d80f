"""Device context: one libyfm_hip context per GPU, with the panel kept resident.

Replaces the reference's per-model preallocated buffers
(``src/models/kalman/kalmanbasemodel.jl:53-69``): the panel is uploaded once and
re-used by every objective evaluation until a different panel is passed.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from . import _lib
from .params import gamma_dim, n_params, state_dim


class Engine:
    """Owns one ``yfm_ctx`` (include/yfm.h) on ``device``."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        ctx = self.lib.yfm_create(device)
        if not ctx:
            raise _lib.YFMError(-2, self.lib.yfm_last_error().decode())
        self.ctx = ctypes.c_void_p(ctx)
        self.device = device
        self._panel = None
        self._mats = None

    def close(self):
        if self.ctx:
            self.lib.yfm_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- precision (TVλ arithmetic, include/yfm.h: yfm_set_precision) -----------------
    @property
    def precision(self) -> int:
        return self.lib.yfm_get_precision(self.ctx)

    @precision.setter
    def precision(self, mode: int) -> None:
        _lib.check(self.lib.yfm_set_precision(self.ctx, int(mode)))

    # ---- page-locked host buffers (yfm_alloc_host) ----------------------------------
    def host_array(self, shape, dtype=np.float64) -> np.ndarray:
        """A Fortran-ordered array in page-locked host memory: θ batches and loglik outputs built in
        it reach the device by DMA without a staging copy.  Freed when the array is collected."""
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        ptr = self.lib.yfm_alloc_host(n)
        if not ptr:
            raise _lib.YFMError(-2, self.lib.yfm_last_error().decode())
        buf = (ctypes.c_char * n).from_address(ptr)
        arr = np.frombuffer(buf, dtype=dtype).reshape(shape, order="F")
        import weakref
        weakref.finalize(buf, self.lib.yfm_free_host, ctypes.c_void_p(ptr))
        return arr

    # ---- panel -------------------------------------------------------------------
    def set_panel(self, data, maturities, force: bool = False):
        """data: N×T (maturities × months) like the reference's ``data`` matrix."""
        Y = np.asfortranarray(np.asarray(data, dtype=np.float64))
        m = np.ascontiguousarray(np.asarray(maturities, dtype=np.float64))
        if Y.ndim != 2 or m.ndim != 1 or Y.shape[0] != m.shape[0]:
            raise ValueError(f"panel must be N×T with N = len(maturities); got {Y.shape}, {m.shape}")
        if (not force and self._panel is not None and self._panel.shape == Y.shape
                and np.array_equal(self._panel, Y, equal_nan=True) and np.array_equal(self._mats, m)):
            return
        N, T = Y.shape
        _lib.check(self.lib.yfm_set_panel(self.ctx, _lib.dptr(Y), N, T, _lib.dptr(m)))
        self._panel = Y.copy(order="F")
        self._mats = m.copy()

    @property
    def T(self):
        return 0 if self._panel is None else self._panel.shape[1]

    # ---- batched evaluation ----------------------------------------------------------
    def loglik(self, kind: int, theta, space: int = 0, T_use=None, out=None) -> np.ndarray:
        """Θ: P×B (or a length-P vector).  Returns B logliks (+loglik, get_loss sign), written into
        `out` when given (e.g. a page-locked `host_array`)."""
        Th = np.asarray(theta, dtype=np.float64)
        if Th.ndim == 1:
            Th = Th[:, None]
        Th = np.asfortranarray(Th)
        P, B = Th.shape
        if P != n_params(kind):
            raise ValueError(f"theta has {P} rows, model kind {kind} needs {n_params(kind)}")
        if out is None:
            out = np.empty(B, dtype=np.float64)
        elif out.shape != (B,) or out.dtype != np.float64 or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous float64 vector of length B")
        tu = None if T_use is None else np.ascontiguousarray(np.broadcast_to(T_use, (B,)), dtype=np.int32)
        _lib.check(self.lib.yfm_loglik_batch(self.ctx, kind, space, _lib.dptr(Th), P, B, _lib.iptr(tu),
                                             _lib.dptr(out)))
        return out

    def loglik_device(self, kind: int, d_theta: int, P: int, B: int, d_out: int, space: int = 0,
                      d_T_use: int | None = None, stream: int | None = None) -> None:
        """Device-pointer variant (raw addresses, e.g. ``torch.Tensor.data_ptr()``); asynchronous on ``stream``."""
        _lib.check(self.lib.yfm_loglik_batch_device(self.ctx, kind, space, ctypes.c_void_p(d_theta), P, B,
                                                    ctypes.c_void_p(d_T_use) if d_T_use else None,
                                                    ctypes.c_void_p(d_out),
                                                    ctypes.c_void_p(stream) if stream else None))

    def filter_states(self, kind: int, theta, space: int = 0, T_use=None):
        """Returns (loglik[B], beta[M, T-1, B], P[M, M, T-1, B]) — a_{t+1|t}, P_{t+1|t} after each filter! call."""
        Th = np.asfortranarray(np.atleast_2d(np.asarray(theta, dtype=np.float64).T).T)
        P, B = Th.shape
        M = state_dim(kind)
        T = self.T
        out = np.empty(B)
        beta = np.empty((M, max(T - 1, 0), B), order="F")
        Pm = np.empty((M, M, max(T - 1, 0), B), order="F")
        tu = None if T_use is None else np.ascontiguousarray(np.broadcast_to(T_use, (B,)), dtype=np.int32)
        _lib.check(self.lib.yfm_filter_states(self.ctx, kind, space, _lib.dptr(Th), P, B, _lib.iptr(tu),
                                              _lib.dptr(beta), _lib.dptr(Pm), _lib.dptr(out)))
        return out, beta, Pm

    @staticmethod
    def _batch(theta, kind):
        Th = np.asfortranarray(np.atleast_2d(np.asarray(theta, dtype=np.float64).T).T)
        if Th.shape[0] != n_params(kind):
            raise ValueError(f"theta has {Th.shape[0]} rows, model kind {kind} needs {n_params(kind)}")
        return Th

    @staticmethod
    def _tuse(T_use, B):
        return None if T_use is None else np.ascontiguousarray(np.broadcast_to(T_use, (B,)), dtype=np.int32)

    def predict(self, kind: int, theta, space: int = 1, T_use=None, horizon: int = 1) -> dict:
        """predict (filter.jl:250-282) per θ_b on hcat(data[:, :T_b], NaN × (horizon−1)).
        Returns arrays with a trailing batch axis: preds/factor_loadings_1/2 (N, ncol, B),
        factors (M, ncol, B), states (L, ncol, B), ncol = T + horizon − 1."""
        Th = self._batch(theta, kind)
        P, B = Th.shape
        M, L, N = state_dim(kind), gamma_dim(kind), self._panel.shape[0]
        ncol = self.T + horizon - 1
        preds = np.empty((N, ncol, B), order="F")
        fl1 = np.empty((N, ncol, B), order="F")
        fl2 = np.empty((N, ncol, B), order="F")
        fac = np.empty((M, ncol, B), order="F")
        st = np.empty((L, ncol, B), order="F")
        _lib.check(self.lib.yfm_predict(self.ctx, kind, space, _lib.dptr(Th), P, B, _lib.iptr(self._tuse(T_use, B)),
                                        horizon, _lib.dptr(preds), _lib.dptr(fac), _lib.dptr(st), _lib.dptr(fl1),
                                        _lib.dptr(fl2)))
        return dict(preds=preds, factors=fac, states=st, factor_loadings_1=fl1, factor_loadings_2=fl2)

    def forecast(self, kind: int, theta, space: int = 1, T_use=None, horizon: int = 1) -> np.ndarray:
        """forecasting.jl:236-250 blocks vcat(factors, states, preds)[:, end-h+1:end]: (M+L+N, h, B)."""
        Th = self._batch(theta, kind)
        P, B = Th.shape
        R = state_dim(kind) + gamma_dim(kind) + self._panel.shape[0]
        out = np.empty((R, horizon, B), order="F")
        _lib.check(self.lib.yfm_forecast(self.ctx, kind, space, _lib.dptr(Th), P, B, _lib.iptr(self._tuse(T_use, B)),
                                         horizon, _lib.dptr(out)))
        return out

    def loss_array(self, kind: int, theta, space: int = 1, T_use=None, K: int = 1) -> np.ndarray:
        """get_loss_array (filter.jl:211-247) per θ_b: (T−1, B)."""
        Th = self._batch(theta, kind)
        P, B = Th.shape
        out = np.empty((max(self.T - 1, 0), B), order="F")
        _lib.check(self.lib.yfm_loss_array(self.ctx, kind, space, _lib.dptr(Th), P, B,
                                           _lib.iptr(self._tuse(T_use, B)), K, _lib.dptr(out)))
        return out

    def estimate(self, kind: int, theta0, space: int = 1, T_use=None, iterations: int = 500, g_tol: float = 1e-6,
                 max_group_iters: int = 10, tol: float = 1e-8) -> dict:
        """Batched estimate_steps! (optimization.jl:137-312): one Nelder–Mead chain per column of Θ₀ (P×R),
        on window T_use[r].  Returns theta_c (P×R), p (P×R unconstrained), init_c (P×R: the reference's
        init_p — the sanitised, rescaled start, constrained), ll (R), status (R), n_evals."""
        Th = self._batch(theta0, kind)
        P, R = Th.shape
        th_c = np.empty((P, R), order="F")
        p = np.empty((P, R), order="F")
        init_c = np.empty((P, R), order="F")
        ll = np.empty(R)
        st = np.empty(R, dtype=np.int32)
        ne = ctypes.c_longlong(0)
        _lib.check(self.lib.yfm_estimate(self.ctx, kind, space, _lib.dptr(Th), P, R, _lib.iptr(self._tuse(T_use, R)),
                                         iterations, g_tol, max_group_iters, tol, _lib.dptr(th_c), _lib.dptr(p),
                                         _lib.dptr(init_c), _lib.dptr(ll), _lib.iptr(st), ctypes.byref(ne)))
        return dict(theta_c=th_c, p=p, init_c=init_c, ll=ll, status=st, n_evals=ne.value)

    def last_flags(self):
        a, b = ctypes.c_longlong(0), ctypes.c_longlong(0)
        _lib.check(self.lib.yfm_last_batch_flags(self.ctx, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_deferred(self) -> int:
        """Candidates of the last batch evaluated on the double-double capacitance path (fixed-loading
        models with an ill-conditioned Z'Z; include/yfm.h yfm_last_batch_deferred)."""
        n = ctypes.c_longlong(0)
        _lib.check(self.lib.yfm_last_batch_deferred(self.ctx, ctypes.byref(n)))
        return n.value

    def last_steady(self) -> int:
        """Wave-steps (64 filter steps each) of the last batch that ran the DNS kernel's frozen-covariance
        steady state (include/yfm.h yfm_last_batch_steady)."""
        n = ctypes.c_longlong(0)
        _lib.check(self.lib.yfm_last_batch_steady(self.ctx, ctypes.byref(n)))
        return int(n.value)


_engines: dict[int, Engine] = {}
_lock = threading.Lock()


def get_engine(device: int = 0) -> Engine:
    with _lock:
        e = _engines.get(device)
        if e is None:
            e = Engine(device)
            _engines[device] = e
        return e
