"""ctypes binding of libyfm_hip.so (include/yfm.h).

This is the same binding a Julia `@ccall` shim performs: plain
pointers and sizes, no torch types.  Loading fails loudly when the library is
missing — there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os
import sys
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("YFM_LIB", _HERE / "libyfm_hip.so"))

# Every symbol include/yfm.h declares, with its ctypes signature.
_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)
_LL = ctypes.POINTER(ctypes.c_longlong)
_V = ctypes.c_void_p
SIGNATURES = {
    "yfm_abi_version": (ctypes.c_int, []),
    "yfm_param_count": (ctypes.c_int, [ctypes.c_int]),
    "yfm_state_dim": (ctypes.c_int, [ctypes.c_int]),
    "yfm_last_error": (ctypes.c_char_p, []),
    "yfm_create": (_V, [ctypes.c_int]),
    "yfm_destroy": (None, [_V]),
    "yfm_set_panel": (ctypes.c_int, [_V, _D, ctypes.c_int, ctypes.c_int, _D]),
    "yfm_loglik_batch": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int, ctypes.c_int, _I, _D]),
    "yfm_loglik_batch_device": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _V, ctypes.c_int, ctypes.c_int, _V,
                                               _V, _V]),
    "yfm_filter_states": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int, ctypes.c_int, _I, _D, _D,
                                         _D]),
    "yfm_last_batch_flags": (ctypes.c_int, [_V, _LL, _LL]),
    "yfm_last_batch_deferred": (ctypes.c_int, [_V, _LL]),
    "yfm_last_batch_steady": (ctypes.c_int, [_V, _LL]),
    "yfm_gamma_dim": (ctypes.c_int, [ctypes.c_int]),
    "yfm_predict": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int, ctypes.c_int, _I, ctypes.c_int,
                                   _D, _D, _D, _D, _D]),
    "yfm_forecast": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int, ctypes.c_int, _I, ctypes.c_int,
                                    _D]),
    "yfm_estimate": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int, ctypes.c_int, _I, ctypes.c_int,
                                    ctypes.c_double, ctypes.c_int, ctypes.c_double, _D, _D, _D, _D, _I, _LL]),
    "yfm_alloc_host": (_V, [ctypes.c_size_t]),
    "yfm_free_host": (ctypes.c_int, [_V]),
    "yfm_set_precision": (ctypes.c_int, [_V, ctypes.c_int]),
    "yfm_get_precision": (ctypes.c_int, [_V]),
    "yfm_loss_array": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _D, ctypes.c_int, ctypes.c_int, _I, ctypes.c_int,
                                      _D]),
}

ABI_VERSION = 2

# precision modes (include/yfm.h: enum yfm_precision)
PREC_CERTIFIED, PREC_FP64 = 0, 1


class YFMError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libyfm_hip error {code}: {msg}")
        self.code = code


_lib = None


def load() -> ctypes.CDLL:
    """Load libyfm_hip.so once.  Import torch first when both are used in one
    process: torch ships its own libamdhip64.so.7 and the dynamic loader then
    binds this library to that same runtime (same SONAME)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not found — build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (no CPU fallback exists)")
    lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.yfm_abi_version() != ABI_VERSION:
        raise ImportError(f"ABI mismatch: library {lib.yfm_abi_version()} vs binding {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.yfm_last_error().decode("utf-8", "replace") if _lib is not None else "?"
        raise YFMError(rc, msg)


def dptr(a) -> ctypes.POINTER(ctypes.c_double):
    return a.ctypes.data_as(_D)


def iptr(a):
    return None if a is None else a.ctypes.data_as(_I)


def loaded_path() -> str:
    return str(LIB_PATH) if _lib is not None else ""


if __name__ == "__main__":  # pragma: no cover
    print(load(), file=sys.stderr)
