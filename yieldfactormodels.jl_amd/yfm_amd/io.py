"""Input and result files in the reference's formats.

* :func:`load_data` — ``src/utils/data_management.jl:1-5``: ``<folder>thread_id__<id>__data.csv``
  (N×T, maturities in rows, months in columns) and ``…__maturities.csv``, comma separated.
* :func:`save_results` — ``src/io.jl:4-31``: the filtered-factor, fit, loading, loss and
  parameter CSVs, named ``<results_folder><model_string>__thread_id__<id>__<what>_<data_type>.csv``.
* :func:`writedlm` — Julia's ``DelimitedFiles.writedlm`` for Float64 matrices: one row per
  line, ``,``-separated, each value printed as Julia prints a Float64 (shortest round-trip
  digits; scientific notation ``d.ddde±x`` outside [1e-4, 1e6); ``NaN``, ``Inf``).  Values
  round-trip exactly; the textual match with Julia's printer is unpinned (no Julia here).
* :func:`julia_round` — ``round(x; digits=d)`` (ties to even, ``round(x·10^d)/10^d``), used by
  the forecast records (databaseoperations.jl:251-255, forecasting.jl:263).

The SQLite shard store with Julia ``Serialization`` BLOBs (databaseoperations.jl) is out of
scope: the BLOB format is Julia-specific.  The forecast drivers write the CSVs that
``export_all_csv`` (databaseoperations.jl:654-661) would produce from it.
"""
from __future__ import annotations

import os
from decimal import Decimal

import numpy as np


def julia_float_str(x: float) -> str:
    """``print(io, x::Float64)`` — shortest round-trip digits in Julia's layout."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Inf" if x > 0 else "-Inf"
    if x == 0.0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    sign = "-" if x < 0 else ""
    d = Decimal(repr(abs(x)))  # shortest round-trip digits (the same digit string as Ryu)
    t = d.as_tuple()
    digits = "".join(map(str, t.digits)).rstrip("0") or "0"
    # value = 0.d1d2… × 10^(e10), with e10 the position of the decimal point
    e10 = len(t.digits) + t.exponent
    if 1e-4 <= abs(x) < 1e6:
        if e10 <= 0:
            s = "0." + "0" * (-e10) + digits
        elif e10 >= len(digits):
            s = digits + "0" * (e10 - len(digits)) + ".0"
        else:
            s = digits[:e10] + "." + digits[e10:]
    else:
        mant = digits[0] + "." + (digits[1:] or "0")
        s = f"{mant}e{e10 - 1}"
    return sign + s


def writedlm(path, A, delim: str = ",") -> None:
    """DelimitedFiles.writedlm(path, A, ',') for a vector (one value per line) or a matrix."""
    A = np.asarray(A, dtype=np.float64)
    if A.ndim == 0:
        A = A.reshape(1, 1)
    if A.ndim == 1:
        A = A[:, None]
    with open(path, "w") as f:
        for row in A:
            f.write(delim.join(julia_float_str(v) for v in row) + "\n")


def readdlm(path, delim: str = ",") -> np.ndarray:
    """DelimitedFiles.readdlm(path, ',') of a numeric CSV → Float64 matrix (NaN/Inf as Julia prints them)."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                rows.append([float(v) for v in line.split(delim)])
    width = max(map(len, rows)) if rows else 0
    return np.array([r + [np.nan] * (width - len(r)) for r in rows], dtype=np.float64).reshape(len(rows), width)


def julia_round(x, digits: int = 3):
    """round.(x; digits) — RoundNearest (ties to even) on x·10^digits, then ÷ 10^digits."""
    x = np.asarray(x, dtype=np.float64)
    step = 10.0 ** digits
    with np.errstate(all="ignore"):
        y = np.rint(x * step) / step
    return np.where(np.isfinite(y), y, x)


def load_data(data_folder: str, thread_id: str):
    """data_management.jl:1-5 → (data N×T, maturities N)."""
    data = readdlm(os.path.join(data_folder, f"thread_id__{thread_id}__data.csv"))
    mats = readdlm(os.path.join(data_folder, f"thread_id__{thread_id}__maturities.csv")).reshape(-1)
    return data, mats


def result_path(model, thread_id: str, what: str) -> str:
    return f"{model.base.results_folder}{model.base.model_string}__thread_id__{thread_id}__{what}"


def save_results(model, results: dict, loss: float, thread_id: str, data_type: str) -> None:
    """io.jl:4-31 (results = predict(...) named tuple as returned by :func:`yfm_amd.predict`)."""
    os.makedirs(model.base.results_folder or ".", exist_ok=True)
    fac = np.vstack([results["factors"], results["states"]])
    writedlm(result_path(model, thread_id, f"factors_filtered_{data_type}.csv"), fac.T)
    writedlm(result_path(model, thread_id, f"fit_filtered_{data_type}.csv"), results["preds"].T)
    writedlm(result_path(model, thread_id, f"factor_loadings_1_filtered_{data_type}.csv"),
             results["factor_loadings_1"].T)
    writedlm(result_path(model, thread_id, f"factor_loadings_2_filtered_{data_type}.csv"),
             results["factor_loadings_2"].T)
    writedlm(result_path(model, thread_id, "loss.csv"), np.array([loss]))
    writedlm(result_path(model, thread_id, "out_params.csv"), model.base.flat_params)
