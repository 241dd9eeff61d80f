"""Write case2431.bin: the 3,000-seed sweep's case 2431 (GNS5, N = 33 → the NP = 48 per-lane kernel, T = 3),
exactly as tests/test_gpu_random.py::random_case draws it (rng = default_rng(1000 + 2431)).

Layout (little-endian): int32 kind, N, T, P, B, space, has_T_use; then N maturities, N×T panel (column-major),
P×B θ (column-major), and B int32 windows when has_T_use.  A data fixture, not code: repro.cpp reads it."""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd"), str(ROOT / "tests")]

from test_gpu_random import random_case  # noqa: E402
from yfm_amd import KIND_GNS  # noqa: E402

rng = np.random.default_rng(1000 + 2431)
N, T, mats, Y, Th, space, T_use = random_case(rng, KIND_GNS)
P, B = Th.shape
with open(HERE / "case2431.bin", "wb") as f:
    np.array([KIND_GNS, N, T, P, B, space, int(T_use is not None)], dtype="<i4").tofile(f)
    np.asarray(mats, dtype="<f8").tofile(f)
    np.asfortranarray(Y, dtype="<f8").T.tofile(f)  # column-major N×T
    np.asfortranarray(Th, dtype="<f8").T.tofile(f)
    if T_use is not None:
        np.asarray(T_use, dtype="<i4").tofile(f)
print(f"case 2431: kind {KIND_GNS} N {N} T {T} P {P} B {B} space {space} windows {T_use is not None}")
