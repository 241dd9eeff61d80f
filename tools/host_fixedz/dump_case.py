"""Write tests/test_gpu_random.py's random_case(seed) as the binary input of tools/host_fixedz/harness.cpp.

    python tools/host_fixedz/dump_case.py <seed> <kind> <out.bin>
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "yieldfactormodels.jl_amd"), ROOT]
from test_gpu_random import random_case  # noqa: E402

seed, kind, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
rng = np.random.default_rng(1000 + seed)
N, T, mats, Y, Th, space, T_use = random_case(rng, kind)
P, B = Th.shape
with open(out, "wb") as f:
    np.array([N, T, B, P, space, T_use is not None, kind], dtype=np.int32).tofile(f)
    np.ascontiguousarray(mats, dtype=np.float64).tofile(f)
    np.asfortranarray(Y).ravel(order="F").tofile(f)
    np.asfortranarray(Th).ravel(order="F").tofile(f)
    if T_use is not None:
        np.ascontiguousarray(T_use, dtype=np.int32).tofile(f)
print(f"seed {seed}: N {N} T {T} B {B} P {P} space {space} windows {T_use is not None}")
