"""Probe for selective certification of the TVλ filter (config 3): per candidate of the bench batch,
the certified (double-double) loglik and FP64 logliks at several group widths (different summation
orders, so different roundings) and over truncated windows.  Output: an npz for offline analysis of
how well FP64 disagreement predicts FP64 error.

    python tools/tvl_detect_probe.py gpurun_out/detect/probe.npz
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]

from yfm_amd import KIND_TVL, _lib  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402
from yfm_amd.engine import get_engine  # noqa: E402


def main(out):
    eng = get_engine()
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    Th = np.asfortranarray(S.theta_batch(KIND_TVL, 16384, seed=S.BATCH_SEED, bad_frac=0.0, scale=0.02))
    eng.set_panel(Y, mats)
    res = {}
    res["cert"] = eng.loglik(KIND_TVL, Th)
    print("cert done", flush=True)
    eng.precision = _lib.PREC_FP64
    for L in (4, 8, 16):
        os.environ["YFM_TVL_LANES"] = str(L)
        res[f"fp64_L{L}"] = eng.loglik(KIND_TVL, Th)
        for tu in (100, 200, 300, 400):
            res[f"fp64_L{L}_T{tu}"] = eng.loglik(KIND_TVL, Th, T_use=np.full(Th.shape[1], tu, np.int32))
        print("fp64", L, flush=True)
    os.environ.pop("YFM_TVL_LANES", None)
    eng.precision = _lib.PREC_CERTIFIED
    for tu in (100, 200, 300, 400):
        res[f"cert_T{tu}"] = eng.loglik(KIND_TVL, Th, T_use=np.full(Th.shape[1], tu, np.int32))
    print("cert windows done", flush=True)
    Path(out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(out, Theta=Th, **res)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/detect/probe.npz")
