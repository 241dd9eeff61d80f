"""Accuracy of the certified TVλ filter of the library YFM_LIB points at (default: the in-tree build) on the
1,024-candidate config-3 fixture (tests/golden/config3/tvl_config3_1024.npz): error distribution against the
binary128 truth, and the factor-1 parity table.  One JSON line.  (A/B helper: tools/archive/r3_tvl_ab.sh.)"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd"), str(ROOT / "tests")]

from yfm_amd import KIND_TVL  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402
from yfm_amd.engine import get_engine  # noqa: E402
from test_gpu_parity import parity_table  # noqa: E402


def main():
    eng = get_engine()
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    with np.load(ROOT / "tests/golden/config3/tvl_config3_1024.npz", allow_pickle=False) as z:
        fx = {k: z[k] for k in z.files}
    eng.set_panel(Y, mats)
    got = eng.loglik(KIND_TVL, fx["Theta"])
    tru = fx["loglik_truth"]
    fin = np.isfinite(tru)
    e = np.abs(got[fin] - tru[fin]) / np.abs(tru[fin])
    out = {"lib": os.environ.get("YFM_LIB", "in-tree"), "n": int(fin.sum()), "max": float(e.max()),
           "n_gt_1e-13": int((e > 1e-13).sum()), "n_gt_1e-12": int((e > 1e-12).sum()),
           "n_gt_1e-9": int((e > 1e-9).sum()), "median": float(np.median(e)),
           "parity": parity_table(got, fx["loglik_oracle"], tru),
           "pattern_ok": bool(np.array_equal(np.isfinite(got), np.isfinite(tru)))}
    eng.precision = 1  # YFM_PREC_FP64
    fp = eng.loglik(KIND_TVL, fx["Theta"])
    ef = np.abs(fp[fin] - tru[fin]) / np.abs(tru[fin])
    out["fp64"] = {"max": float(ef.max()), "p99": float(np.quantile(ef, 0.99)), "median": float(np.median(ef))}
    if len(sys.argv) > 1:
        np.savez(sys.argv[1], cert=got, fp64=fp)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
