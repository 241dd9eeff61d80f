"""Dump DNS logliks of the library named by YFM_LIB (config-2 batch; a ragged/NaN case) to an .npz, so two
builds that should give the same bits can be compared in a second process (A/B of layout-only changes)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "yieldfactormodels.jl_amd"), str(ROOT)]
import torch  # noqa: F401,E402
from yfm_amd import KIND_DNS, get_engine  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

eng = get_engine(0)
out = {}
mats = S.maturities_30()
Y = S.simulate_panel(KIND_DNS, 600)
eng.set_panel(Y, mats)
Th = S.theta_batch(KIND_DNS, 65536)
out["c2"] = eng.loglik(KIND_DNS, Th)
Y2 = Y.copy(order="F")
Y2[:, [50, 51, 300]] = np.nan
eng.set_panel(Y2, mats)
sub = np.asfortranarray(Th[:, :4096 + 23])
tu = np.full(sub.shape[1], 600, dtype=np.int32)
tu[::37] = np.arange(tu[::37].size) % 590 + 5
out["ragged"] = eng.loglik(KIND_DNS, sub, T_use=tu)
np.savez(sys.argv[1], **out)
print("dumped", sys.argv[1], {k: int(np.isfinite(v).sum()) for k, v in out.items()})
