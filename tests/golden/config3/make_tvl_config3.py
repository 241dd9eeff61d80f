"""Generate tests/golden/config3/tvl_config3_sample.npz: config 3's workload (TVλ EKF, N = 360 maturities,
T = 600) on the first 64 candidates of the bench batch (bench.py make_workload(3): seed
BATCH_SEED, scale 0.02), with
  * loglik_oracle — the C restatement of the reference's dense path (oracle/yfm_oracle.c:
    F = ZPZ' + σ²I, getrf + getri, logdet LU, every step), and
  * loglik_truth  — the binary128 evaluation of the same recursion (oracle/yfm_truth.c).
The panel is not stored: it is regenerated from its seed (yfm_amd.synthetic.simulate_panel).

    python tests/golden/config3/make_tvl_config3.py      (≈ 1-2 min on 8 cores)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[3]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]

from oracle.truth import loglik_oracle, loglik_truth  # noqa: E402
from yfm_amd import KIND_TVL  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402


def main():
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    Th = np.asfortranarray(S.theta_batch(KIND_TVL, 16384, seed=S.BATCH_SEED, bad_frac=0.0, scale=0.02)[:, :64])
    ora = loglik_oracle(KIND_TVL, Y, mats, Th)
    tru = loglik_truth(KIND_TVL, Y, mats, Th)
    np.savez_compressed(Path(__file__).parent / "tvl_config3_sample.npz", Theta=Th, loglik_oracle=ora,
                        loglik_truth=tru, panel_seed=S.PANEL_SEED, batch_seed=S.BATCH_SEED)
    e = np.abs(ora - tru) / np.abs(tru)
    print(f"oracle vs truth: max {e.max():.3e}, within 1e-9: {(e <= 1e-9).mean():.3f}")


if __name__ == "__main__":
    main()
