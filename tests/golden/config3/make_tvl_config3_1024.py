"""Generate tests/golden/config3/tvl_config3_1024.npz: config 3's workload (TVλ EKF, N = 360, T = 600) on
the first 1,024 candidates of the bench batch (bench.py make_workload(3): seed BATCH_SEED, scale 0.02),
with the dense C oracle (oracle/yfm_oracle.c, the reference's algorithm in FP64) and the binary128
truth (oracle/yfm_truth.c).  A larger sample than tvl_config3_sample.npz for two questions: how far
the reference's own FP64 path is from exact arithmetic on this workload, and whether the certified
kernel reproduces the truth on every candidate.

    python tests/golden/config3/make_tvl_config3_1024.py      (≈ 30 min on 8 cores: the dense oracle)
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

N_SAMPLE = 1024


def main():
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, 600, maturities=mats)
    Th = np.asfortranarray(S.theta_batch(KIND_TVL, 16384, seed=S.BATCH_SEED, bad_frac=0.0, scale=0.02)[:, :N_SAMPLE])
    tru = loglik_truth(KIND_TVL, Y, mats, Th)
    ora = loglik_oracle(KIND_TVL, Y, mats, Th)
    np.savez_compressed(Path(__file__).parent / "tvl_config3_1024.npz", Theta=Th, loglik_oracle=ora,
                        loglik_truth=tru, panel_seed=S.PANEL_SEED, batch_seed=S.BATCH_SEED)
    fin = np.isfinite(tru)
    e = np.abs(ora[fin] - tru[fin]) / np.abs(tru[fin])
    print(f"oracle vs truth: max {e.max():.3e}, p99 {np.quantile(e, 0.99):.3e}, within 1e-9: {(e <= 1e-9).mean():.3f}")


if __name__ == "__main__":
    main()
