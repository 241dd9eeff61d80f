"""Run two config-2 DNS launches through the library named by YFM_LIB (a YFM_PHASE_PROBE build prints
per-wave cycle counts by phase from the second, timed one; tools/r4_phase.sh)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "yieldfactormodels.jl_amd"), str(ROOT)]
import torch  # noqa: F401,E402
from yfm_amd import KIND_DNS, get_engine  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

eng = get_engine(0)
eng.set_panel(S.simulate_panel(KIND_DNS, 600), S.maturities_30())
Th = S.theta_batch(KIND_DNS, 65536)
eng.loglik(KIND_DNS, Th)
print("=== timed launch", flush=True)
eng.loglik(KIND_DNS, Th)
