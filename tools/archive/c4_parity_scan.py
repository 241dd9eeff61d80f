"""Factor-1 parity over the whole config-4 job where it is hardest: every (θ, window) whose loglik is small
against the terms it sums (|ll| < --llmax), plus a random sample of the rest, against the dense FP64 oracle
and the binary128 truth.  A loglik near 0 is a sum of ~10^4-sized terms that cancels, so its relative error
is the absolute error of those terms over |ll|.

    python tools/c4_parity_scan.py [--llmax 20] [--sample 512] [--steady 0|1]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]
import torch  # noqa: E402,F401
from oracle.truth import loglik_oracle, loglik_truth  # noqa: E402
from yfm_amd import KIND_DNS, get_engine  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--llmax", type=float, default=20.0)
ap.add_argument("--sample", type=int, default=512)
ap.add_argument("--steady", type=int, default=1)
a = ap.parse_args()
if not a.steady:
    os.environ["YFM_DNS_STEADY"] = "0"
eng = get_engine(0)
T, per = 600, 4096
wins = np.arange(361, 601)
Th_all = S.theta_batch(KIND_DNS, per, seed=S.BATCH_SEED)
Th = np.asfortranarray(np.tile(Th_all, (1, len(wins))))
tu = np.repeat(wins, per).astype(np.int32)
mats = S.maturities_30()
Y = S.simulate_panel(KIND_DNS, T)
eng.set_panel(Y, mats)
got = eng.loglik(KIND_DNS, Th, space=0, T_use=tu)
fin = np.isfinite(got)
small = np.flatnonzero(fin & (np.abs(got) < a.llmax))
rest = np.setdiff1d(np.flatnonzero(fin), small)
samp = np.random.default_rng(0).choice(rest, size=min(a.sample, rest.size), replace=False)
sel = np.concatenate([small, samp])
sub = np.asfortranarray(Th[:, sel])
orc = loglik_oracle(KIND_DNS, Y, mats, sub, T_use=tu[sel], nthreads=16)
tru = loglik_truth(KIND_DNS, Y, mats, sub, T_use=tu[sel], nthreads=16)
g = got[sel]
eg = np.abs(g - tru) / np.abs(tru)
eo = np.abs(orc - tru) / np.abs(tru)
ego = np.abs(g - orc) / np.abs(orc)
ok = (ego <= 1e-9) | (eg <= eo)
absg = np.abs(g - tru)
out = {"evaluations": int(fin.sum()), "small_ll_candidates": int(small.size), "llmax": a.llmax,
       "sample_rest": int(samp.size), "steady": a.steady,
       "failing_factor1": int((~ok).sum()),
       "failing_small": int((~ok[:small.size]).sum()), "failing_rest": int((~ok[small.size:]).sum()),
       "gpu_truth_abs_max_small": float(absg[:small.size].max()) if small.size else 0.0,
       "gpu_truth_abs_max_rest": float(absg[small.size:].max()) if samp.size else 0.0,
       "oracle_truth_abs_max_small": float(np.abs(orc - tru)[:small.size].max()) if small.size else 0.0,
       "worst": []}
for k in np.argsort(-(eg - eo))[:10]:
    out["worst"].append({"theta": int(sel[k] % per), "window": int(tu[sel[k]]), "ll": float(tru[k]), "gpu_rel": float(eg[k]),
                         "oracle_rel": float(eo[k]), "gpu_abs": float(absg[k]), "ok": bool(ok[k])})
print(json.dumps(out, indent=1))
