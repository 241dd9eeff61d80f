"""Sweep the TVλ EKF kernel (config 3: N = 360, T = 600) over batch sizes and group widths.

    python tools/bench_tvl.py [--T 600] [--batches 1,1024,16384] [--lanes auto,8,16,64]

Prints one JSON line per (B, L): evals/s from HIP events around `reps` launches.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))

from yfm_amd import KIND_TVL, Engine, n_params  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=600)
    ap.add_argument("--batches", default="1,1024,16384")
    ap.add_argument("--lanes", default="auto,4,8,16,32,64")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    mats = S.maturities_360()
    Y = S.simulate_panel(KIND_TVL, args.T, maturities=mats)
    eng = Engine(0)
    eng.set_panel(Y, mats)
    P = n_params(KIND_TVL)
    stream = torch.cuda.current_stream()
    for B in [int(x) for x in args.batches.split(",")]:
        Th = S.theta_batch(KIND_TVL, B, seed=41, bad_frac=0.0, scale=0.02)
        d_th = torch.from_numpy(np.ascontiguousarray(Th.T)).cuda()
        d_out = torch.empty(B, dtype=torch.float64, device="cuda")
        ref = None
        for L in args.lanes.split(","):
            if L == "auto":
                os.environ.pop("YFM_TVL_LANES", None)
            else:
                os.environ["YFM_TVL_LANES"] = L
            run = lambda: eng.loglik_device(KIND_TVL, d_th.data_ptr(), P, B, d_out.data_ptr(),
                                            stream=stream.cuda_stream)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                run()
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            out = d_out.cpu().numpy()
            if ref is None:
                ref = out
            fin = np.isfinite(ref)
            dev = float(np.max(np.abs(out[fin] - ref[fin]) / np.abs(ref[fin]))) if fin.any() else 0.0
            print(json.dumps({"B": B, "L": L, "ms": ms, "evals_per_s": B / (ms * 1e-3), "T": args.T,
                              "max_rel_vs_first": dev}), flush=True)
    os.environ.pop("YFM_TVL_LANES", None)


if __name__ == "__main__":
    main()
