"""Rolling re-estimation throughput — the reference's own printed number ("average seconds per
task", forecasting.jl:144-189): every forecast origin of config 4 (expanding windows
T_w = 361..600 of the T = 600, N = 30 DNS panel) re-estimated with estimate_steps!'s defaults
(NelderMead opt1: 500 iterations, g_tol 1e-6; max_group_iters 10, tol 1e-8), all windows as ONE
batched yfm_estimate call, next to ONE window's chain on the faithful CPU path (oracle/optim_nm.py
driving the dense C restatement oracle/yfm_oracle.c, single thread — what one reference process
does per task).

    python tools/bench_estimate.py [--windows 240] [--cpu-window 480]
    python tools/bench_estimate.py --model tvl [--N 30] [--windows 240]

`--model tvl`: the same job for the TVλ EKF (certified double-double kernel, the library default), the
rolling re-estimation of forecasting.jl:140-176 with every window started from θ₀ (the reference seeds TVλ
from the fitted DNS parameters, paramoperations.jl:78-89 — a start, not a different computation).  A TVλ
chain on the faithful CPU path takes hours, so the CPU leg times the dense port's per-evaluation cost at
the CPU window (single thread) and reports per task = that × the GPU job's evaluations per chain.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))
sys.path.insert(0, str(ROOT))

from oracle import optim_nm as NM  # noqa: E402  (CPU reference leg only)
from yfm_amd import KIND_DNS, KIND_TVL, Engine, n_params  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402
from yfm_amd.params import transform_params, untransform_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=240)
    ap.add_argument("--cpu-window", type=int, default=480)
    ap.add_argument("--model", choices=["dns", "tvl"], default="dns")
    ap.add_argument("--N", type=int, default=30, help="maturities (TVλ: 30 = the config-4 grid, 360 = config 3)")
    ap.add_argument("--iterations", type=int, default=500)
    ap.add_argument("--max-group-iters", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    kind = KIND_TVL if args.model == "tvl" else KIND_DNS
    mats = S.maturities_30() if args.N == 30 else S.maturities_360()
    Y = S.simulate_panel(kind, 600, maturities=mats)
    th0 = S.theta0_constrained(kind)
    P = n_params(kind)
    wins = np.arange(601 - args.windows, 601, dtype=np.int32)
    eng = Engine(0)
    eng.set_panel(Y, mats)
    Th0 = np.repeat(th0[:, None], len(wins), axis=1)
    eng.estimate(kind, Th0[:, :2], space=1, T_use=wins[:2], iterations=5, max_group_iters=1)  # warm up
    t0 = time.perf_counter()
    r = eng.estimate(kind, Th0, space=1, T_use=wins, iterations=args.iterations, max_group_iters=args.max_group_iters)
    gpu_s = time.perf_counter() - t0
    name = "TVλ EKF (certified)" if kind == KIND_TVL else "DNS"
    out = {"metric": f"rolling re-estimation (estimate_steps!, NelderMead opt1), {name} T≤600 N={len(mats)}",
           "windows": int(len(wins)), "iterations": args.iterations, "max_group_iters": args.max_group_iters,
           "gpu_seconds_all_windows": gpu_s, "gpu_seconds_per_task": gpu_s / len(wins),
           "gpu_objective_evals": int(r["n_evals"]), "status_counts": np.bincount(r["status"], minlength=3).tolist(),
           "ll_median": float(np.median(r["ll"]))}
    if not args.no_cpu:
        lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
        D = ctypes.POINTER(ctypes.c_double)
        Tw = int(args.cpu_window)
        Yw = np.asfortranarray(Y[:, :Tw])
        calls = [0]

        def f(theta):
            calls[0] += 1
            th = np.ascontiguousarray(theta, dtype=np.float64)
            o = np.empty(1)
            lib.yfm_oracle_loglik(kind, 0, Yw.ctypes.data_as(D), len(mats), Tw, mats.ctypes.data_as(D),
                                  th.ctypes.data_as(D), P, 1, None, o.ctypes.data_as(D), 1)
            if math.isnan(o[0]):
                raise NM.InitThrow()
            return -o[0]

        if kind == KIND_TVL:
            # per-evaluation cost of the dense port (one thread), times the evaluations one chain made here
            x = untransform_params(kind, th0)
            f(x)
            n, t0 = 0, time.perf_counter()
            while n < 3 or time.perf_counter() - t0 < 5.0:
                f(x)
                n += 1
            per_eval = (time.perf_counter() - t0) / n
            per_task = per_eval * r["n_evals"] / len(wins)
            out.update({"cpu_window": Tw, "cpu_seconds_per_eval": per_eval, "cpu_evals_timed": n, "cpu_threads": 1,
                        "cpu_kind": "port (oracle/yfm_oracle.c, dense N×N inverse per step)",
                        "cpu_seconds_one_task_est": per_task,
                        "cpu_estimate": "per-eval time at the CPU window × the GPU job's evaluations per chain",
                        "speedup_per_task": per_task / (gpu_s / len(wins)),
                        "cpu_16_processes_seconds_all_windows_est": per_task * len(wins) / 16,
                        "speedup_vs_16_processes": per_task * len(wins) / 16 / gpu_s})
        else:
            t0 = time.perf_counter()
            ref = NM.estimate_steps(f, th0, transform=lambda x: transform_params(kind, x),
                                    untransform=lambda x: untransform_params(kind, x))
            cpu_s = time.perf_counter() - t0
            k = int(np.flatnonzero(wins == Tw)[0])
            out.update({"cpu_window": Tw, "cpu_seconds_one_task": cpu_s, "cpu_objective_evals": calls[0],
                        "cpu_threads": 1, "cpu_kind": "port (oracle/optim_nm.py + oracle/yfm_oracle.c)",
                        "gpu_vs_cpu_ll_rel": abs(r["ll"][k] - ref.ll) / abs(ref.ll),
                        "speedup_per_task": cpu_s / (gpu_s / len(wins)),
                        # like for like: the reference runs one task per process, so 16 host cores take
                        # ≈ windows/16 of these tasks each (one mid-size window stands for the average)
                        "cpu_16_processes_seconds_all_windows_est": cpu_s * len(wins) / 16,
                        "speedup_vs_16_processes": cpu_s * len(wins) / 16 / gpu_s})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
