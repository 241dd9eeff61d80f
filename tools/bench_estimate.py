"""Rolling re-estimation throughput — the reference's own printed number ("average seconds per
task", forecasting.jl:144-189): every forecast origin of config 4 (expanding windows
T_w = 361..600 of the T = 600, N = 30 DNS panel) re-estimated with estimate_steps!'s defaults
(NelderMead opt1: 500 iterations, g_tol 1e-6; max_group_iters 10, tol 1e-8), all windows as ONE
batched yfm_estimate call, next to ONE window's chain on the faithful CPU path (oracle/optim_nm.py
driving the dense C restatement oracle/yfm_oracle.c, single thread — what one reference process
does per task).

    python tools/bench_estimate.py [--windows 240] [--cpu-window 480]
    python tools/bench_estimate.py --model tvl [--N 30] [--windows 240]

Optimised CPU leg (default; `--no-cpu-opt` skips it): the same estimate_steps! chains on the host cores, each
chain one process running oracle/optim_nm.py over the optimised C filter (oracle/yfm_cpu_fast.c: the collapsed /
capacitance form the GPU runs, one evaluation per call, one thread), `threads` processes at once (the box's CPU
share, bench.cpu_topology) — the reference's own layout of one task per process, on this build's algorithm.  DNS
runs all windows; TVλ (≈ 40 s per chain on one core) a sample of one window per process, scaled to all windows.
Reported beside it: the evaluation-only bound (the chains' consumed evaluations ÷ the filter's single-evaluation
rate × threads: no optimiser cost at all) and a labelled linear extrapolation to 128 cores.  It runs before the
GPU is touched (the worker processes are spawned from a process that has not initialised the GPU).

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


def _native_fast_lib() -> tuple[str, str]:
    """The optimised C filter built with -march=native for this host (as bench.py's cpu_baseline does), or the
    in-tree x86-64-v3 build if that fails: (path, flags)."""
    import subprocess
    import tempfile
    out = Path(tempfile.mkdtemp(prefix="yfm_cpu_"))
    try:
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s", "native", f"OUT={out}"], check=True,
                       capture_output=True, timeout=120)
        return str(out / "libyfm_cpu_fast_native.so"), "-O3 -march=native"
    except Exception:  # noqa: BLE001
        return str(ROOT / "oracle" / "libyfm_cpu_fast.so"), "-O3 -march=x86-64-v3 (native build failed)"


def _fast_objective(kind, Yw, mats, P, lib_path):
    """-loglik of one θ (unconstrained) on the optimised C filter, one thread; NaN → InitThrow as compute_loss."""
    lib = ctypes.CDLL(lib_path)
    D = ctypes.POINTER(ctypes.c_double)
    Yf = np.asfortranarray(Yw)
    N, Tw = Yf.shape
    calls = [0]

    def f(theta):
        calls[0] += 1
        th = np.ascontiguousarray(theta, dtype=np.float64)
        o = np.empty(1)
        lib.yfm_cpu_fast_loglik(kind, 0, Yf.ctypes.data_as(D), N, Tw, mats.ctypes.data_as(D), th.ctypes.data_as(D), P,
                                1, None, o.ctypes.data_as(D), 1)
        if math.isnan(o[0]):
            raise NM.InitThrow()
        return -o[0]
    return f, calls


def _cpu_chain(job):
    """One window's estimate_steps! chain on the optimised CPU filter (a pool worker): (seconds, evaluations, ll)."""
    kind, Y, mats, Tw, th0, iterations, max_group_iters, lib_path = job
    P = len(th0)
    f, calls = _fast_objective(kind, np.asarray(Y)[:, :Tw], mats, P, lib_path)
    t0 = time.perf_counter()
    ref = NM.estimate_steps(f, th0, transform=lambda x: transform_params(kind, x),
                            untransform=lambda x: untransform_params(kind, x), iterations=iterations,
                            max_group_iters=max_group_iters)
    return time.perf_counter() - t0, calls[0], float(ref.ll)


def cpu_optimised_leg(kind, Y, mats, wins, th0, args) -> dict:
    """The chains of `wins` (all, or a sample for TVλ) on `threads` worker processes; see the module docstring."""
    import multiprocessing as mp
    import os
    from bench import cpu_topology
    topo = cpu_topology()
    threads = topo["threads_used"]
    P = len(th0)
    lib_path, flags = _native_fast_lib()
    # single-evaluation rate of the optimised filter at a mid-size window, one thread: one θ per call (what a chain
    # asks for) and a batch of 64 per call (the filter's vector width filled: the evaluation-only bound)
    Tm = int(wins[len(wins) // 2])
    f, _ = _fast_objective(kind, Y[:, :Tm], mats, P, lib_path)
    x = untransform_params(kind, th0)
    f(x)
    n, t0 = 0, time.perf_counter()
    while n < 20 or time.perf_counter() - t0 < 2.0:
        f(x)
        n += 1
    per_eval = (time.perf_counter() - t0) / n
    lib = ctypes.CDLL(lib_path)
    Dp = ctypes.POINTER(ctypes.c_double)
    Yf = np.asfortranarray(Y[:, :Tm])
    Xb = np.asfortranarray(np.repeat(x[:, None], 64, axis=1))
    ob = np.empty(64)
    n, t0 = 0, time.perf_counter()
    while n < 3 or time.perf_counter() - t0 < 2.0:
        lib.yfm_cpu_fast_loglik(kind, 0, Yf.ctypes.data_as(Dp), Yf.shape[0], Tm, mats.ctypes.data_as(Dp),
                                Xb.ctypes.data_as(Dp), P, 64, None, ob.ctypes.data_as(Dp), 1)
        n += 1
    per_eval_batched = (time.perf_counter() - t0) / (64 * n)
    sample = wins if kind == KIND_DNS else wins[np.linspace(0, len(wins) - 1, threads).round().astype(int)]
    order = sorted(sample.tolist(), reverse=True)  # longest windows first: the pool's tail is short ones
    jobs = [(kind, Y, mats, int(Tw), th0, args.iterations, args.max_group_iters, lib_path) for Tw in order]
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(threads) as pool:
        res = pool.map(_cpu_chain, jobs, chunksize=1)
    wall = time.perf_counter() - t0
    secs = np.array([r[0] for r in res])
    evals = np.array([r[1] for r in res])
    scale = len(wins) / len(sample)
    wall_all = wall * scale
    return {"cpu_optimised_seconds_all_windows": wall_all,
            "cpu_optimised_measured": {"windows_run": int(len(sample)), "processes": threads, "wall_seconds": wall,
                                       "scaled_to_all_windows": scale != 1.0,
                                       "chain_seconds_mean": float(secs.mean()), "chain_evals_mean": float(evals.mean()),
                                       "host_cpu": topo["host_cpu"], "topology": topo},
            "cpu_optimised_seconds_per_eval_1_thread": per_eval,
            "cpu_optimised_seconds_per_eval_1_thread_batch64": per_eval_batched,
            "cpu_optimised_eval_window": Tm, "cpu_optimised_build": flags,
            "cpu_optimised_eval_only_bound_seconds": float(evals.mean()) * len(wins) * per_eval_batched / threads,
            "cpu_optimised_extrapolated_128_cores_seconds": wall_all * threads / 128.0,
            "cpu_optimised_kind": "NOT the reference algorithm: oracle/optim_nm.py (Optim NelderMead restated in "
                                  "Python) over oracle/yfm_cpu_fast.c (the GPU's collapsed / capacitance form in C, "
                                  "-O3, one evaluation per call), one chain per process",
            "cpu_optimised_note": "eval_only_bound = the chains' evaluations × the per-evaluation time of a FULL "
                                  "64-candidate batch ÷ processes (no optimiser cost, every vector lane busy — "
                                  "a chain asks for one point at a time); extrapolated_128_cores = the measured wall × threads / 128 "
                                  "(linear scaling assumed, an upper bound on the CPU's speed)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=240)
    ap.add_argument("--cpu-window", type=int, default=480)
    ap.add_argument("--model", choices=["dns", "tvl"], default="dns")
    ap.add_argument("--N", type=int, default=30, help="maturities (TVλ: 30 = the config-4 grid, 360 = config 3)")
    ap.add_argument("--iterations", type=int, default=500)
    ap.add_argument("--max-group-iters", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-cpu-opt", action="store_true")
    ap.add_argument("--precision", choices=["certified", "fp64"], default="certified",
                    help="TVλ arithmetic of the GPU leg (the library default is certified; fp64 is the reference's class)")
    args = ap.parse_args()
    kind = KIND_TVL if args.model == "tvl" else KIND_DNS
    mats = S.maturities_30() if args.N == 30 else S.maturities_360()
    Y = S.simulate_panel(kind, 600, maturities=mats)
    th0 = S.theta0_constrained(kind)
    P = n_params(kind)
    wins = np.arange(601 - args.windows, 601, dtype=np.int32)
    # the optimised CPU leg first: its worker processes start before this process touches the GPU
    cpu_opt = None if args.no_cpu_opt else cpu_optimised_leg(kind, Y, mats, wins, th0, args)
    torch.cuda.set_device(0)
    eng = Engine(0)
    from yfm_amd import _lib
    eng.precision = _lib.PREC_FP64 if args.precision == "fp64" else _lib.PREC_CERTIFIED
    eng.set_panel(Y, mats)
    Th0 = np.repeat(th0[:, None], len(wins), axis=1)
    eng.estimate(kind, Th0[:, :2], space=1, T_use=wins[:2], iterations=5, max_group_iters=1)  # warm up
    t0 = time.perf_counter()
    r = eng.estimate(kind, Th0, space=1, T_use=wins, iterations=args.iterations, max_group_iters=args.max_group_iters)
    gpu_s = time.perf_counter() - t0
    name = f"TVλ EKF ({args.precision})" if kind == KIND_TVL else "DNS"
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
    if cpu_opt:
        out.update(cpu_opt)
        out["gpu_over_cpu_optimised"] = cpu_opt["cpu_optimised_seconds_all_windows"] / gpu_s
        out["gpu_over_cpu_optimised_128_cores"] = cpu_opt["cpu_optimised_extrapolated_128_cores_seconds"] / gpu_s
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
