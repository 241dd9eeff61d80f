"""Benchmark: batched DNS Kalman log-likelihood evals/s on MI355X (BASELINE.json config 2).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One "step" = one batched loglik over B = 65,536 parameter vectors per GPU
(T = 600 months × N = 30 maturities, FP64), inputs resident in HBM; for N > 1
the step also all-gathers the per-candidate logliks over RCCL and reduces the
best candidate (weak scaling: every rank evaluates its own 65,536 θ).

Prints ONE JSON line on rank 0 (contract in the task statement) with a
`roofline` object (FP64 VALU bound, SURVEY §8d algorithmic flops) and a
`cpu_baseline` object (the faithful dense-LU C restatement, oracle/yfm_oracle.c,
on a bounded sample of the same workload, OpenMP over the host cores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))
sys.path.insert(0, str(ROOT))

from yfm_amd import KIND_DNS, Engine, n_params, state_dim  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, AMD spec (the local guide lists no FP64 figure)


def alg_flops(kind: int, N: int, M: int, T: int) -> float:
    """SURVEY.md §8(d) algorithmic FP64 flops per loglik eval (capacitance/Woodbury form):
    (T-1)·F_step + 2NM² (G = Z'Z) + 2(M²)³ (Lyapunov), F_step = 4NM + 3N + 12⅔M³ + 6M² + 6M + 8."""
    f_step = 4 * N * M + 3 * N + (38.0 / 3.0) * M ** 3 + 6 * M * M + 6 * M + 8
    return (T - 1) * f_step + 2 * N * M * M + 2 * (M * M) ** 3


def cpu_baseline(Y, mats, Th, seconds: float, gpu_out):
    """Faithful reference-path restatement on the host: time a bounded sample of the same workload."""
    lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
    D = ctypes.POINTER(ctypes.c_double)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    Yf = np.asfortranarray(Y)
    N, T = Yf.shape
    P = Th.shape[0]
    done, t0 = 0, time.perf_counter()
    chunk = 2 * threads
    res = []
    while time.perf_counter() - t0 < seconds and done + chunk <= Th.shape[1]:
        sub = np.asfortranarray(Th[:, done:done + chunk])
        out = np.empty(chunk)
        lib.yfm_oracle_loglik(KIND_DNS, 0, Yf.ctypes.data_as(D), N, T, mats.ctypes.data_as(D), sub.ctypes.data_as(D),
                              P, chunk, None, out.ctypes.data_as(D), threads)
        res.append(out)
        done += chunk
    dt = time.perf_counter() - t0
    ref = np.concatenate(res)
    got = gpu_out[:done]
    fin = np.isfinite(ref)
    same_pattern = bool(np.array_equal(np.isfinite(got), fin) and np.array_equal(np.isnan(got), np.isnan(ref)))
    err = np.abs(got[fin] - ref[fin]) / np.abs(ref[fin])
    # adjudicate with the extended-precision truth proxy on the first 512 of the sample
    from oracle.kalman_ld import loglik_ld
    k = min(512, done)
    tru = loglik_ld(KIND_DNS, mats, Y, Th[:, :k])
    ft = np.isfinite(tru)
    e_gpu = np.abs(got[:k][ft] - tru[ft]) / np.abs(tru[ft])
    e_ref = np.abs(ref[:k][ft] - tru[ft]) / np.abs(tru[ft])
    return {"value": done / dt, "unit": "evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} of the benchmark's θ (T={T}, N={N}) in {dt:.1f} s, dense N×N getrf+getri + logdet LU "
                      f"per step (oracle/yfm_oracle.c, -O3, OpenMP {threads} threads)",
            "parity": {"pattern_match": same_pattern, "gpu_vs_oracle_max_rel": float(err.max()) if err.size else 0.0,
                       "frac_within_1e-9": float((err <= 1e-9).mean()) if err.size else 1.0,
                       "truth_subset": k, "gpu_vs_truth_max_rel": float(e_gpu.max()) if e_gpu.size else 0.0,
                       "oracle_vs_truth_max_rel": float(e_ref.max()) if e_ref.size else 0.0}}


def pmc_traffic(kernel_substr: str = "fixedz_loglik_kernel<32, 3, 1, false>"):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc passes
    (tools/profile_pmc.sh → profiles/<round>/pmc_summary.json): (FETCH_SIZE + WRITE_SIZE) KB × 1024, raw
    (gfx950 FETCH_SIZE can under-count narrow reads by up to 2×, MI355X_MICROARCH.md §HBM)."""
    for rnd in sorted((ROOT / "profiles").glob("r*/pmc_summary.json"), reverse=True):
        d = json.loads(rnd.read_text())
        for k, v in d.items():
            if kernel_substr in k and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                return (v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0, str(rnd.relative_to(ROOT))
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="θ per GPU")
    ap.add_argument("--T", type=int, default=600)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    kind, N, T, B = KIND_DNS, 30, args.T, args.batch
    M, P = state_dim(kind), n_params(kind)
    mats = S.maturities_30()
    Y = S.simulate_panel(kind, T)
    Th = S.theta_batch(kind, B, seed=S.BATCH_SEED + rank)  # weak scaling: each rank its own 65,536 θ
    eng = Engine(dev.index)
    eng.set_panel(Y, mats)
    d_th = torch.from_numpy(np.ascontiguousarray(Th.T)).to(dev)  # (B, P) C-order == P×B column-major
    d_out = torch.empty(B, dtype=torch.float64, device=dev)
    gathered = torch.empty(world * B, dtype=torch.float64, device=dev) if world > 1 else None
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.loglik_device(kind, d_th.data_ptr(), P, B, d_out.data_ptr(), space=0, stream=stream.cuda_stream)
        if world > 1:  # RCCL over xGMI: gather logliks, reduce the best candidate
            dist.all_gather_into_tensor(gathered, d_out)
            torch.argmax(torch.nan_to_num(gathered, nan=-np.inf))

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    ms_per_step = 1e3 * wall / args.steps
    value = world * B / (wall / args.steps)
    f_eval = alg_flops(kind, N, M, T)
    achieved = f_eval * B / (ev_ms * 1e-3) / 1e12  # TFLOP/s of the dominant kernel (per GPU)
    traffic, traffic_src = pmc_traffic()
    out_host = d_out.cpu().numpy()
    n_neginf, n_nan = int(np.isneginf(out_host).sum()), int(np.isnan(out_host).sum())

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(Y, mats, Th, args.cpu_seconds, out_host)

    if rank == 0:
        line = {
            "metric": "Kalman loglik evals/sec (DNS, T=600, N=30)",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (DNS-simulated panel, seeded θ batch with 1% non-stationary Φ)",
            "config": {"workload": "config2: DNS loglik over 65,536 θ per GPU", "kind": "DNS (1C)", "T": T,
                       "N": N, "batch_per_gpu": B, "global_batch": world * B,
                       "parallelism": f"dp{world} (θ sharded, RCCL all-gather of logliks + argmax)"},
            "roofline": {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes": B * (P + 1) * 8 + T * (32 + 4) * 8,
                         "kernel_ms": ev_ms, "flops_per_eval": f_eval,
                         "note": "achieved = SURVEY §8d algorithmic flops × B ÷ HIP-event time per step"},
            "cpu_baseline": cpu,
            "outputs": {"neg_inf": n_neginf, "nan": n_nan},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
