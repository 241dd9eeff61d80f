"""Benchmark: batched Kalman log-likelihood evals/s on MI355X (BASELINE.json configs 2-5).

    python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Default (`--config 2`, the metric's headline workload): one "step" = one batched DNS
loglik over B = 65,536 parameter vectors per GPU (T = 600 months × N = 30 maturities,
FP64), inputs resident in HBM; for N > 1 the step also all-gathers the per-candidate
logliks over RCCL and reduces the best candidate (weak scaling).

Other configs (same JSON contract, `config.workload` names them):
  3  TVλ EKF, N = 360 maturities, T = 600, B = 16,384 θ per GPU (weak scaling)
  4  rolling re-estimation: 240 expanding windows T_w = 361..600 × 4,096 θ = 983,040 evals,
     every window's θ split evenly over the GPUs, RCCL all-gather of logliks (strong scaling)
  5  5-factor GNS extension: 1,048,576 candidates split over the GPUs, RCCL argmax (strong)

Prints ONE JSON line on rank 0 with a `roofline` object (FP64 VALU bound, SURVEY §8d
algorithmic flops ÷ HIP-event time of the launches on the library's stream) and a
`cpu_baseline` object (the faithful dense-LU C restatement, oracle/yfm_oracle.c, on a
bounded sample of the same workload, OpenMP over the host cores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))
sys.path.insert(0, str(ROOT))

from yfm_amd import KIND_DNS, KIND_GNS, KIND_TVL, Engine, n_params, state_dim  # noqa: E402
from yfm_amd import distributed as D  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, AMD spec (the local guide lists no FP64 figure)
METRIC = "Kalman loglik evals/sec (DNS, T=600, N=30)"


def alg_flops_step(kind: int, N: int, M: int) -> float:
    """SURVEY.md §8(d) algorithmic FP64 flops of one update step (capacitance/Woodbury form):
    fixed loadings 4NM + 3N + 12⅔M³ + 6M² + 6M + 8; TVλ ≈ 62N + 939 (+ N+1 exps, not counted)."""
    if kind == KIND_TVL:
        return 62.0 * N + 939.0
    return 4 * N * M + 3 * N + (38.0 / 3.0) * M ** 3 + 6 * M * M + 6 * M + 8


def alg_flops(kind: int, N: int, M: int, T) -> np.ndarray:
    """Per-eval algorithmic flops for window lengths T (scalar or array): (T-1)·F_step + 2NM² + 2(M²)³."""
    T = np.asarray(T, dtype=np.float64)
    return (T - 1) * alg_flops_step(kind, N, M) + 2 * N * M * M + 2 * (M * M) ** 3


@dataclass
class Workload:
    config: int
    kind: int
    label: str
    mats: np.ndarray
    Y: np.ndarray
    Theta: np.ndarray          # this rank's θ (P×B)
    T_use: np.ndarray | None   # this rank's window lengths (B) or None
    global_batch: int
    scaling: str
    gather: bool               # all-gather every candidate's loglik
    extra: dict = field(default_factory=dict)
    counts: list | None = None  # per-rank batch sizes when they differ


def make_workload(config: int, world: int, rank: int, T: int, batch: int | None) -> Workload:
    if config == 2:
        B = batch or 65536
        mats = S.maturities_30()
        return Workload(2, KIND_DNS, f"config2: DNS loglik over {B:,} θ per GPU", mats, S.simulate_panel(KIND_DNS, T),
                        S.theta_batch(KIND_DNS, B, seed=S.BATCH_SEED + rank), None, world * B, "weak", True)
    if config == 3:
        B = batch or 16384
        mats = S.maturities_360()
        Th = S.theta_batch(KIND_TVL, B, seed=S.BATCH_SEED + rank, bad_frac=0.0, scale=0.02)
        return Workload(3, KIND_TVL, f"config3: TVλ EKF loglik, N=360, over {B:,} θ per GPU", mats,
                        S.simulate_panel(KIND_TVL, T, maturities=mats), Th, None, world * B, "weak", True)
    if config == 4:
        per = batch or 4096
        wins = np.arange(361, 601) if T == 600 else np.arange(max(2, T - 239), T + 1)
        counts = [per] * len(wins)
        idx = D.window_shards(counts, world, rank)
        Th_all = S.theta_batch(KIND_DNS, per, seed=S.BATCH_SEED)  # the same 4,096 θ re-fit per window
        Th = np.asfortranarray(Th_all[:, idx % per])
        tu = np.repeat(wins, per)[idx].astype(np.int32)
        mats = S.maturities_30()
        return Workload(4, KIND_DNS, f"config4: DNS rolling windows, {len(wins)} expanding windows × {per:,} θ "
                        f"= {len(wins) * per:,} evals split over {world} GPU(s)", mats, S.simulate_panel(KIND_DNS, T),
                        Th, tu, len(wins) * per, "strong", True, {"windows": [int(wins[0]), int(wins[-1])]},
                        [len(D.window_shards(counts, world, r)) for r in range(world)])
    if config == 5:
        total = batch or 1 << 20
        lo, hi = D.shard_range(total, world, rank)
        # θ_b for b in [lo, hi) of the global search (generated per shard from the global seed stream)
        Th_all = S.theta_batch(KIND_GNS, hi, seed=S.BATCH_SEED, bad_frac=0.0, scale=0.1)
        mats = S.maturities_30()
        return Workload(5, KIND_GNS, f"config5: 5-factor GNS global search, {total:,} candidates split over "
                        f"{world} GPU(s), RCCL argmax", mats, S.simulate_panel(KIND_GNS, T),
                        np.asfortranarray(Th_all[:, lo:hi]), None, total, "strong", False, {"offset": lo})
    raise ValueError(config)


def cpu_baseline(w: Workload, seconds: float, gpu_out: np.ndarray):
    """Faithful reference-path restatement on the host: time a bounded sample of the same workload."""
    lib = ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so"))
    Dp = ctypes.POINTER(ctypes.c_double)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    Yf = np.asfortranarray(w.Y)
    N, T = Yf.shape
    P = w.Theta.shape[0]
    # sample order: the batch as laid out, except for windows (config 4), where a seeded permutation
    # keeps the sample's mix of window lengths equal to the workload's
    order = np.arange(w.Theta.shape[1]) if w.T_use is None else np.random.default_rng(0).permutation(w.Theta.shape[1])
    done, t0 = 0, time.perf_counter()
    chunk = threads if w.kind == KIND_TVL else 2 * threads
    res = []
    while time.perf_counter() - t0 < seconds and done + chunk <= w.Theta.shape[1]:
        sel = order[done:done + chunk]
        sub = np.asfortranarray(w.Theta[:, sel])
        out = np.empty(chunk)
        tu = None
        if w.T_use is not None:
            tu = np.ascontiguousarray(w.T_use[sel], dtype=np.int32)
        lib.yfm_oracle_loglik(w.kind, 0, Yf.ctypes.data_as(Dp), N, T, w.mats.ctypes.data_as(Dp), sub.ctypes.data_as(Dp),
                              P, chunk, None if tu is None else tu.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                              out.ctypes.data_as(Dp), threads)
        res.append(out)
        done += chunk
    dt = time.perf_counter() - t0
    ref = np.concatenate(res) if res else np.zeros(0)
    got = gpu_out[order[:done]]
    fin = np.isfinite(ref)
    same_pattern = bool(np.array_equal(np.isfinite(got), fin) and np.array_equal(np.isnan(got), np.isnan(ref)))
    err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), 1e-300)
    parity = {"pattern_match": same_pattern, "gpu_vs_oracle_max_rel": float(err.max()) if err.size else 0.0,
              "frac_within_1e-9": float((err <= 1e-9).mean()) if err.size else 1.0}
    if w.kind in (KIND_DNS, KIND_GNS) and w.T_use is None:
        # adjudicate with the extended-precision truth proxy on the first 512 of the sample
        from oracle.kalman_ld import loglik_ld
        k = min(512, done)
        tru = loglik_ld(w.kind, w.mats, w.Y, w.Theta[:, :k])
        ft = np.isfinite(tru)
        e_gpu = np.abs(got[:k][ft] - tru[ft]) / np.abs(tru[ft])
        e_ref = np.abs(ref[:k][ft] - tru[ft]) / np.abs(tru[ft])
        parity.update(truth_subset=k, gpu_vs_truth_max_rel=float(e_gpu.max()) if e_gpu.size else 0.0,
                      oracle_vs_truth_max_rel=float(e_ref.max()) if e_ref.size else 0.0)
    win = "" if w.T_use is None else " with the workload's window lengths"
    # config 1 (BASELINE.json configs[0]): one θ, single thread — the reference's own CPU case
    th0 = np.asfortranarray(w.Theta[:, :1])
    one = np.empty(1)
    n1, t1 = 0, time.perf_counter()
    while n1 < 3 or (time.perf_counter() - t1 < 2.0 and n1 < 200):
        lib.yfm_oracle_loglik(w.kind, 0, Yf.ctypes.data_as(Dp), N, T, w.mats.ctypes.data_as(Dp), th0.ctypes.data_as(Dp),
                              P, 1, None, one.ctypes.data_as(Dp), 1)
        n1 += 1
    ms1 = 1e3 * (time.perf_counter() - t1) / n1
    return {"value": done / dt if dt > 0 else 0.0, "unit": "evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} of the benchmark's θ (T={T}, N={N}){win} in {dt:.1f} s, dense N×N getrf+getri + "
                      f"logdet LU per step (oracle/yfm_oracle.c, -O3, OpenMP {threads} threads)",
            "single_theta_1_thread": {"ms_per_eval": ms1, "evals_per_s": 1e3 / ms1, "evals_timed": n1},
            "parity": parity}


def pmc_executed_flops(kernel_substr: str):
    """Executed FP64 flops per filter step of the dominant kernel from the committed PMC valu pass (T = 600):
    (FMA·2 + ADD + MUL)·64 + MFMA_MOPS_F64·512 (the expression of rocprof's SQ_INSTS_VALU_FLOPS_FP64)."""
    for rnd in sorted((ROOT / "profiles").glob("r*/**/pmc_summary.json"), reverse=True):
        d = json.loads(rnd.read_text())
        for k, v in d.items():
            if kernel_substr in k and "fp64_flops_executed_per_step" in v:
                return v["fp64_flops_executed_per_step"]
    return None


def pmc_traffic(kernel_substr: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc passes
    (tools/profile_all.sh → profiles/<round>/**/pmc_summary.json), corrected as
    MI355X_MICROARCH.md §HBM prescribes for gfx950: FETCH_SIZE counts half the bytes of wide
    coalesced reads, so traffic = 2·FETCH_SIZE + WRITE_SIZE (both reported in KiB)."""
    for rnd in sorted((ROOT / "profiles").glob("r*/**/pmc_summary.json"), reverse=True):
        d = json.loads(rnd.read_text())
        for k, v in d.items():
            if kernel_substr in k and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                return (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0, str(rnd.relative_to(ROOT))
    return None, None


DOMINANT = {KIND_DNS: "fixedz_loglik_kernel<30, 3, 1, false>", KIND_TVL: "tvl_loglik_kernel",
            KIND_GNS: "fixedz_loglik_kernel<30, 5, 2, false>"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--batch", type=int, default=None, help="θ per GPU (2, 3), per window (4), total (5)")
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

    w = make_workload(args.config, world, rank, args.T, args.batch)
    kind = w.kind
    M, P = state_dim(kind), n_params(kind)
    N, T = w.Y.shape
    B = w.Theta.shape[1]
    eng = Engine(dev.index)
    eng.set_panel(w.Y, w.mats)
    d_th = torch.from_numpy(np.ascontiguousarray(w.Theta.T)).to(dev)  # (B, P) C-order == P×B column-major
    d_tu = torch.from_numpy(w.T_use).to(dev) if w.T_use is not None else None
    d_out = torch.empty(B, dtype=torch.float64, device=dev)
    offset = w.extra.get("offset", 0)
    counts = w.counts or [B] * world
    stream = torch.cuda.current_stream(dev)

    # N > 1: the kernel runs on a compute stream into one of two output buffers while the
    # previous step's collectives (RCCL all-gather + argmax) run on torch's stream — step k's
    # gather overlaps step k+1's filter.  Events order buffer reuse both ways.
    comp = torch.cuda.Stream(dev) if world > 1 else stream
    outs = [d_out, torch.empty_like(d_out)] if world > 1 else [d_out]
    k_done = [torch.cuda.Event() for _ in outs]
    c_done = [torch.cuda.Event() for _ in outs]
    k_times = []  # (start, end) HIP events around each timed launch, on the launch stream
    timing = [False]
    it = [0]

    def step():
        i = it[0] % len(outs)
        it[0] += 1
        o = outs[i]
        if world > 1:
            comp.wait_event(c_done[i])  # the collective that last read buffer i has finished
        if timing[0]:
            ks, ke = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ks.record(comp)
        eng.loglik_device(kind, d_th.data_ptr(), P, B, o.data_ptr(), space=0,
                          d_T_use=d_tu.data_ptr() if d_tu is not None else None, stream=comp.cuda_stream)
        if timing[0]:
            ke.record(comp)
            k_times.append((ks, ke))
        if world > 1:  # RCCL over xGMI: gather logliks and/or reduce the best candidate
            k_done[i].record(comp)
            stream.wait_event(k_done[i])
            if w.gather:
                D.gather_logliks(o, counts)
            D.best_candidate_device(o, offset)
            c_done[i].record(stream)

    for e in c_done:
        e.record(stream)
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    timing[0] = True
    t0 = time.perf_counter()
    ev0.record(stream)
    comp.wait_stream(stream)
    for _ in range(args.steps):
        step()
    stream.wait_stream(comp)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    timing[0] = False
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    # kernel time of one batch: HIP events around each launch in the timed region, on its stream
    kernel_ms = float(np.mean([ks.elapsed_time(ke) for ks, ke in k_times]))

    ms_per_step = 1e3 * wall / args.steps
    value = w.global_batch / (wall / args.steps)
    f_rank = float(np.sum(alg_flops(kind, N, M, w.T_use if w.T_use is not None else T)) if w.T_use is not None
                   else alg_flops(kind, N, M, T) * B)
    achieved = f_rank / (kernel_ms * 1e-3) / 1e12  # TFLOP/s of this GPU's launches
    traffic, traffic_src = pmc_traffic(DOMINANT[kind])
    exe = pmc_executed_flops(DOMINANT[kind])
    steps = float(np.sum(w.T_use - 1)) if w.T_use is not None else float(B * (T - 1))
    exe_tf = exe * steps / (kernel_ms * 1e-3) / 1e12 if exe else None
    out_host = d_out.cpu().numpy()
    n_neginf, n_nan = int(np.isneginf(out_host).sum()), int(np.isnan(out_host).sum())

    # host-pointer boundary (yfm_loglik_batch: θ in over PCIe, logliks back, synchronous) —
    # reported beside the metric, never as `value` (inputs are not HBM-resident there)
    host_rate = None
    if rank == 0 and world == 1:
        Th_host = np.asfortranarray(w.Theta)
        tu_host = w.T_use
        eng.loglik(kind, Th_host, space=0, T_use=tu_host)
        reps = max(3, min(args.steps, 10))
        th0 = time.perf_counter()
        for _ in range(reps):
            eng.loglik(kind, Th_host, space=0, T_use=tu_host)
        host_s = (time.perf_counter() - th0) / reps
        host_rate = {"evals_per_s": B / host_s, "ms_per_call": 1e3 * host_s, "calls": reps,
                     "note": "yfm_loglik_batch with host θ / host logliks (H2D + kernel + D2H, synchronous)"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(w, args.cpu_seconds, out_host)

    if rank == 0:
        line = {
            "metric": METRIC if args.config == 2 else f"Kalman loglik evals/sec (config {args.config})",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": w.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (model-simulated panel, seeded θ batch)",
            "config": {"workload": w.label, "kind": {KIND_DNS: "DNS (1C)", KIND_TVL: "TVλ (EKF)",
                                                      KIND_GNS: "GNS5 (extension)"}[kind],
                       "T": T, "N": N, "batch_per_gpu": B, "global_batch": w.global_batch,
                       "parallelism": f"dp{world} (θ sharded, RCCL "
                                      f"{'all-gather of logliks + ' if w.gather else ''}argmax)", **w.extra},
            "roofline": {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes": B * (P + 1) * 8 + T * (N + 4) * 8,
                         "kernel_ms": kernel_ms, "flops_per_eval": f_rank / max(B, 1),
                         "executed_tflops": exe_tf, "executed_frac": exe_tf / FP64_PEAK_TFLOPS if exe_tf else None,
                         "note": "achieved = SURVEY §8d algorithmic flops of this GPU's batch ÷ HIP-event time of its "
                                 "launches on the library stream; the §8d count is for the capacitance form, this "
                                 "build's collapsed form executes about half of it (executed_* = PMC-counted FP64 "
                                 "flops of the same launch from profiles/, which is why frac can exceed 1)"},
            "cpu_baseline": cpu,
            "host_pointer_rate": host_rate,
            "outputs": {"neg_inf": n_neginf, "nan": n_nan},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
