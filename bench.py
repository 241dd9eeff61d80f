"""Benchmark: batched Kalman log-likelihood evals/s on MI355X (BASELINE.json configs 2-5).

    python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N > 1` without a launcher (WORLD_SIZE unset) starts the N ranks itself
(yfm_amd.distributed.spawn_local_ranks: one fresh process per GPU, 127.0.0.1 rendezvous), so
`python bench.py --gpus 8` and the torchrun form run the same N-rank job; a rank whose process
group does not have N members exits non-zero.

Default (`--config 2`, the metric's headline workload): one "step" = one batched DNS
loglik over B = 65,536 parameter vectors per GPU (T = 600 months × N = 30 maturities,
FP64), inputs resident in HBM; for N > 1 the step also all-gathers the per-candidate
logliks over RCCL and reduces the best candidate (weak scaling).

Other configs (same JSON contract, `config.workload` names them):
  3  TVλ EKF, N = 360 maturities, T = 600, B = 16,384 θ per GPU (weak scaling)
  4  rolling re-estimation: 240 expanding windows T_w = 361..600 × 4,096 θ = 983,040 evals,
     every window's θ split evenly over the GPUs, RCCL all-gather of logliks (strong scaling)
  5  5-factor GNS extension: 1,048,576 candidates split over the GPUs, RCCL argmax (strong)

Prints ONE JSON line on rank 0 with a `roofline` object (FP64 VALU bound: the algorithmic flops
of the formulation the dominant kernel runs ÷ HIP-event time of its launches on the library's
stream) and a `cpu_baseline` object (the faithful dense-LU C restatement, oracle/yfm_oracle.c, on
a bounded sample of the same workload, OpenMP over the host cores; plus the optimised CPU variant
and the binary128-adjudicated parity of the sample).  TVλ runs in the library's default certified
(double-double) precision; `fp64_mode` reports the FP64 mode beside it.
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
from yfm_amd import _lib  # noqa: E402
from yfm_amd import distributed as D  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, AMD spec (the local guide lists no FP64 figure)
# v_fma_f64 microbenchmark at steady clock, straight-line (tools/fp64_waves.hip, profiles/r5/micro/fp64_waves.txt):
# 76.1 TFLOP/s at 8 waves per SIMD, 72.7 at ONE wave per SIMD with 32 independent chains (62.2 with 4).  (The
# round-1 probe, tools/fp64_peak.hip, kept its loop branch in every 16 FMAs and read 42.9 at one wave: loop overhead,
# not a one-wave issue limit.)
FP64_MEASURED_TFLOPS = 76.1
FP64_ONE_WAVE_TFLOPS = 72.7
METRIC = "Kalman loglik evals/sec (DNS, T=600, N=30)"


def collapsed_update_flops(M: int) -> float:
    """FP64 operations of one collapsed-form measurement + time update at state dimension M, as
    yfm_fixedz.hpp runs it (a division / reciprocal counts as one operation): ĉ = G⁻¹Z'y from z̃,
    the residual ỹ'ỹ − z̃'ĉ, S = P + R, its LDLᵀ, the solves for c and the M columns of R, q,
    β_{t|t}, P_{t|t}, β ← δ + Φβ, P ← ΦPΦ' + Q and the loglik accumulation."""
    nz = M - 1
    f = nz + 2 * M * nz + 2 * nz + 1          # z̃/σ², ĉ, residual, ĉ₀ += ȳ
    f += M + M * (M + 1) // 2                 # c = ĉ − β, S = P + R (lower)
    f += sum(2 * j + 1 + (M - 1 - j) * (2 * j + 1) for j in range(M)) + (M - 1)  # LDLᵀ + det
    solve = 2 * M * (M - 1) + M
    f += solve + 2 * M + 2                    # x = S⁻¹c, c'x, q
    f += 2 * M * M                            # β_{t|t} = β + P x
    f += M * solve + M * M * (M + 1)          # S⁻¹R column by column, P_{t|t} = P S⁻¹R
    f += 2 * M * M + 2 * M ** 3 + M * M * (M + 1)  # β ← δ + Φβ, A = ΦP, P = AΦ' + Q
    return f + 3


def steady_update_flops(M: int) -> float:
    """FP64 operations of one steady-state step of the DNS kernel (frozen covariance, yfm_fixedz.hpp
    FixedZFilter::steady_step): ĉ, the residual, c = ĉ − β, x = S⁻¹c with the cached LDLᵀ factors,
    c'x, q, β_{t|t} = β + P x, β ← δ + Φβ and the loglik accumulation — the covariance half is not run."""
    nz = M - 1
    f = nz + 2 * M * nz + 2 * nz + 1 + M      # z̃/σ², ĉ, residual, ĉ₀ += ȳ, c = ĉ − β
    f += 2 * M * (M - 1) + M + 2 * M + 2      # x = S⁻¹c, c'x, q
    f += 2 * M * M + 2 * M * M                # β_{t|t} = β + P x, β ← δ + Φβ
    if M > 3:                                 # GNS5 refactors the constant S each steady step (no cached factors)
        f += M * (M + 1) // 2                 # S = P + R (lower)
        f += sum(2 * j + 1 + (M - 1 - j) * (2 * j + 1) for j in range(M)) + (M - 1)  # LDLᵀ + det
    return f + 3


def alg_flops_step(kind: int, N: int, M: int) -> float:
    """Algorithmic FP64 flops of one update step of the formulation this build runs:
    fixed loadings (DNS, GNS5): the collapsed form — z̃ = Z'ỹ (2N(M−1)) plus the M×M update;
    TVλ: the capacitance form of SURVEY.md §8(d), 62N + 939 (+ N+1 exps, not counted)."""
    if kind == KIND_TVL:
        return 62.0 * N + 939.0
    return 2.0 * N * (M - 1) + collapsed_update_flops(M)


def survey_flops_step(kind: int, N: int, M: int) -> float:
    """SURVEY.md §8(d)'s per-step count (capacitance/Woodbury form): 4NM + 3N + 12⅔M³ + 6M² + 6M + 8."""
    if kind == KIND_TVL:
        return 62.0 * N + 939.0
    return 4 * N * M + 3 * N + (38.0 / 3.0) * M ** 3 + 6 * M * M + 6 * M + 8


def alg_flops(kind: int, N: int, M: int, T, step=alg_flops_step) -> np.ndarray:
    """Per-eval flops for window lengths T (scalar or array): (T-1)·F_step + 2NM² + 2(M²)³ (init)."""
    T = np.asarray(T, dtype=np.float64)
    return (T - 1) * step(kind, N, M) + 2 * N * M * M + 2 * (M * M) ** 3


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
        # the windows longest first: waves run in rounds of one per SIMD, so the last, partial round holds the
        # shortest windows (longest-processing-time-first; at 8 GPUs a rank's 1,920 waves take 1.875 rounds)
        wins = np.arange(600, 360, -1) if T == 600 else np.arange(T, max(2, T - 239) - 1, -1)
        counts = [per] * len(wins)
        idx = D.window_shards(counts, world, rank)
        Th_all = S.theta_batch(KIND_DNS, per, seed=S.BATCH_SEED)  # the same 4,096 θ re-fit per window
        Th = np.asfortranarray(Th_all[:, idx % per])
        tu = np.repeat(wins, per)[idx].astype(np.int32)
        mats = S.maturities_30()
        return Workload(4, KIND_DNS, f"config4: DNS rolling windows, {len(wins)} expanding windows × {per:,} θ "
                        f"= {len(wins) * per:,} evals split over {world} GPU(s)", mats, S.simulate_panel(KIND_DNS, T),
                        Th, tu, len(wins) * per, "strong", True,
                        {"windows": [int(wins.min()), int(wins.max())], "window_order": "longest first"},
                        [len(D.window_shards(counts, world, r)) for r in range(world)])
    if config == 5:
        total = batch or 1 << 20
        lo, hi = D.shard_range(total, world, rank)
        # θ_b for b in [lo, hi) of the global search: candidate b depends only on (seed, b)
        mats = S.maturities_30()
        return Workload(5, KIND_GNS, f"config5: 5-factor GNS global search, {total:,} candidates split over "
                        f"{world} GPU(s), RCCL argmax", mats, S.simulate_panel(KIND_GNS, T),
                        S.theta_range(KIND_GNS, lo, hi, scale=0.1), None, total, "strong", False, {"offset": lo})
    raise ValueError(config)


def _host_cpu() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_topology() -> dict:
    """The host CPU share this process may use: logical CPUs in its affinity mask, the cgroup CPU quota
    (cpu.max; the GPU boxes grant each job a share of a larger machine), and the host's physical
    cores.  The CPU baselines run min(affinity, quota) OpenMP threads — every CPU the job may use,
    no more (more threads than the quota would only time-slice)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    phys = set()
    try:
        pid = cid = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                cid = line.split(":")[1].strip()
            elif not line.strip():
                if cid is not None:
                    phys.add((pid, cid))
                pid = cid = None
    except OSError:
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return {"threads_used": threads, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "host_logical_cpus": os.cpu_count(), "host_physical_cores": len(phys) or None, "host_cpu": _host_cpu()}


def _native_libs():
    """The dense port and the optimised variant built with -march=native for THIS host (the in-tree
    builds target x86-64-v3 so they load anywhere); falls back to the in-tree builds."""
    import subprocess
    import tempfile
    out = Path(tempfile.mkdtemp(prefix="yfm_cpu_"))
    try:
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "-s", "native", f"OUT={out}"], check=True,
                       capture_output=True, timeout=120)
        return (ctypes.CDLL(str(out / "libyfm_oracle_native.so")), ctypes.CDLL(str(out / "libyfm_cpu_fast_native.so")),
                "-O3 -march=native")
    except Exception:  # noqa: BLE001
        return (ctypes.CDLL(str(ROOT / "oracle" / "libyfm_oracle.so")),
                ctypes.CDLL(str(ROOT / "oracle" / "libyfm_cpu_fast.so")), "-O3 -march=x86-64-v3 (native build failed)")


def _timed(fn, w: Workload, order, chunk, threads, seconds, min_chunks=1):
    """Evaluate the sample w.Theta[:, order] chunk by chunk with fn(…) until `seconds` have passed;
    returns (evals/s, evaluated count, logliks)."""
    Dp = ctypes.POINTER(ctypes.c_double)
    Yf = np.asfortranarray(w.Y)
    N, T = Yf.shape
    P = w.Theta.shape[0]
    done, res, t0 = 0, [], time.perf_counter()
    while (time.perf_counter() - t0 < seconds or len(res) < min_chunks) and done + chunk <= len(order):
        sel = order[done:done + chunk]
        sub = np.asfortranarray(w.Theta[:, sel])
        out = np.empty(chunk)
        tu = None if w.T_use is None else np.ascontiguousarray(w.T_use[sel], dtype=np.int32)
        fn(w.kind, 0, Yf.ctypes.data_as(Dp), N, T, w.mats.ctypes.data_as(Dp), sub.ctypes.data_as(Dp), P, chunk,
           None if tu is None else tu.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), out.ctypes.data_as(Dp), threads)
        res.append(out)
        done += chunk
    dt = time.perf_counter() - t0
    return (done / dt if dt > 0 else 0.0), done, (np.concatenate(res) if res else np.zeros(0))


def cpu_baseline(w: Workload, seconds: float, gpu_out: np.ndarray):
    """CPU paths on the host cores, each on a bounded sample of the same workload:
      value                  — the faithful restatement of the reference (oracle/yfm_oracle.c: N×N
                               getrf+getri + logdet LU every step), OpenMP over the host threads;
      dense_batch_1_thread   — the same on a threads×64 batch at 1 thread (BASELINE.md protocol);
      single_theta_1_thread  — config 1: one θ, one thread;
      optimised              — the CPU counterpart of the GPU algorithm (oracle/yfm_cpu_fast.c:
                               collapsed form, 8 candidates per vector; TVλ capacitance form), at
                               the host threads and at 1 thread — NOT the reference's algorithm;
      parity                 — GPU vs the dense oracle on the sample, adjudicated by the binary128
                               truth (oracle/yfm_truth.c): (within 1e-9, adjudicated, failing)."""
    from oracle.truth import loglik_truth
    dense, fast, flags = _native_libs()
    topo = cpu_topology()
    threads = topo["threads_used"]
    B = w.Theta.shape[1]
    # sample order: the batch as laid out, except for windows (config 4), where a seeded permutation
    # keeps the sample's mix of window lengths equal to the workload's
    order = np.arange(B) if w.T_use is None else np.random.default_rng(0).permutation(B)
    tvl = w.kind == KIND_TVL
    # a small batch (config 3 at B = 1 or 1,024) is cycled so every timed chunk below is full
    order = np.resize(order, max(B, 64 * 2 * threads))
    rate, done, ref = _timed(dense.yfm_oracle_loglik, w, order, threads if tvl else 2 * threads, threads, seconds)
    N, T = w.Y.shape
    win = "" if w.T_use is None else " with the workload's window lengths"
    out = {"value": rate, "unit": "evals/s", "cores": threads, "kind": "port", "host_cpu": _host_cpu(),
           "topology": topo,
           "sample": f"{done} of the benchmark's θ (T={T}, N={N}){win}, dense N×N getrf+getri + logdet LU per step "
                     f"(oracle/yfm_oracle.c, {flags}, OpenMP {threads} threads)"}
    # a threads×64 batch at 1 thread (bounded: TVλ evals take seconds each)
    r1, n1, _ = _timed(dense.yfm_oracle_loglik, w, order, 1, 1, min(seconds, 8.0), min_chunks=3)
    out["dense_batch_1_thread"] = {"evals_per_s": r1, "evals_timed": n1, "batch": threads * 64,
                                   "note": "bounded by time; the full batch would take "
                                           f"{threads * 64 / max(r1, 1e-12):.0f} s"}
    th0 = np.asfortranarray(w.Theta[:, :1])
    w1 = Workload(w.config, w.kind, w.label, w.mats, w.Y, th0, None, 1, w.scaling, False)
    r0, n0, _ = _timed(dense.yfm_oracle_loglik, w1, np.zeros(200, dtype=np.int64), 1, 1, 2.0, min_chunks=3)
    out["single_theta_1_thread"] = {"ms_per_eval": 1e3 / r0, "evals_per_s": r0, "evals_timed": n0}
    ro, no, _ = _timed(fast.yfm_cpu_fast_loglik, w, order, 64 * threads if not tvl else 4 * threads, threads,
                       min(seconds, 5.0), min_chunks=2)
    ro1, no1, _ = _timed(fast.yfm_cpu_fast_loglik, w, order, 64 if not tvl else 4, 1, min(seconds, 3.0), min_chunks=2)
    full = topo["host_physical_cores"]
    out["optimised"] = {"evals_per_s": ro, "evals_timed": no, "cores": threads, "evals_per_s_1_thread": ro1,
                        "evals_timed_1_thread": no1,
                        "extrapolated_all_physical_cores": (ro1 * full if full else None),
                        "extrapolation": f"1-thread rate × {full} physical cores of the host (linear scaling "
                                         "assumed, an upper bound; only the measured rates are timed)",
                        "kind": "optimised CPU variant, NOT the reference algorithm: "
                                + ("capacitance form, one candidate per thread" if tvl else
                                   "collapsed form of DESIGN.md §3.1, 8 candidates per SIMD vector")
                                + f" (oracle/yfm_cpu_fast.c, {flags})"}
    # parity on the dense sample, adjudicated by the binary128 truth
    k = min(done, 64 if tvl else 512)
    sel = order[:k]
    got = gpu_out[sel]
    tru = loglik_truth(w.kind, w.Y, w.mats, w.Theta[:, sel], T_use=None if w.T_use is None else w.T_use[sel],
                       nthreads=threads)
    o = ref[:k]
    pat = bool(np.array_equal(np.isfinite(got), np.isfinite(o)) and np.array_equal(np.isnan(got), np.isnan(o)))
    fin = np.isfinite(o) & np.isfinite(got)
    e_go = np.abs(got[fin] - o[fin]) / np.maximum(np.abs(o[fin]), 1e-300)
    e_gt = np.abs(got[fin] - tru[fin]) / np.maximum(np.abs(tru[fin]), 1e-300)
    e_ot = np.abs(o[fin] - tru[fin]) / np.maximum(np.abs(tru[fin]), 1e-300)
    within = e_go <= 1e-9
    adj = ~within & (e_gt <= e_ot)
    g_all = gpu_out[order[:done]]
    both = np.isfinite(ref) & np.isfinite(g_all)  # −Inf − −Inf would be NaN: compare finite pairs only
    e_all = np.abs(g_all[both] - ref[both]) / np.maximum(np.abs(ref[both]), 1e-300)
    # a finite oracle value the GPU did not reproduce counts as outside 1e-9
    n_ref = int(np.isfinite(ref).sum())
    out["parity"] = {"pattern_match": pat, "sample": int(k), "within_1e-9": int(within.sum()),
                     "adjudicated": int(adj.sum()), "failing": int((~within & ~adj).sum()),
                     "gpu_vs_truth_max_rel": float(e_gt.max()) if e_gt.size else 0.0,
                     "oracle_vs_truth_max_rel": float(e_ot.max()) if e_ot.size else 0.0,
                     "frac_within_1e-9_whole_sample": float(np.sum(e_all <= 1e-9) / n_ref) if n_ref else 1.0,
                     "rule": "within 1e-9 of the dense oracle, or |gpu − truth| ≤ |oracle − truth| (binary128 truth)"}
    return out


def pmc_executed_flops(kernel_substr: str, evals: int):
    """Executed FP64 flops per filter step of the dominant kernel from the committed PMC valu pass (T = 600):
    (FMA·2 + ADD + MUL)·64 + MFMA_MOPS_F64·512 (the expression of rocprof's SQ_INSTS_VALU_FLOPS_FP64)."""
    for rnd in sorted((ROOT / "profiles").glob("r*/**/pmc_summary.json"), reverse=True):
        d = json.loads(rnd.read_text())
        for k, v in d.items():
            if kernel_substr in k and "fp64_flops_executed_per_step" in v and \
                    int(v.get("evals_per_launch", evals)) == int(evals):  # the same launch size only
                return v["fp64_flops_executed_per_step"]
    return None


def pmc_traffic(kernel_substr: str, evals: int):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc passes
    (tools/profile_all.sh → profiles/<round>/**/pmc_summary.json), corrected as
    MI355X_MICROARCH.md §HBM prescribes for gfx950: FETCH_SIZE counts half the bytes of wide
    coalesced reads, so traffic = 2·FETCH_SIZE + WRITE_SIZE (both reported in KiB)."""
    for rnd in sorted((ROOT / "profiles").glob("r*/**/pmc_summary.json"), reverse=True):
        d = json.loads(rnd.read_text())
        for k, v in d.items():
            if kernel_substr in k and "FETCH_SIZE" in v and "WRITE_SIZE" in v and \
                    int(v.get("evals_per_launch", evals)) == int(evals):  # the same launch size only
                return (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0, str(rnd.relative_to(ROOT))
    return None, None


# the instantiation each configuration runs: fixedz_loglik_kernel<NP, M, LEAD, RECORD, STEADY, SPLIT_FORM>
# (DNS: frozen-covariance steady state by default; GNS5: full recursion unless YFM_GNS5_STEADY=1)
DOMINANT = {(KIND_DNS, "steady"): "fixedz_loglik_kernel<30, 3, 1, false, true, false>",
            (KIND_DNS, "full"): "fixedz_loglik_kernel<30, 3, 1, false, false, false>",
            (KIND_GNS, "steady"): "fixedz_loglik_kernel<30, 5, 2, false, true, false>",
            (KIND_GNS, "full"): "fixedz_loglik_kernel<30, 5, 2, false, false, false>",
            (KIND_TVL, "fp64"): "tvl_loglik_kernel", (KIND_TVL, "certified"): "tvl_dd_loglik_kernel"}


def dominant_kernel(kind, prec):
    env = os.environ.get
    if kind == KIND_TVL:
        return DOMINANT[(kind, prec)]
    if env("YFM_DNS_STEADY", "1").startswith("0"):
        return DOMINANT[(kind, "full")]
    if kind == KIND_GNS:
        return DOMINANT[(kind, "steady" if env("YFM_GNS5_STEADY", "0").startswith("1") else "full")]
    return DOMINANT[(kind, "steady")]


def roofline(kind, prec, N, M, T, T_use, B, P, kernel_ms, steady_lane_steps=0):
    """The dominant kernel against the FP64 VALU roofline: achieved = algorithmic flops of the
    formulation it runs (alg_flops) for this GPU's batch ÷ HIP-event time per launch.  Filter steps
    run in the DNS/GNS5 kernel's frozen-covariance steady state (`steady_lane_steps`, measured by the
    kernel: yfm_last_batch_steady × 64) count the steady step's flops instead of the full update's."""
    Tb = T_use if T_use is not None else np.full(B, T)
    f_rank = float(np.sum(alg_flops(kind, N, M, Tb)))
    f_rank -= steady_lane_steps * (collapsed_update_flops(M) - steady_update_flops(M))
    f_survey = float(np.sum(alg_flops(kind, N, M, Tb, survey_flops_step)))
    achieved = f_rank / (kernel_ms * 1e-3) / 1e12
    name = dominant_kernel(kind, prec)
    traffic, traffic_src = pmc_traffic(name, B)
    exe = pmc_executed_flops(name, B)
    steps = float(np.sum(Tb - 1))
    exe_tf = exe * steps / (kernel_ms * 1e-3) / 1e12 if exe else None
    return {"bound": "fp64-valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS, "frac_vs_measured_peak": achieved / FP64_MEASURED_TFLOPS,
            "measured_peak": FP64_MEASURED_TFLOPS, "one_wave_peak": FP64_ONE_WAVE_TFLOPS,
            "traffic": traffic, "traffic_source": traffic_src,
            "algorithmic_bytes": B * (P + 1) * 8 + T * (N + 4) * 8, "kernel": name, "kernel_ms": kernel_ms,
            "flops_per_eval": f_rank / max(B, 1),
            "flop_model": ("SURVEY §8d capacitance form (62N + 939 per step)" if kind == KIND_TVL else
                           "collapsed form: 2N(M−1) for Z'ỹ + the M×M update (bench.py collapsed_update_flops); "
                           "frozen-covariance steady steps: 2N(M−1) + the mean update (steady_update_flops)"),
            "steady_lane_steps": int(steady_lane_steps),
            "survey_equiv_tflops": f_survey / (kernel_ms * 1e-3) / 1e12,
            "executed_tflops": exe_tf, "executed_frac": exe_tf / FP64_PEAK_TFLOPS if exe_tf else None,
            "executed_frac_vs_measured_peak": exe_tf / FP64_MEASURED_TFLOPS if exe_tf else None,
            "note": "kernel_ms = HIP events around each library call in the timed region, on its stream "
                    "(TVλ: init + filter kernels); executed_* = PMC-counted FP64 flops of the same kernel "
                    "(profiles/); peak = AMD spec, measured_peak = v_fma_f64 microbenchmark at 8 waves/SIMD "
                    "(one_wave_peak: at one wave/SIMD, the occupancy of these kernels)"
                    + ("; certified precision runs the same algorithm in double-double (≈7× the FP64 "
                       "instructions), frac is of the algorithm's FP64 count" if kind == KIND_TVL and prec == "certified"
                       else "")}


def emulate_world(args) -> dict:
    """Predict the N-GPU efficiency of a configuration from ONE GPU: build every rank's shard of world W exactly as
    make_workload does for that rank and time it alone (HIP events around `steps` launches after `warmup`), then
    the whole workload at world 1.  Strong scaling (configs 4, 5): predicted_efficiency = T₁ / (W · max_R T_R) —
    the slowest rank's filter time sets the step; the collectives are not included (bench.py overlaps step k's
    RCCL all-gather / argmax with step k+1's filter on separate streams).  Weak scaling (configs 2, 3): every rank
    runs a full per-GPU batch, predicted_efficiency = T_rank0 / max_R T_R."""
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = Engine(0)
    eng.precision = {"certified": _lib.PREC_CERTIFIED, "fp64": _lib.PREC_FP64}[args.precision]
    W = args.emulate_world
    ranks = list(range(W)) if args.emulate_rank is None else [args.emulate_rank]
    stream = torch.cuda.Stream(dev)

    def time_shard(w: Workload) -> dict:
        kind = w.kind
        P, B = n_params(kind), w.Theta.shape[1]
        eng.set_panel(w.Y, w.mats)
        d_th = torch.from_numpy(np.ascontiguousarray(w.Theta.T)).to(dev)
        d_tu = torch.from_numpy(w.T_use).to(dev) if w.T_use is not None else None
        d_out = torch.empty(B, dtype=torch.float64, device=dev)

        def launch():
            eng.loglik_device(kind, d_th.data_ptr(), P, B, d_out.data_ptr(), space=0,
                              d_T_use=d_tu.data_ptr() if d_tu is not None else None, stream=stream.cuda_stream)
        t_end = time.perf_counter() + args.settle_seconds
        while time.perf_counter() < t_end:  # the card's steady clock, as the timed region of main()
            launch()
            stream.synchronize()
        for _ in range(args.warmup):
            launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for a, b in ev:
            a.record(stream)
            launch()
            b.record(stream)
        stream.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        Tb = w.T_use if w.T_use is not None else np.full(B, w.Y.shape[1])
        waves = -(-B // 64) if kind != KIND_TVL else None  # fixed loadings: one candidate per lane
        return {"batch": int(B), "filter_steps": int(np.sum(np.asarray(Tb, dtype=np.int64) - 1)),
                "kernel_ms_mean": float(np.mean(ms)), "kernel_ms_min": float(np.min(ms)),
                "waves": waves, "waves_per_simd": waves / 1024.0 if waves else None,
                "logliks_finite": int(torch.isfinite(d_out).sum().item())}

    full = time_shard(make_workload(args.config, 1, 0, args.T, args.batch))
    shards = {r: time_shard(make_workload(args.config, W, r, args.T, args.batch)) for r in ranks}
    w0 = make_workload(args.config, W, 0, args.T, args.batch)
    t_max = max(s["kernel_ms_mean"] for s in shards.values())
    if w0.scaling == "strong":
        pred = full["kernel_ms_mean"] / (W * t_max)
        rule = "T_1 / (W · max_R T_R): the whole workload on one GPU against W× the slowest rank's shard"
    else:
        pred = shards[min(shards)]["kernel_ms_mean"] / t_max
        rule = "weak scaling: every rank a full per-GPU batch; T_rank0 / max_R T_R"
    return {"metric": f"predicted {W}-GPU scaling efficiency (config {args.config}, emulated on one GPU)",
            "config": args.config, "workload": w0.label, "scaling": w0.scaling, "emulated_world": W,
            "world1": full, "ranks": {str(r): s for r, s in shards.items()},
            "max_rank_kernel_ms": t_max,
            "rank_imbalance": t_max / min(s["kernel_ms_mean"] for s in shards.values()),
            "predicted_efficiency": pred, "rule": rule, "steps": args.steps, "warmup": args.warmup,
            "note": "kernel_ms = HIP events around each whole loglik call on its stream (init + filter + deferral "
                    "kernels); collectives excluded (overlapped with the next step's filter in main()); the "
                    "fixed-loading kernels run one wave per SIMD (1,024 per MI355X), so waves_per_simd above an "
                    "integer leaves a partial last round of waves"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--batch", type=int, default=None, help="θ per GPU (2, 3), per window (4), total (5)")
    ap.add_argument("--T", type=int, default=600)
    ap.add_argument("--precision", choices=["certified", "fp64"], default="certified",
                    help="TVλ arithmetic (include/yfm.h yfm_set_precision; the library default is certified)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--settle-seconds", type=float, default=0.5,
                    help="untimed load before the warmup steps so the timed steps run at the card's steady clock")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-rate", action="store_true",
                    help="skip the host-pointer (PCIe-inclusive) timing, e.g. for PMC passes: its chunked "
                         "dispatches would mix into the per-dispatch counter averages")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = host collectives, ranks may share a GPU "
                         "(multi-rank rehearsal on a one-GPU box)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="predict the W-GPU efficiency on one GPU: time every rank's shard of world W alone "
                         "(emulate_world); prints one JSON line and exits")
    ap.add_argument("--emulate-rank", type=int, default=None, help="with --emulate-world: time this rank only")
    args = ap.parse_args()

    if args.emulate_world > 1:
        print(json.dumps(emulate_world(args)), flush=True)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here (this parent never touches the GPU) and exit with their status
        sys.exit(D.spawn_local_ranks(str(Path(__file__).resolve()), sys.argv[1:], args.gpus,
                                     env=dict(os.environ, YFM_LAUNCHER="bench.py --gpus (spawn_local_ranks)")))
    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        gpu = local
    elif world > 1:  # gloo rehearsal: ranks may share GPUs (collectives through host memory)
        gpu = local % torch.cuda.device_count()
        torch.cuda.set_device(gpu)
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
        gpu = 0
    dev = torch.device("cuda", gpu)
    collective_world = 1
    if world > 1:
        # the world size the collectives actually span (RCCL / gloo all-reduce of one per rank)
        one = torch.ones(1, dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(one)
        collective_world = int(one.item())
    if collective_world != args.gpus or world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the job has WORLD_SIZE {world} and the collective spans "
                 f"{collective_world} rank(s)")

    w = make_workload(args.config, world, rank, args.T, args.batch)
    kind = w.kind
    M, P = state_dim(kind), n_params(kind)
    N, T = w.Y.shape
    B = w.Theta.shape[1]
    eng = Engine(dev.index)
    eng.set_panel(w.Y, w.mats)
    PREC = {"certified": _lib.PREC_CERTIFIED, "fp64": _lib.PREC_FP64}
    eng.precision = PREC[args.precision]
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
    # the per-step collectives with every buffer allocated here, once (no per-step torch.full/cat)
    reducer = D.StepReducer(counts, dev) if world > 1 else None
    k_times = []  # (start, end) HIP events around each timed launch, on the launch stream
    # the roofline's kernel time comes from HIP event pairs around every 8th timed launch: a pair around every
    # launch costs ≈ 7.5 µs of wall time per config-2 step (0.1895 vs 0.1820 ms, profiles/r5/events/) — measurement
    # overhead the hot path does not have — while the bracketed launches' mean stays the rocprofv3 kernel duration
    EVENT_EVERY = max(1, int(os.environ.get("YFM_BENCH_EVENT_EVERY", "8")))
    timing = [False]
    it = [0]
    n_timed = [0]  # timed launches so far in this timed region
    best = [None]  # [loglik, global index] of the last step's argmax reduction (N > 1)

    def step():
        i = it[0] % len(outs)
        it[0] += 1
        o = outs[i]
        if world > 1:
            comp.wait_event(c_done[i])  # the collective that last read buffer i has finished
        ev = timing[0] and n_timed[0] % EVENT_EVERY == 0  # the first timed launch always
        n_timed[0] += 1 if timing[0] else 0
        if ev:
            ks, ke = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ks.record(comp)
        eng.loglik_device(kind, d_th.data_ptr(), P, B, o.data_ptr(), space=0,
                          d_T_use=d_tu.data_ptr() if d_tu is not None else None, stream=comp.cuda_stream)
        if ev:
            ke.record(comp)
            k_times.append((ks, ke))
        if world > 1:  # RCCL over xGMI: gather logliks and/or reduce the best candidate
            k_done[i].record(comp)
            stream.wait_event(k_done[i])
            if w.gather:
                reducer.gather(o)
            best[0] = reducer.best(o, offset)
            c_done[i].record(stream)

    settle = {"seconds": 0.0, "steps": 0}

    def settle_clock(seconds):
        """Untimed steps until `seconds` of wall time have passed (before the W warmup steps): the card
        leaves its idle clock only after ~0.1-0.3 s of load, so a short run timed from a cold start
        measures the clock ramp (round 2: 20 steps gave 0.415 ms/step, 200 steps 0.364 ms)."""
        t0 = time.perf_counter()
        for _ in range(4):
            step()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / 4
        if world > 1:  # every rank runs the same number of steps (each one takes part in the collectives)
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        n = min(int(seconds / max(dt, 1e-6)), 20000)
        for _ in range(n):
            step()
        torch.cuda.synchronize(dev)
        settle["seconds"] += time.perf_counter() - t0
        settle["steps"] += n + 4

    def timed(steps, warmup):
        """warmup untimed steps, then `steps` timed ones between barriers; (wall s, mean kernel ms)."""
        k_times.clear()
        n_timed[0] = 0
        for e in c_done:
            e.record(stream)
        if args.settle_seconds > 0:
            settle_clock(args.settle_seconds)
        for _ in range(warmup):
            step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        timing[0] = True
        t0 = time.perf_counter()
        comp.wait_stream(stream)
        for _ in range(steps):
            step()
        stream.wait_stream(comp)
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
        return wall, float(np.mean([ks.elapsed_time(ke) for ks, ke in k_times]))

    wall, kernel_ms = timed(args.steps, args.warmup)
    best_main = best[0]
    # every rank's mean kernel time and its filter steps (Σ (T_use − 1) of its shard): when the ranks' work
    # differs (window shards of config 4, a ragged last shard) the max/min ratio shows the imbalance
    per_rank = None
    if world > 1:
        Tb_r = w.T_use if w.T_use is not None else np.full(B, T)
        mine = torch.tensor([kernel_ms, float(np.sum(np.asarray(Tb_r, dtype=np.float64) - 1)), float(B)],
                            dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        allr = torch.empty(3 * world, dtype=torch.float64, device=mine.device)
        dist.all_gather_into_tensor(allr, mine)
        allr = allr.view(world, 3).cpu().numpy()
        kms = allr[:, 0]
        per_rank = {"per_rank_kernel_ms": [float(x) for x in kms],
                    "per_rank_filter_steps": [int(x) for x in allr[:, 1]],
                    "per_rank_batch": [int(x) for x in allr[:, 2]],
                    "imbalance": float(kms.max() / kms.min()) if kms.min() > 0 else None,
                    "steps_imbalance": float(allr[:, 1].max() / allr[:, 1].min()) if allr[:, 1].min() > 0 else None}
    ms_per_step = 1e3 * wall / args.steps
    value = w.global_batch / (wall / args.steps)
    steady_ws = eng.last_steady() if kind in (KIND_DNS, KIND_GNS) else 0  # frozen-covariance wave-steps of the last launch
    roof = roofline(kind, args.precision, N, M, T, w.T_use, B, P, kernel_ms, steady_lane_steps=64 * steady_ws)
    roof["kernel_ms_source"] = (f"HIP event pairs on the launch stream around every {EVENT_EVERY}th launch of the "
                                  f"timed region ({len(k_times)} of {args.steps}); each pair brackets the whole "
                                  f"loglik call (filter kernel + deferral launch)")
    out_host = d_out.cpu().numpy()
    if os.environ.get("YFM_BENCH_DUMP") and rank == 0:  # A/B runs (tools/ab_run.sh): the logliks, for a bitwise compare
        np.save(os.environ["YFM_BENCH_DUMP"], out_host)
    # DNS, GNS5: the same workload with the full covariance recursion every step (YFM_DNS_STEADY=0), beside the
    # default — the steady state must not change a loglik by more than rounding (tests/test_gpu_steady.py)
    steady = None
    if kind in (KIND_DNS, KIND_GNS):
        Tb = w.T_use if w.T_use is not None else np.full(B, T)
        os.environ["YFM_DNS_STEADY"] = "0"
        try:
            wall_full, kms_full = timed(args.steps, max(1, args.warmup // 2))
            full_host = d_out.cpu().numpy()
        finally:
            os.environ.pop("YFM_DNS_STEADY", None)
        fin = np.isfinite(full_host)
        da = np.abs(out_host[fin] - full_host[fin])
        dr = da / np.abs(full_host[fin])
        worst = None
        if dr.size:
            k = int(np.argmax(dr))
            gi = int(np.flatnonzero(fin)[k])
            worst = {"index": gi, "loglik": float(full_host[gi]), "rel": float(dr[k]), "abs": float(da[k]),
                     "window": int(Tb[gi])}
        steady = {"steady_lane_steps": 64 * steady_ws, "frac_of_filter_steps": 64 * steady_ws / float(np.sum(Tb - 1)),
                  "full_recursion_evals_per_s": w.global_batch / (wall_full / args.steps),
                  "full_recursion_kernel_ms": kms_full,
                  "vs_full_recursion_max_rel": float(dr.max()) if dr.size else 0.0,
                  "vs_full_recursion_max_abs": float(da.max()) if da.size else 0.0,
                  "vs_full_recursion_worst": worst,
                  "vs_full_recursion_max_rel_abs_ll_ge_1": float(dr[np.abs(full_host[fin]) >= 1.0].max())
                  if np.any(np.abs(full_host[fin]) >= 1.0) else 0.0,
                  "pattern_match": bool(np.array_equal(np.isfinite(out_host), fin)),
                  "note": "the covariance recursion of filter.jl:158-176 is data-independent for fixed loadings; each "
                          "candidate freezes P once its change per step is at the rounding level (a step set by its "
                          "own θ), a wave whose candidates are all frozen runs the mean update only "
                          "(DESIGN.md §3.1; YFM_DNS_STEADY=0 disables it).  The relative change is against |loglik|: "
                          "a loglik near 0 (a sum of ~10^4-sized terms that cancels) shows a large relative change "
                          "for a rounding-sized absolute one — see vs_full_recursion_worst and the |ll| ≥ 1 column"}
    n_neginf, n_nan = int(np.isneginf(out_host).sum()), int(np.isnan(out_host).sum())
    n_deferred = eng.last_deferred()  # candidates of the last timed batch on the double-double path

    # TVλ: the FP64 mode of the same workload beside the certified default (not the metric's value)
    fp64_mode = None
    if kind == KIND_TVL and args.precision == "certified":
        eng.precision = _lib.PREC_FP64
        wall64, kms64 = timed(args.steps, max(1, args.warmup // 2))
        f64_host = d_out.cpu().numpy()
        eng.precision = PREC[args.precision]
        fin = np.isfinite(out_host)
        d64 = np.abs(f64_host[fin] - out_host[fin]) / np.abs(out_host[fin])
        fp64_mode = {"evals_per_s": w.global_batch / (wall64 / args.steps), "ms_per_step": 1e3 * wall64 / args.steps,
                     "roofline": roofline(kind, "fp64", N, M, T, w.T_use, B, P, kms64),
                     "vs_certified": {"frac_within_1e-9": float(np.mean(d64 <= 1e-9)), "max_rel": float(d64.max()),
                                      "pattern_match": bool(np.array_equal(np.isfinite(f64_host), fin))}}

    # host-pointer boundary (yfm_loglik_batch: θ in over PCIe, logliks back, synchronous) —
    # reported beside the metric, never as `value` (inputs are not HBM-resident there)
    host_rate = None
    if rank == 0 and world == 1 and not args.no_host_rate:
        Th_host = np.asfortranarray(w.Theta)
        tu_host = w.T_use
        eng.loglik(kind, Th_host, space=0, T_use=tu_host)
        reps = max(3, min(args.steps, 10))
        th0 = time.perf_counter()
        for _ in range(reps):
            eng.loglik(kind, Th_host, space=0, T_use=tu_host)
        host_s = (time.perf_counter() - th0) / reps
        # the same with θ and the logliks in page-locked memory (yfm_alloc_host)
        th_pin = eng.host_array(Th_host.shape)
        th_pin[...] = Th_host
        out_pin = eng.host_array((B,))
        eng.loglik(kind, th_pin, space=0, T_use=tu_host, out=out_pin)
        th0 = time.perf_counter()
        for _ in range(reps):
            eng.loglik(kind, th_pin, space=0, T_use=tu_host, out=out_pin)
        pin_s = (time.perf_counter() - th0) / reps
        host_rate = {"evals_per_s": B / host_s, "ms_per_call": 1e3 * host_s, "calls": reps,
                     "pinned_evals_per_s": B / pin_s, "pinned_ms_per_call": 1e3 * pin_s,
                     "note": "yfm_loglik_batch with host θ / host logliks (H2D + kernel + D2H, synchronous); "
                             "pinned_* with both in yfm_alloc_host memory"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(w, args.cpu_seconds, out_host)
        ro1 = cpu["optimised"].get("evals_per_s_1_thread")
        cpu["gpu_over_cpu"] = {"dense_port": value / cpu["value"],
                               "optimised": value / cpu["optimised"]["evals_per_s"],
                               "optimised_1_thread": value / ro1 if ro1 else None,
                               "optimised_extrapolated_all_physical_cores":
                                   (value / cpu["optimised"]["extrapolated_all_physical_cores"]
                                    if cpu["optimised"]["extrapolated_all_physical_cores"] else None)}

    if rank == 0:
        line = {
            "metric": METRIC if args.config == 2 else f"Kalman loglik evals/sec (config {args.config})",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "collective_world_size": collective_world,
            "launcher": os.environ.get("YFM_LAUNCHER", "torchrun" if world > 1 else "single"),
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_settle": {"seconds": round(settle["seconds"], 3), "steps": settle["steps"],
                             "note": "untimed steps before the warmup (--settle-seconds)"},
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": w.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (model-simulated panel, seeded θ batch)",
            "config": {"workload": w.label, "kind": {KIND_DNS: "DNS (1C)", KIND_TVL: "TVλ (EKF)",
                                                      KIND_GNS: "GNS5 (extension)"}[kind],
                       "T": T, "N": N, "batch_per_gpu": B, "global_batch": w.global_batch,
                       "precision": ("certified (double-double)" if args.precision == "certified" else "fp64")
                       if kind == KIND_TVL else "fp64",
                       "parallelism": f"dp{world} (θ sharded, RCCL "
                                      f"{'all-gather of logliks + ' if w.gather else ''}argmax)", **w.extra},
            "roofline": roof,
            "cpu_baseline": cpu,
            "host_pointer_rate": host_rate,
            "outputs": {"neg_inf": n_neginf, "nan": n_nan, "deferred_double_double": n_deferred},
        }
        if per_rank:
            line.update(per_rank)
        if fp64_mode:
            if cpu and cpu["optimised"].get("evals_per_s_1_thread"):
                # the FP64 mode against the optimised CPU filter, which computes in FP64 too
                ro1 = cpu["optimised"]["evals_per_s_1_thread"]
                fp64_mode["gpu_over_cpu"] = {"optimised": fp64_mode["evals_per_s"] / cpu["optimised"]["evals_per_s"],
                                             "optimised_1_thread": fp64_mode["evals_per_s"] / ro1}
            line["fp64_mode"] = fp64_mode
        if steady:
            line["steady_state"] = steady
        if best_main is not None:
            line["best_candidate"] = {"loglik": float(best_main[0].item()), "index": int(best_main[1].item())}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
