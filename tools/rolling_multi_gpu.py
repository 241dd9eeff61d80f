"""Rolling re-estimation over one process per GPU (config 4's driver, forecasting.jl:81-224):

    torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/rolling_multi_gpu.py [--windows 240]

Every rank takes a load-balanced share of the 240 expanding-window estimation chains
(yfm_amd.distributed.balanced_window_assignment), runs them as one batched yfm_estimate on its GPU,
and the per-window results are all-gathered over RCCL.  Rank 0 prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yieldfactormodels.jl_amd"))

from yfm_amd import KIND_DNS, Engine  # noqa: E402
from yfm_amd import distributed as D  # noqa: E402
from yfm_amd import synthetic as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=240)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    mats = S.maturities_30()
    Y = S.simulate_panel(KIND_DNS, 600)
    wins = np.arange(601 - args.windows, 601, dtype=np.int32)
    Th0 = np.repeat(S.theta0_constrained(KIND_DNS)[:, None], len(wins), axis=1)
    eng = Engine(local)
    eng.set_panel(Y, mats)

    def estimate(Th, tu):
        return eng.estimate(KIND_DNS, Th, space=1, T_use=tu)

    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    r = D.sharded_estimate(Th0, wins, estimate, device=torch.device("cuda", local)) if world > 1 else estimate(Th0, wins)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"metric": "rolling re-estimation windows/s", "value": len(wins) / dt, "n_gpus": world,
                          "seconds": dt, "windows": int(len(wins)), "mean_ll": float(np.mean(r["ll"]))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
