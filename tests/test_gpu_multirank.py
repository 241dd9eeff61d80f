"""Multi-rank paths with the HIP library in every rank, on one GPU (the pool's boxes have one;
the 8-GPU RCCL run is the driver's): two processes share cuda:0 and talk through gloo.  The
code under test is the production path — bench.py's double-buffered step with the kernel on a
compute stream and the collectives ordered by events, and the sharded rolling re-estimation
with rank-0 CSV output — only the transport differs from RCCL (yfm_amd.distributed._comm_device)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_argmax(engine):
    """torchrun --nproc-per-node 2 bench.py --config 5 (strong scaling: each rank evaluates half of
    the candidates, the logliks are reduced to the global argmax): the reported best candidate is
    the host argmax of a single-process evaluation of all candidates."""
    from yfm_amd import KIND_GNS
    from yfm_amd import synthetic as S
    B = 8192
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"), "--gpus", "2",
           "--config", "5", "--batch", str(B), "--T", "120", "--steps", "4", "--warmup", "1", "--no-cpu-baseline",
           "--dist-backend", "gloo"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == B and line["value"] > 0
    Y = S.simulate_panel(KIND_GNS, 120)
    Th = S.theta_range(KIND_GNS, 0, B, scale=0.1)  # the bench's global candidate stream
    engine.set_panel(Y, S.maturities_30())
    ll = np.nan_to_num(engine.loglik(KIND_GNS, Th), nan=-np.inf)
    assert line["best_candidate"]["index"] == int(np.argmax(ll))
    assert line["best_candidate"]["loglik"] == ll.max()


def test_bench_self_launches_n_ranks():
    """`python bench.py --gpus 2` with no launcher (the driver's command shape): bench.py starts the two
    ranks itself (yfm_amd.distributed.spawn_local_ranks), both share cuda:0 over gloo, and the line
    reports the two-rank job — n_gpus 2, the collective's world size 2, the global batch of both ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "2", "--batch", "4096", "--T", "120",
           "--steps", "3", "--warmup", "1", "--settle-seconds", "0", "--no-cpu-baseline", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = lines[0]
    print({k: line[k] for k in ("n_gpus", "collective_world_size", "launcher", "value", "per_rank_kernel_ms",
                                "imbalance", "per_rank_filter_steps")})
    assert line["n_gpus"] == 2 and line["collective_world_size"] == 2
    assert len(line["per_rank_kernel_ms"]) == 2 and min(line["per_rank_kernel_ms"]) > 0 and line["imbalance"] >= 1.0
    assert line["per_rank_filter_steps"] == [4096 * 119] * 2
    assert line["config"]["global_batch"] == 2 * 4096 and "spawn_local_ranks" in line["launcher"]


@pytest.mark.parametrize("config", [4, 5])
def test_bench_emulate_world(config):
    """`bench.py --emulate-world 4` (the one-GPU prediction of the strong-scaled configurations' N-GPU
    efficiency): every rank's shard is timed, the shards are the ranks' own (their batches add up to the whole
    job), and the prediction is T₁ / (W · max_R T_R), a number in (0, 1.2]."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--config", str(config), "--batch", "512" if config == 4 else "65536",
           "--T", "120", "--emulate-world", "4", "--steps", "3", "--warmup", "1", "--settle-seconds", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print({k: line[k] for k in ("predicted_efficiency", "max_rank_kernel_ms", "rank_imbalance")})
    assert sorted(line["ranks"]) == ["0", "1", "2", "3"]
    assert sum(s["batch"] for s in line["ranks"].values()) == line["world1"]["batch"]
    assert sum(s["filter_steps"] for s in line["ranks"].values()) == line["world1"]["filter_steps"]
    t1, tmax = line["world1"]["kernel_ms_mean"], line["max_rank_kernel_ms"]
    assert abs(line["predicted_efficiency"] - t1 / (4 * tmax)) < 1e-12
    assert 0.0 < line["predicted_efficiency"] <= 1.2


def _rolling_worker(rank, world, port, Y, mats, out_dir, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch  # noqa: F401
    import torch.distributed as dist
    sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]
    from yfm_amd import create_model
    from yfm_amd import synthetic as S
    from yfm_amd.forecasting import run_rolling_forecasts
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model, _ = create_model("1C", mats, 30, results_location=out_dir + "/")
    th0 = S.theta0_constrained(0)
    out = run_rolling_forecasts(model, Y, "7", 50, 11, 3, th0[:, None], window_type="both", max_group_iters=1,
                                iterations=20, group=dist.group.WORLD)
    ret[rank] = {wt: {k: v for k, v in res.items() if isinstance(v, np.ndarray)} for wt, res in out.items()}
    dist.barrier()
    dist.destroy_process_group()


def _driver_worker(rank, world, port, root, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch  # noqa: F401
    import torch.distributed as dist
    sys.path[:0] = [str(ROOT), str(ROOT / "yieldfactormodels.jl_amd")]
    import yfm_amd
    os.chdir(root)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = yfm_amd.run("7", 44, 2, True, "1C", window_type="expanding", max_group_iters=1, iterations=20,
                        seed=5, group=dist.group.WORLD)
    info = model.last_run
    ret[rank] = {"params": np.asarray(info["params"]), "files": list(info["files"]),
                 "rolling": sorted(info.get("rolling", {}).keys())}
    dist.barrier()
    dist.destroy_process_group()


def _driver_inputs(root, Y, mats):
    from yfm_amd import io as yio
    d = root / "YieldFactorModels.jl" / "data"
    d.mkdir(parents=True)
    yio.writedlm(d / "thread_id__7__data.csv", Y)
    yio.writedlm(d / "thread_id__7__maturities.csv", mats)


def _tree(root):
    return sorted(str(p.relative_to(root)) for p in root.rglob("*.csv"))


def test_run_driver_two_ranks(engine, tmp_path):
    """yfm_amd.run(group=…) with a MISSING init file on 2 ranks.  Rank 0 alone writes the random
    start (broadcast to rank 1) and every result file; the CSV tree is exactly the single-process run's."""
    from yfm_amd import io as yio
    from yfm_amd import synthetic as S
    import yfm_amd
    mats = S.maturities_30()
    Y = S.simulate_panel(0, 600)[:, :50].copy(order="F")
    two, one = tmp_path / "two", tmp_path / "one"
    for d in (two, one):
        _driver_inputs(d, Y, mats)
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_driver_worker, args=(2, _free_port(), str(two), ret), nprocs=2, join=True)
    np.testing.assert_array_equal(ret[0]["params"], ret[1]["params"])  # the same start and estimate
    assert ret[1]["files"] == [] and ret[1]["rolling"] == [] and ret[0]["files"]
    cwd = os.getcwd()
    os.chdir(one)
    try:
        model = yfm_amd.run("7", 44, 2, True, "1C", window_type="expanding", max_group_iters=1, iterations=20, seed=5)
    finally:
        os.chdir(cwd)
    np.testing.assert_array_equal(model.last_run["params"], ret[0]["params"])
    files = _tree(two)
    assert files == _tree(one) and any("init_params_1C.csv" in f for f in files)
    assert any("expanding_window_forecasts" in f for f in files)
    for name in files:
        np.testing.assert_array_equal(yio.readdlm(two / name), yio.readdlm(one / name), err_msg=name)


def test_rolling_forecasts_two_ranks(engine, tmp_path):
    """run_rolling_forecasts with a 2-rank group: the estimation chains split over the ranks give
    exactly the single-process results, and only rank 0 predicts and writes the CSVs."""
    from yfm_amd import create_model
    from yfm_amd import io as yio
    from yfm_amd import synthetic as S
    from yfm_amd.forecasting import run_rolling_forecasts
    mats = S.maturities_30()
    Y = S.simulate_panel(0, 600)[:, :56].copy(order="F")
    mgr = mp.Manager()
    ret = mgr.dict()
    d2 = tmp_path / "two"
    d2.mkdir()
    mp.spawn(_rolling_worker, args=(2, _free_port(), Y, mats, str(d2), ret), nprocs=2, join=True)
    assert ret[1] == {}
    d1 = tmp_path / "one"
    d1.mkdir()
    model, _ = create_model("1C", mats, 30, results_location=str(d1) + "/")
    one = run_rolling_forecasts(model, Y, "7", 50, 11, 3, S.theta0_constrained(0)[:, None], window_type="both",
                                max_group_iters=1, iterations=20)
    for wt in ("expanding", "moving"):
        for k, v in ret[0][wt].items():
            np.testing.assert_array_equal(v, one[wt][k], err_msg=(wt, k))
    files = sorted(p.name for p in d2.iterdir())
    assert files == sorted(p.name for p in d1.iterdir()) and len(files) >= 12
    for name in files:
        np.testing.assert_array_equal(yio.readdlm(d2 / name), yio.readdlm(d1 / name))
