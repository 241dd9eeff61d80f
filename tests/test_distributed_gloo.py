"""Multi-process (world_size 2, gloo, CPU) tests of the sharding / gather / argmax logic.

The per-rank compute here is the NumPy oracle (test infrastructure); on GPUs the
same code runs with the HIP library per rank and the nccl (RCCL) backend (bench.py)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from yfm_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 65536, 65537):
        for w in (1, 2, 3, 8):
            parts = [D.shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [h - l for l, h in parts]
            assert max(sizes) - min(sizes) <= 1


def test_window_shards_cover_and_balance():
    counts = [5, 8, 3, 4096]
    for w in (2, 3, 8):
        allidx = np.sort(np.concatenate([D.window_shards(counts, w, r) for r in range(w)]))
        np.testing.assert_array_equal(allidx, np.arange(sum(counts)))
        per = [len(D.window_shards(counts, w, r)) for r in range(w)]
        assert max(per) - min(per) <= len(counts)


def _steps_worker(rank, world, port, ret):
    """bench.py's config-4 shard on this rank: Σ (T_use − 1) over its candidates, all-gathered as bench.py does."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wins = np.arange(361, 601)
    per = 4096
    counts = [per] * len(wins)
    idx = D.window_shards(counts, world, rank)
    tu = np.repeat(wins, per)[idx]
    mine = torch.tensor([float(np.sum(tu - 1)), float(len(idx))], dtype=torch.float64)
    allr = torch.empty(2 * world, dtype=torch.float64)
    dist.all_gather_into_tensor(allr, mine)
    if rank == 0:
        ret["steps"] = allr.view(world, 2)[:, 0].numpy().copy()
        ret["n"] = allr.view(world, 2)[:, 1].numpy().copy()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_window_shards_equal_filter_steps(world):
    """config 4's window shards give every rank the same Σ T_use (its filter steps, which
    set its kernel time) to within one window's share — the longest window's steps once per window whose
    4,096 candidates do not split evenly."""
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_steps_worker, args=(world, _free_port(), ret), nprocs=world, join=True)
    steps, n = ret["steps"], ret["n"]
    assert n.sum() == 240 * 4096
    if 4096 % world == 0:  # every window splits evenly: identical work per rank
        assert steps.max() == steps.min()
    # otherwise at most one window's per-rank share of filter steps apart
    share = 4096 / world * 599
    assert steps.max() - steps.min() <= share, (steps, share)
    print(f"world {world}: per-rank filter steps {steps}, max/min {steps.max() / steps.min():.6f}")


def _worker(rank, world, port, Theta, Y, mats, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import kalman_oracle as O

    def evaluate(Th):
        return torch.tensor([O.loglik(0, mats, 3, Y, Th[:, b]) for b in range(Th.shape[1])], dtype=torch.float64)

    res = D.sharded_loglik(Theta, evaluate)
    if rank == 0:
        ret["ll"] = res.loglik.numpy()
        ret["best"] = (res.best_index, res.best_value)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_equals_single_process(world):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from oracle import kalman_oracle as O
    from yfm_amd import synthetic as S
    Y = S.simulate_panel(0, 40)
    mats = S.maturities_30()
    Theta = S.theta_batch(0, 7, seed=3, bad_frac=0.0)
    Theta[:, 4] = S.theta0(0)
    ref = np.array([O.loglik(0, mats, 3, Y, Theta[:, b]) for b in range(7)])
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), Theta, Y, mats, ret), nprocs=world, join=True)
    np.testing.assert_array_equal(ret["ll"], ref)
    assert ret["best"][0] == int(np.argmax(ref)) and ret["best"][1] == ref.max()


def _argmax_worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank 0: [1, NaN, 5], rank 1: [5, 2] — the global maximum 5 is tied: lowest global index (2) wins
    local = torch.tensor([[1.0, float("nan"), 5.0], [5.0, 2.0]][rank], dtype=torch.float64)
    offset = [0, 3][rank]
    dev = D.best_candidate_device(local, offset)
    host = D.best_candidate(local, offset)
    allv = D.gather_logliks(local, [3, 2])
    red = D.StepReducer([3, 2], local.device)  # bench.py's preallocated per-step form
    steps = [(red.gather(local).clone(), red.best(local, offset).clone()) for _ in range(3)]
    if rank == 0:
        ret["dev"] = dev.tolist()
        ret["host"] = host
        ret["all"] = allv.tolist()
        ret["red"] = [(g.tolist(), b.tolist()) for g, b in steps]
    dist.barrier()
    dist.destroy_process_group()


def test_argmax_reduce_ties_nan_and_ragged_gather():
    """The bench's device-side argmax (yfm_amd.distributed.best_candidate_device) and the host
    reduce agree: NaN (init throw) never wins, ties go to the lowest global index; the ragged
    all-gather returns every rank's logliks in global order."""
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_argmax_worker, args=(2, _free_port(), ret), nprocs=2, join=True)
    assert ret["dev"] == [5.0, 2.0] and ret["host"] == (2, 5.0)
    assert np.array_equal(np.array(ret["all"]), np.array([1.0, np.nan, 5.0, 5.0, 2.0]), equal_nan=True)
    for g, b in ret["red"]:  # StepReducer: the same results on every step from its persistent buffers
        assert np.array_equal(np.array(g), np.array(ret["all"]), equal_nan=True) and b == [5.0, 2.0]


@pytest.mark.parametrize("config", [4, 5])
def test_bench_sharding_covers_every_unit_once(config):
    """bench.py's per-rank workloads (configs 4 and 5, strong scaling) partition the global job:
    every (window, θ) pair / candidate is evaluated by exactly one of N ranks, N = 1, 2, 4, 8."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    import bench
    for world in (1, 2, 4, 8):
        seen = []
        sizes = []
        for rank in range(world):
            w = bench.make_workload(config, world, rank, 60, 16)
            sizes.append(w.Theta.shape[1])
            if config == 4:
                # (window length, θ column) pairs; θ columns repeat the same 16 starts per window
                seen += list(zip(w.T_use.tolist(), map(tuple, np.round(w.Theta.T, 12).tolist())))
            else:
                seen += list(range(w.extra["offset"], w.extra["offset"] + w.Theta.shape[1]))
        assert len(seen) == len(set(seen)) == w.global_batch
        assert max(sizes) - min(sizes) <= (60 if config == 4 else 1)


def test_balanced_window_assignment():
    T_use = np.arange(361, 601)
    for world in (1, 2, 4, 8):
        parts = D.balanced_window_assignment(T_use, world)
        allidx = np.sort(np.concatenate(parts))
        np.testing.assert_array_equal(allidx, np.arange(len(T_use)))
        loads = [T_use[p].sum() for p in parts]
        assert max(loads) - min(loads) <= T_use.max()


def _estimate_worker(rank, world, port, Theta0, T_use, Y, mats, ret):
    """Each rank runs its chains on the CPU restatement (oracle/optim_nm.py over the NumPy oracle)
    — the collective pattern is the one the GPU path uses."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import math
    from oracle import kalman_oracle as O
    from oracle import optim_nm as NM
    from yfm_amd.params import transform_params, untransform_params

    def estimate(Th, tu):
        out = dict(theta_c=np.empty_like(Th), ll=np.empty(Th.shape[1]), status=np.zeros(Th.shape[1], np.int32))
        for b in range(Th.shape[1]):
            def f(th, b=b):
                v = O.loglik(0, mats, 3, Y[:, :tu[b]], th)
                if math.isnan(v):
                    raise NM.InitThrow()
                return -v
            r = NM.estimate_steps(f, Th[:, b], transform=lambda x: transform_params(0, x),
                                  untransform=lambda x: untransform_params(0, x), max_group_iters=1, iterations=6)
            out["theta_c"][:, b], out["ll"][b], out["status"][b] = r.theta_c, r.ll, r.status
        return out

    res = D.sharded_estimate(Theta0, T_use, estimate)
    if rank == 0:
        ret["theta_c"] = res["theta_c"]
        ret["ll"] = res["ll"]
        single = estimate(Theta0, T_use)
        ret["single_theta_c"] = single["theta_c"]
        ret["single_ll"] = single["ll"]
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_estimate_equals_single_process():
    """The distributed rolling re-estimation (yfm_amd.distributed.sharded_estimate) returns, on every
    rank, exactly the per-window results a single process computes (chains are independent)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    from yfm_amd import synthetic as S
    Y = S.simulate_panel(0, 30)
    mats = S.maturities_30()
    T_use = np.array([30, 12, 25, 20, 8], dtype=np.int32)
    Theta0 = np.repeat(S.theta0_constrained(0)[:, None], 5, axis=1)
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_estimate_worker, args=(2, _free_port(), Theta0, T_use, Y, mats, ret), nprocs=2, join=True)
    np.testing.assert_array_equal(ret["theta_c"], ret["single_theta_c"])
    np.testing.assert_array_equal(ret["ll"], ret["single_ll"])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_config5_shards_are_the_single_gpu_candidates(world):
    """Strong scaling evaluates the same job at every world size: the rank shards of bench config 5,
    concatenated in rank order, are exactly the single-GPU candidate matrix (candidate b depends
    only on (seed, b): yfm_amd.synthetic.theta_range)."""
    import bench
    one = bench.make_workload(5, 1, 0, 30, 5000).Theta
    parts = [bench.make_workload(5, world, r, 30, 5000).Theta for r in range(world)]
    np.testing.assert_array_equal(np.hstack(parts), one)


def test_theta_range_blocks_are_consistent():
    from yfm_amd import synthetic as S
    full = S.theta_range(2, 0, 2 * S.RANGE_BLOCK + 10)
    np.testing.assert_array_equal(S.theta_range(2, S.RANGE_BLOCK - 3, S.RANGE_BLOCK + 7),
                                  full[:, S.RANGE_BLOCK - 3:S.RANGE_BLOCK + 7])
