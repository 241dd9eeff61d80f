"""Multi-GPU sharding of batched loglik evaluations (one process per GPU).

The reference distributes work only across independent Julia processes that
claim forecast origins through mkdir locks (`src/forecasting.jl:54-79`); there
is no in-filter exchange.  Here every (θ, window) evaluation is independent, so a
batch is split into contiguous per-rank shards with no data-path collective; the
only collectives are

* ``all_gather`` of the per-candidate logliks (RCCL over xGMI with the ``nccl``
  backend; gloo on CPU for tests), and
* an argmax reduction of the best candidate — RCCL has no argmax, so each rank
  contributes (best loglik, global index) and the pairs are all-gathered.

For expanding windows (config 4) the split is *within* each window
(`window_shards`): every rank gets an equal slice of every window's candidates,
which balances the T_use-dependent cost that a split by window would not.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch
import torch.distributed as dist


def free_port(host: str = "127.0.0.1") -> int:
    """An unused TCP port on `host` for a local rendezvous (MASTER_PORT)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def spawn_local_ranks(script: str, argv: list[str], nprocs: int, env: dict | None = None,
                      timeout: float | None = None) -> int:
    """Run `python script argv…` as `nprocs` ranks of one job on this node, the way
    `torch.distributed.run --nnodes=1 --nproc-per-node nprocs --master-addr 127.0.0.1` would: each child
    gets RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = nprocs, MASTER_ADDR = 127.0.0.1 and a free
    MASTER_PORT, and selects its GPU from LOCAL_RANK itself.  The children are fresh processes started
    by a parent that must not have initialised the GPU (it only waits); stdout/stderr pass through.
    Returns 0 when every rank exits 0, else the first non-zero exit status (ranks still running after
    a failure are terminated, so a rank stuck in a collective cannot hang the job)."""
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(nprocs),
                LOCAL_WORLD_SIZE=str(nprocs))
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=e))
    rc = 0
    deadline = None if timeout is None else time.monotonic() + timeout
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                try:
                    code = p.wait(timeout=0.2 / len(pending))
                except subprocess.TimeoutExpired:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:
                        q.terminate()
            if deadline is not None and pending and time.monotonic() >= deadline:
                for q in pending:
                    q.kill()
                return rc or 124
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) of n items for `rank` (sizes differ by at most 1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def window_shards(counts, world: int, rank: int) -> np.ndarray:
    """Global indices this rank evaluates when window w owns `counts[w]` consecutive candidates:
    the rank's balanced slice of every window, concatenated in window order."""
    idx = []
    off = 0
    for c in counts:
        lo, hi = shard_range(int(c), world, rank)
        idx.append(np.arange(off + lo, off + hi))
        off += int(c)
    return np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)


@dataclass
class GatherResult:
    loglik: torch.Tensor  # all candidates, global order
    best_index: int
    best_value: float


def _comm_device(group, device) -> torch.device:
    """Where a collective's buffers live: the tensors' own device for nccl (RCCL over xGMI), the
    host for gloo (CPU tests, and multi-rank rehearsals that share one GPU)."""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else device


def gather_logliks(local: torch.Tensor, counts: list[int], group=None) -> torch.Tensor:
    """All-gather per-rank loglik vectors of (possibly unequal) `counts` into global rank order."""
    world = dist.get_world_size(group)
    m = max(counts)
    cdev = _comm_device(group, local.device)
    buf = torch.full((m,), float("nan"), dtype=local.dtype, device=cdev)
    buf[: local.numel()] = local.to(cdev)
    out = torch.empty(world * m, dtype=local.dtype, device=cdev)
    dist.all_gather_into_tensor(out, buf, group=group)
    return torch.cat([out[r * m: r * m + counts[r]] for r in range(world)]).to(local.device)


def best_candidate(local: torch.Tensor, global_offset: int, group=None) -> tuple[int, float]:
    """Global argmax of loglik over all ranks (NaN treated as -inf; ties → lowest global index)."""
    v = torch.nan_to_num(local, nan=-float("inf"))
    if v.numel():
        i = int(torch.argmax(v).item())
        pair = torch.tensor([float(v[i].item()), float(global_offset + i)], dtype=torch.float64, device=local.device)
    else:
        pair = torch.tensor([-float("inf"), float("inf")], dtype=torch.float64, device=local.device)
    world = dist.get_world_size(group)
    cdev = _comm_device(group, local.device)
    allp = torch.empty(2 * world, dtype=torch.float64, device=cdev)
    dist.all_gather_into_tensor(allp, pair.to(cdev), group=group)
    allp = allp.view(world, 2).cpu().numpy()
    best = max(range(world), key=lambda r: (allp[r, 0], -allp[r, 1]))
    return int(allp[best, 1]), float(allp[best, 0])


def best_candidate_device(local: torch.Tensor, global_offset: int, group=None) -> torch.Tensor:
    """Same reduction as `best_candidate` without a host round trip (for timed loops): returns a
    device tensor [best loglik, global index].  Every rank contributes (max, its global index);
    one all-gather of 16 B per rank; the first maximal pair in rank order wins (lowest index)."""
    if local.numel():
        v = torch.nan_to_num(local, nan=-float("inf"))
        i = torch.argmax(v)
        pair = torch.stack([v[i], (i + global_offset).to(torch.float64)])
    else:  # an empty shard (B < world size) still takes part in the all-gather
        pair = torch.tensor([-float("inf"), float("inf")], dtype=torch.float64, device=local.device)
    world = dist.get_world_size(group)
    cdev = _comm_device(group, local.device)
    allp = torch.empty(2 * world, dtype=torch.float64, device=cdev)
    dist.all_gather_into_tensor(allp, pair.to(cdev), group=group)
    allp = allp.view(world, 2)
    r = torch.argmax(allp[:, 0])
    return allp[r].to(local.device)


class StepReducer:
    """The per-step collectives of a timed loop (bench.py, N > 1) with every buffer allocated once:
    the all-gather of this rank's logliks (ragged `counts` allowed) and the argmax reduction of
    `best_candidate_device`, both on the current stream, with no per-step tensor allocation
    (`gather_logliks` / `best_candidate_device` allocate and concatenate on every call).

    gather(local) returns the global loglik vector (a view into a persistent buffer, overwritten by
    the next call); best(local, global_offset) returns the device tensor [best loglik, global index]
    (also persistent)."""

    def __init__(self, counts: list[int], device: torch.device, dtype=torch.float64, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.counts = [int(c) for c in counts]
        self.m = max(self.counts) if self.counts else 0
        cdev = _comm_device(group, device)
        self.cdev, self.device = cdev, device
        self.equal = all(c == self.m for c in self.counts)
        n_local = self.counts[self.rank]
        # send buffer: only for ragged counts (the pad tail stays NaN) or a host-staged backend
        self.send = None
        if not self.equal or cdev != device:
            self.send = torch.full((self.m,), float("nan"), dtype=dtype, device=cdev)
        self.recv = torch.empty(self.world * self.m, dtype=dtype, device=cdev)
        self.glob = self.recv if self.equal and cdev == device else torch.empty(sum(self.counts), dtype=dtype,
                                                                              device=device)
        self._slices = []
        off = 0
        for r, c in enumerate(self.counts):
            self._slices.append((self.recv[r * self.m: r * self.m + c], self.glob[off: off + c]))
            off += c
        self.n_local = n_local
        # argmax buffers
        self.v = torch.empty(max(n_local, 1), dtype=dtype, device=device)
        self.vmax = torch.empty((), dtype=dtype, device=device)
        self.imax = torch.empty((), dtype=torch.int64, device=device)
        self.pair = torch.empty(2, dtype=dtype, device=device)
        self.pair_c = self.pair if cdev == device else torch.empty(2, dtype=dtype, device=cdev)
        self.allp = torch.empty(2 * self.world, dtype=dtype, device=cdev)
        self.rmax = torch.empty((), dtype=dtype, device=cdev)
        self.rarg = torch.empty((), dtype=torch.int64, device=cdev)
        self.sel = torch.empty((1, 2), dtype=dtype, device=cdev)
        self.out = torch.empty(2, dtype=dtype, device=device)

    def gather(self, local: torch.Tensor) -> torch.Tensor:
        src = local
        if self.send is not None:
            self.send[: self.n_local].copy_(local)
            src = self.send
        dist.all_gather_into_tensor(self.recv, src, group=self.group)
        if self.glob is not self.recv:
            for a, b in self._slices:
                b.copy_(a)
        return self.glob

    def best(self, local: torch.Tensor, global_offset: int) -> torch.Tensor:
        if self.n_local:
            torch.nan_to_num(local, nan=-float("inf"), out=self.v)
            torch.max(self.v, 0, out=(self.vmax, self.imax))
            self.pair[0].copy_(self.vmax)
            self.pair[1].copy_(self.imax)
            self.pair[1].add_(float(global_offset))
        else:  # an empty shard (B < world size) still takes part in the all-gather
            self.pair[0].fill_(-float("inf"))
            self.pair[1].fill_(float("inf"))
        if self.pair_c is not self.pair:
            self.pair_c.copy_(self.pair)
        dist.all_gather_into_tensor(self.allp, self.pair_c, group=self.group)
        ap = self.allp.view(self.world, 2)
        torch.max(ap[:, 0], 0, out=(self.rmax, self.rarg))  # first maximal rank (lowest global index)
        torch.index_select(ap, 0, self.rarg.view(1), out=self.sel)
        self.out.copy_(self.sel.view(2))
        return self.out


def sharded_loglik(Theta: np.ndarray, evaluate: Callable[[np.ndarray], torch.Tensor], group=None,
                   device=None) -> GatherResult:
    """Evaluate Θ (P×B, identical on every rank) sharded over the group: rank r evaluates its
    contiguous block with `evaluate` (a rank-local callable returning a tensor of logliks), then
    the logliks are all-gathered and the best candidate reduced."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    B = Theta.shape[1]
    lo, hi = shard_range(B, world, rank)
    local = evaluate(np.asfortranarray(Theta[:, lo:hi]))
    if device is not None:
        local = local.to(device)
    counts = [shard_range(B, world, r)[1] - shard_range(B, world, r)[0] for r in range(world)]
    allv = gather_logliks(local, counts, group)
    bi, bv = best_candidate(local, lo, group)
    return GatherResult(allv, bi, bv)


def balanced_window_assignment(T_use, world: int) -> list[np.ndarray]:
    """Assign estimation chains (one per window, cost ∝ window length) to ranks: longest first onto
    the least-loaded rank (LPT), so every rank gets about the same number of filter steps.  Returns
    each rank's chain indices in ascending order (deterministic on every rank)."""
    T_use = np.asarray(T_use, dtype=np.int64)
    load = np.zeros(world)
    parts = [[] for _ in range(world)]
    for i in np.argsort(-T_use, kind="stable"):
        r = int(np.argmin(load))
        parts[r].append(int(i))
        load[r] += T_use[i]
    return [np.array(sorted(p), dtype=np.int64) for p in parts]


def sharded_estimate(Theta0: np.ndarray, T_use, estimate: Callable, group=None, device=None) -> dict:
    """Distributed batched estimate_steps!: the R chains (columns of Θ₀, windows T_use) are split
    over the ranks by `balanced_window_assignment`; each rank runs `estimate(Θ₀_shard, T_use_shard)`
    (a rank-local callable returning dict(theta_c P×r, ll r, status r), e.g. Engine.estimate on its
    GPU) and the results are all-gathered into global chain order on every rank — the only
    collective (RCCL with the nccl backend; no data-path exchange inside a chain)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    T_use = np.asarray(T_use, dtype=np.int32)
    P, R = Theta0.shape
    parts = balanced_window_assignment(T_use, world)
    mine = parts[rank]
    if mine.size:
        res = estimate(np.asfortranarray(Theta0[:, mine]), np.ascontiguousarray(T_use[mine]))
        local = np.vstack([res["theta_c"], res["ll"][None, :], np.asarray(res["status"], np.float64)[None, :]])
    else:
        local = np.zeros((P + 2, 0))
    m = max(len(p) for p in parts)
    buf = torch.full((P + 2, m), float("nan"), dtype=torch.float64)
    buf[:, :local.shape[1]] = torch.from_numpy(local)
    if device is not None:
        buf = buf.to(_comm_device(group, device))
    out = torch.empty((world * (P + 2), m), dtype=torch.float64, device=buf.device)
    dist.all_gather_into_tensor(out, buf.contiguous(), group=group)
    out = out.view(world, P + 2, m).cpu().numpy()
    glob = np.empty((P + 2, R))
    for r, idx in enumerate(parts):
        glob[:, idx] = out[r, :, :len(idx)]
    return dict(theta_c=glob[:P], ll=glob[P], status=glob[P + 1].astype(np.int32), assignment=parts)
