"""The local N-rank launcher of bench.py --gpus N (yfm_amd.distributed.spawn_local_ranks), on CPU with
gloo: every rank joins one process group of N members, and a failing rank fails the job (the ranks
left waiting in a collective are terminated rather than hanging)."""
from __future__ import annotations

import json
import sys
import textwrap

from conftest import PKG, ROOT

WORKER = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    out, fail_rank = sys.argv[1], int(sys.argv[2])
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    one = torch.ones(1)
    dist.all_reduce(one)
    if r == fail_rank:
        sys.exit(3)
    dist.barrier()
    json.dump({"rank": r, "world": w, "sum": float(one.item()), "local": int(os.environ["LOCAL_RANK"]),
               "addr": os.environ["MASTER_ADDR"]}, open(f"{out}/rank{r}.json", "w"))
""")


def _spawn(tmp_path, n, fail_rank):
    sys.path[:0] = [str(PKG), str(ROOT)]
    from yfm_amd.distributed import spawn_local_ranks
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    return spawn_local_ranks(str(script), [str(tmp_path), str(fail_rank)], n, timeout=120)


def test_launcher_starts_n_ranks(tmp_path):
    assert _spawn(tmp_path, 3, -1) == 0
    got = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [g["rank"] for g in got] == [0, 1, 2] and all(g["world"] == 3 and g["sum"] == 3.0 for g in got)
    assert [g["local"] for g in got] == [0, 1, 2] and all(g["addr"] == "127.0.0.1" for g in got)


def test_launcher_propagates_a_failing_rank(tmp_path):
    rc = _spawn(tmp_path, 2, 1)
    assert rc == 3
    assert not (tmp_path / "rank0.json").exists()  # rank 0 was left in the barrier and terminated
