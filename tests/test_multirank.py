"""The N>1 bench path on CPU: the strong-scaling window split and the only cross-rank exchange
(max of the timed region, sum of early-terminated windows) run under gloo with world_size 2
(windows are independent replicas, no collective inside the iteration)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from _paths import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


@pytest.mark.parametrize("total,world", [(512, 1), (512, 2), (512, 8), (7, 3), (1, 2)])
def test_rank_windows_partition(total, world):
    parts = [bench.rank_windows(total, world, r) for r in range(world)]
    flat = [i for p in parts for i in p]
    assert flat == list(range(total))
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = bench.rank_windows(512, world, rank)
    elapsed = 0.5 + rank  # rank 1 is the slow one
    early = len(mine) % 3 + rank
    out = bench.aggregate(dist, elapsed, early, "cpu")
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, len(mine), out))


def test_gloo_two_ranks_aggregate():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [n for _, n, _ in res] == [256, 256]
    expect_early = (256 % 3) + (256 % 3 + 1)
    for _, _, (elapsed, early) in res:
        assert elapsed == 1.5 and early == expect_early
