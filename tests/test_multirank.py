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


def _gather_worker(rank, world, port, total, q):
    import numpy as np
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = bench.rank_windows(total, world, rank)
    sums = [{"initial_cost": 10.0 + i, "final_cost": 1.0 + i, "num_iterations": 13, "num_successful_steps": 12,
             "termination_type": 1} for i in mine]
    got = bench.gather_rows(dist, bench.summary_rows(mine, sums), total, "cpu")
    poses = bench.gather_rows(dist, np.full((len(mine), 14), float(rank)), total, "cpu")
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, got.tolist(), poses.tolist()))


@pytest.mark.parametrize("total", [8, 7])
def test_gloo_two_ranks_gather(total):
    """SURVEY.md §8e end-of-run gather: per-window summaries and final poses of every rank reach
    every rank in window order, also when the ranks hold different counts (7 = 4 + 3)."""
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, got, poses in res:
        got, poses = np.array(got), np.array(poses)
        assert got.shape == (total, len(bench.SUMMARY_COLS))
        assert np.array_equal(got[:, 0], np.arange(total))
        assert np.array_equal(got[:, 2], 1.0 + np.arange(total))
        n0 = len(bench.rank_windows(total, 2, 0))
        assert np.all(poses[:n0] == 0.0) and np.all(poses[n0:] == 1.0)


def test_launcher_starts_n_ranks():
    """`bench.py --gpus 2` without WORLD_SIZE starts two ranks through a torch.distributed.run child
    process (127.0.0.1 rendezvous); the dry-run mode exercises the rank env and the gather on gloo
    without touching a GPU."""
    import json
    import subprocess
    env = dict(os.environ, OKVISGPU_BENCH_DRYRUN="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--windows", "9"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d == {"world": 2, "gpus": 2, "windows": 9, "in_order": True, "master_addr": "127.0.0.1"}


def test_launcher_strong_scaling_default():
    """Without --windows / --windows-per-gpu the job is the fixed 2,048-window batch split across the
    ranks (strong scaling, BASELINE north_star), gathered in window order."""
    import json
    import subprocess
    env = dict(os.environ, OKVISGPU_BENCH_DRYRUN="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d == {"world": 2, "gpus": 2, "windows": bench.DEFAULT_WINDOWS, "in_order": True,
                 "master_addr": "127.0.0.1"}
    args = bench.parse_args([])
    assert bench.job_windows(args, 8) is True and args.windows == 2048
    assert len(bench.rank_windows(args.windows, 8, 7)) == 256


def test_launcher_weak_scaling():
    """--windows-per-gpu: every rank holds that many windows of its own (weak scaling): the job
    total grows with the rank count and the gather still returns every window in order."""
    import json
    import subprocess
    env = dict(os.environ, OKVISGPU_BENCH_DRYRUN="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--windows-per-gpu", "5"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert d == {"world": 2, "gpus": 2, "windows": 10, "in_order": True, "master_addr": "127.0.0.1"}


def test_world_size_mismatch_is_an_error():
    import subprocess
    env = dict(os.environ, OKVISGPU_BENCH_DRYRUN="1", WORLD_SIZE="1")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "WORLD_SIZE" in out.stderr
