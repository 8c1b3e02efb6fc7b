"""Multi-process (world size 2, gloo, CPU) tests of bench.py's N-GPU logic: each rank
has its own stream, and the job reports the slowest rank's time and all ranks' bytes."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = 1.0 + rank  # rank 1 is the slow one
    nbytes = (rank + 1) * 1000
    t, tot = bench.aggregate(elapsed, nbytes, dist, torch.device("cpu"))
    seeds = [None] * world
    dist.all_gather_object(seeds, bench.stream_seed("vmimage", rank))
    q.put((rank, t, tot, seeds))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_aggregation():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    out = [q.get(timeout=120) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    for rank, t, tot, seeds in out:
        assert t == pytest.approx(2.0)        # MAX over ranks
        assert tot == pytest.approx(3000.0)   # SUM over ranks
        assert len(set(seeds)) == world       # independent streams per GPU


def test_single_rank_aggregation():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    assert bench.aggregate(1.5, 42, None, None) == (1.5, 42.0)
