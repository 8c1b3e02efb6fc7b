"""One stream sharded over ranks (proxmox-backup_amd/shard.py).

CPU: world-size 2 and 3 over gloo, with the oracle standing in for the two C-ABI
phases (candidates_device / resolve_device) on CPU tensors -- checks the halo
exchange, the candidate all-gather and the concatenation order against the oracle's
single-stream cut list.  GPU: the same driver with the HIP phases, ranks simulated
in one process (one GPU), and a one-rank run through torch.distributed.
"""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import gen_np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KiB, MiB = 1024, 1024 * 1024


class OracleChunker:
    """CPU stand-in with the Chunker methods shard.py calls (tests only)."""

    def __init__(self, avg):
        import oracle
        self.o = oracle
        self.avg = avg

    def cuts_bound(self, length):
        return length // max(self.avg // 4, 65) + 3

    def candidates_device(self, ptr, length, pre, base, out_ptr, cap):
        data = np.ctypeslib.as_array((ctypes.c_uint8 * length).from_address(ptr)) if length else \
            np.zeros(0, np.uint8)
        assert len(pre) == min(base, 63)
        buf = np.concatenate([np.frombuffer(pre, np.uint8), data])
        c = self.o.candidates(self.avg, buf).astype(np.int64) + (base - len(pre))
        if c.size > cap:
            e = RuntimeError("capacity")
            e.needed = int(c.size)
            raise e
        if c.size:
            np.ctypeslib.as_array((ctypes.c_int64 * c.size).from_address(out_ptr))[:] = c
        return int(c.size)

    def resolve_device(self, ptr, n, end, is_final=True):
        cand = np.ctypeslib.as_array((ctypes.c_uint64 * n).from_address(ptr)).copy() if n else \
            np.zeros(0, np.uint64)
        cuts = self.o.resolve(self.avg, cand, end)
        if is_final and (cuts.size == 0 or int(cuts[-1]) != end):
            cuts = np.append(cuts, np.uint64(end))
        return cuts


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(n):
    return gen_np.gen_vmimage(n, 0x5EED0003, 700 * MiB + 4096 * 3 + 40)


def _worker(rank, world, port, n, avg, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "proxmox-backup_amd")]
    import torch
    import torch.distributed as dist
    import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # loopback: the hostname may not resolve
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = _stream(n)
    base, ln = shard.shard_ranges(n, world)[rank]
    local = torch.from_numpy(data[base:base + ln].copy())
    tail = local[max(0, ln - shard.HALO):]
    cuts = shard.chunk_sharded(OracleChunker(avg), local.data_ptr(), ln, base, n, tail, dist,
                               rank, world, torch.device("cpu"))
    q.put((rank, cuts.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_stream_gloo(oracle, world):
    n, avg = 6 * MiB + 13, 64 * KiB
    ref = oracle.chunk_feed(avg, _stream(n)).tolist()
    if not ref or ref[-1] != n:
        ref.append(n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, avg, q)) for r in range(world)]
    [p.start() for p in procs]
    out = [q.get(timeout=180) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    for rank, cuts in out:
        assert cuts == ref, rank


def test_collectives_without_a_group():
    """One rank: the torch.distributed module passed with no initialised process group
    (or None) means nothing to exchange -- no collective is called."""
    import torch
    import torch.distributed as dist

    import shard
    assert not dist.is_initialized()
    tail = torch.arange(63, dtype=torch.uint8)
    cand = torch.tensor([70, 900], dtype=torch.int64)
    for d in (dist, None):
        assert shard.exchange_halo(tail, d, 0, 1) == b""
        assert shard.gather_candidates(cand, d, 1) is cand
    with pytest.raises(ValueError):
        shard.exchange_halo(torch.zeros(64, dtype=torch.uint8), dist, 0, 1)


def test_shard_ranges():
    import shard
    for total, world in [(64 << 30, 8), (1000, 3), (8 * 7 + 5, 7)]:
        rs = shard.shard_ranges(total, world)
        assert rs[0][0] == 0 and sum(l for _, l in rs) == total
        assert all(b % 8 == 0 for b, _ in rs)
        assert all(rs[i][0] + rs[i][1] == rs[i + 1][0] for i in range(world - 1))


@pytest.mark.gpu
@pytest.mark.parametrize("nshards,avg", [(1, 1 * MiB), (3, 1 * MiB), (4, 4096), (5, 256)])
def test_sharded_phases_gpu(gpu, oracle, nshards, avg):
    """The HIP phases over simulated ranks (one process, one GPU): unaligned shard
    starts, a shard boundary inside a window, the stream head shard (base < 63)."""
    import torch
    import shard
    n = 40 * MiB + 77 if avg >= 4096 else 3 * MiB + 5
    data = _stream(n)
    ref = oracle.chunk_feed(avg, data)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    dev = torch.from_numpy(data).cuda()
    rng = np.random.default_rng(nshards)
    bounds = [0] + sorted(int(x) for x in rng.choice(np.arange(64, n - 64), nshards - 1,
                                                      replace=False)) + [n]
    if nshards >= 3:
        bounds[1] = 40  # head shard shorter than the window: the next base is < 63
    with gpu.Chunker(avg) as ch:
        parts = []
        for a, b in zip(bounds[:-1], bounds[1:]):
            pre = data[max(0, a - 63):a].tobytes()
            parts.append(shard.phase_a(ch, dev.data_ptr() + a, b - a, a, pre, dev.device))
        allc = torch.cat(parts).contiguous()
        got = ch.resolve_device(allc.data_ptr(), int(allc.numel()), n, True)
        whole = oracle.candidates(avg, data)
    assert np.array_equal(allc.cpu().numpy().astype(np.uint64), whole)
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_sharded_single_rank_gpu(gpu, oracle):
    """chunk_sharded end to end with world size 1 (no collective needed)."""
    import torch
    import shard
    n, avg = 24 * MiB + 8, 256 * KiB
    data = _stream(n)
    ref = oracle.chunk_feed(avg, data)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    dev = torch.from_numpy(data).cuda()
    with gpu.Chunker(avg) as ch:
        got = shard.chunk_sharded(ch, dev.data_ptr(), n, 0, n, dev[n - 63:], None, 0, 1,
                                  dev.device)
    assert np.array_equal(got, ref)
