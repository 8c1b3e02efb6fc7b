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
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # loopback: the hostname may not resolve
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


def _run_bench(args, env=None, timeout=300):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=e,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_launcher_two_ranks():
    """`bench.py --gpus 2` with no launcher starts 2 rank processes itself (gloo / CPU
    oracle stand-in here): one JSON line from rank 0 with n_gpus 2, value = all ranks'
    bytes / the slowest rank's time, per-rank seeds seed + rank."""
    rc, out, err = _run_bench(["--gpus", "2", "--cpu-standin", "--size-gib", "0.01",
                               "--steps", "2", "--warmup", "1"])
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["stand_in"] is True
    recs = sorted(out["per_rank"], key=lambda r: r["rank"])
    assert [r["rank"] for r in recs] == [0, 1]
    assert recs[1]["seed"] == recs[0]["seed"] + 1
    # every record names its world, its device (here the stand-in process) and its own time
    assert all(r["world_size"] == 2 and r["avg_launch_ms"] > 0 for r in recs)
    assert recs[0]["device"]["pid"] != recs[1]["device"]["pid"]
    mx = max(r["elapsed_s"] for r in recs)
    tot = sum(r["bytes"] for r in recs)
    assert out["value"] == pytest.approx(tot * 2 / (1 << 30) / mx, rel=1e-3)
    assert out["ms_per_step"] == pytest.approx(mx / 2 * 1e3, rel=1e-3)


def test_bench_refuses_missing_gpus():
    """--gpus 2 on a box with fewer GPUs (here none) fails loudly instead of running 1."""
    rc, out, err = _run_bench(["--gpus", "2", "--steps", "1"], timeout=120)
    assert rc == 2 and out is None and "GPU" in err


def test_bench_refuses_world_mismatch():
    rc, out, err = _run_bench(["--gpus", "4", "--cpu-standin", "--steps", "1"],
                              env={"WORLD_SIZE": "2", "RANK": "0"}, timeout=120)
    assert rc == 2 and "disagrees" in err


def test_bench_share_gpu_refuses_without_gpu():
    """The one-GPU rehearsal (PBS_BENCH_SHARE_GPU=1) still needs a GPU: here it fails
    loudly instead of falling back to anything."""
    if _has_gpu():
        pytest.skip("a GPU is visible")
    rc, out, err = _run_bench(["--gpus", "2", "--steps", "1", "--size-gib", "0.01"],
                              env={"PBS_BENCH_SHARE_GPU": "1"}, timeout=180)
    assert rc == 2 and out is None and "GPU" in err


def _has_gpu():
    import torch
    return torch.cuda.device_count() > 0


def _oracle_cuts(oracle, workload, seed, size, avg):
    import numpy as np
    gen = {"vmimage": oracle.gen_vmimage, "random": oracle.gen_random}[workload]
    ref = oracle.chunk_feed(avg, gen(size, seed, 0))
    if ref.size == 0 or int(ref[-1]) != size:
        ref = np.append(ref, np.uint64(size))
    return [int(x) for x in ref]


def test_kfd_gpu_count_without_hip():
    """The launcher counts GPUs from sysfs only; the visible-devices lists narrow it."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    n = bench.kfd_gpu_count()
    assert n is None or n >= 0
    if n:
        old = os.environ.get("HIP_VISIBLE_DEVICES")
        os.environ["HIP_VISIBLE_DEVICES"] = "0"
        try:
            assert bench.kfd_gpu_count() == 1
        finally:
            if old is None:
                os.environ.pop("HIP_VISIBLE_DEVICES")
            else:
                os.environ["HIP_VISIBLE_DEVICES"] = old


def test_standin_records_cut_lists(oracle):
    """Every rank's record carries its cut list (and its SHA-256), so the multi-rank runs
    can be diffed against the oracle rank by rank; each is verified against the golden
    record (tests/golden/bench_cuts.json)."""
    size = int(0.01 * (1 << 30)) // 8 * 8
    rc, out, err = _run_bench(["--gpus", "2", "--cpu-standin", "--size-gib", "0.01", "--avg", "65536",
                               "--steps", "1", "--warmup", "0"])
    assert rc == 0, err[-2000:]
    assert out["verified"] is True
    for r in out["per_rank"]:  # (find_cuts(is_final)'s list: the stream end appended)
        ref = _oracle_cuts(oracle, "vmimage", r["seed"], size, 65536)
        assert r["cuts"] == ref and r["chunks"] == len(ref) and r["verified"] is True


def test_bench_verification_fails_loudly(tmp_path):
    """A cut list that differs from the golden record, or a stream without one, makes
    bench.py print verified false / null and exit 3 (the line still printed)."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = json.load(open(os.path.join(root, "tests", "golden", "bench_cuts.json")))
    size = int(0.01 * (1 << 30)) // 8 * 8
    k = f"vmimage:{size}:{4 << 20}:{0x5EED0004:#x}"  # rank 1's entry
    doc["streams"][k]["cuts_sha256"] = "0" * 64
    bad = tmp_path / "golden.json"
    bad.write_text(json.dumps(doc))
    rc, out, err = _run_bench(["--gpus", "2", "--cpu-standin", "--size-gib", "0.01", "--steps", "1",
                               "--warmup", "0"], env={"PBS_BENCH_GOLDEN": str(bad)})
    assert rc == 3 and out["verified"] is False
    recs = sorted(out["per_rank"], key=lambda r: r["rank"])
    assert recs[0]["verified"] is True and recs[1]["verified"] is False
    rc, out, err = _run_bench(["--gpus", "2", "--cpu-standin", "--size-gib", "0.02", "--steps", "1",
                               "--warmup", "0"])
    assert rc == 3 and out["verified"] is False
    assert all(r["verified"] is None and "no golden entry" in r["verify_note"] for r in out["per_rank"])
    rc, out, err = _run_bench(["--gpus", "2", "--cpu-standin", "--size-gib", "0.02", "--steps", "1",
                               "--warmup", "0", "--verify", "0"])
    assert rc == 0 and "verified" not in out


def test_bench_golden_script_pinned(oracle):
    """tests/golden/make_bench_golden.py reproduces its committed small entries, and its
    streaming oracle (ora_chunk_generated, the stream generated 16 MiB at a time) equals
    chunk_feed over the whole generated buffer with the tail appended."""
    import json
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    import make_bench_golden as mbg
    have = json.load(open(mbg.OUT))["streams"]
    todo = [s for s in mbg.streams() if s[1] < (64 << 20)]
    assert len(todo) == 4
    for s in todo:
        assert mbg.record(*s) == have[mbg.key(*s)]
    # every bench stream has an entry: config 3 ranks 0-7, config 5, config 2, all averages
    assert all(mbg.key(*s) in have for s in mbg.streams())
    n = (40 << 20) + 13
    for kind, seed in (("vmimage", 0x5EED0003), ("random", 0x5EED0002), ("counter", 0)):
        buf = oracle.gen_block(kind, n, seed)
        ref = oracle.chunk_feed(65536, buf)
        ref = np.append(ref, np.uint64(n)) if ref.size == 0 or int(ref[-1]) != n else ref
        assert np.array_equal(oracle.chunk_generated(kind, seed, 65536, n, piece=(3 << 20) + 5), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["streams", "sharded"])
def test_bench_share_gpu_rehearsal(oracle, mode):
    """The N-rank GPU path of bench.py with both ranks on GPU 0 over gloo: one line from
    rank 0, labelled as a rehearsal, n_gpus 2, MAX/SUM aggregation, and every rank's cut
    list equal to the oracle's -- its own stream (seed + rank) in the streams mode, the
    whole stream in the sharded mode (halo and candidate all-gathers staged through host
    memory, since gloo takes CPU tensors).  The RCCL collectives are covered by
    test_bench_rccl_world1."""
    gib = 0.25
    size = int(gib * (1 << 30)) // 8 * 8
    rc, out, err = _run_bench(["--gpus", "2", "--size-gib", str(gib), "--steps", "2", "--warmup", "1",
                               "--mode", mode, "--cpu-baseline", "0", "--host-inclusive-gib", "0",
                               "--secondary-random", "0"],
                              env={"PBS_BENCH_SHARE_GPU": "1"}, timeout=240)
    assert rc == 0, err[-2000:]
    assert out["n_gpus"] == 2 and out["metric"].startswith("REHEARSAL") and "rehearsal" in out
    assert out["backend"] == "gloo"
    recs = sorted(out["per_rank"], key=lambda r: r["rank"])
    assert [r["rank"] for r in recs] == [0, 1]
    for r in recs:  # device identity and the rank's own kernel time (one shared GPU here)
        assert r["world_size"] == 2 and r["avg_launch_ms"] > 0
        assert r["device"]["index"] == 0 and r["device"].get("pci")
    if mode == "streams":
        assert recs[1]["seed"] == recs[0]["seed"] + 1
        for r in recs:
            assert r["bytes"] == size
            assert r["cuts"] == _oracle_cuts(oracle, "vmimage", r["seed"], size, 4 << 20), r["rank"]
    else:
        ref = _oracle_cuts(oracle, "vmimage", recs[0]["seed"], size, 4 << 20)
        assert sum(r["bytes"] for r in recs) == size
        for r in recs:
            assert r["cuts"] == ref, r["rank"]
    mx = max(r["elapsed_s"] for r in recs)
    tot = sum(r["bytes"] for r in recs)
    assert out["value"] == pytest.approx(tot * 2 / (1 << 30) / mx, rel=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["streams", "sharded"])
def test_bench_rccl_world1(oracle, mode):
    """bench.py under torch.distributed.run with one rank and its RCCL ("nccl") group
    (PBS_BENCH_DIST_WORLD1=1): the device-tensor barrier, MAX/SUM all-reduces, the
    per-rank all_gather_object and (sharded) the halo and candidate all-gathers all run
    through RCCL on the GPU -- the collectives of the 8-GPU run, at world size 1."""
    import subprocess
    import sys
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gib = 0.25
    size = int(gib * (1 << 30)) // 8 * 8
    e = dict(os.environ, PBS_BENCH_DIST_WORLD1="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PBS_BENCH_SHARE_GPU"):
        e.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "1", "--size-gib", str(gib), "--steps", "2",
           "--warmup", "1", "--mode", mode, "--cpu-baseline", "0", "--host-inclusive-gib", "0",
           "--secondary-random", "0"]
    p = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["backend"] == "nccl"
    (r,) = out["per_rank"]
    assert r["world_size"] == 1 and r["avg_launch_ms"] > 0 and r["device"].get("pci")
    assert r["bytes"] == size
    assert r["cuts"] == _oracle_cuts(oracle, "vmimage", r["seed"], size, 4 << 20)
    assert out["value"] == pytest.approx(size * 2 / (1 << 30) / r["elapsed_s"], rel=1e-2)
