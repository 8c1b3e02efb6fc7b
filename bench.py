"""Benchmark of the MI355X content-defined chunker (BASELINE.json metric).

One "step" = one pass of the chunker over the whole device-resident synthetic stream
(phase A scan + exact blocks + sort + min/max resolve + cut list to the host).
Default workload = BASELINE config 3: 64 GiB VM-image-like stream, 4 MiB average.
Multi-GPU (config 4): one independent stream per rank (seed + rank), no data-path
collective; an all-reduce (RCCL) of the per-rank elapsed time (MAX) and byte count.
--mode sharded: ONE stream of --size-gib split over the ranks (strong scaling; SURVEY
8(e)): halo all-gather, per-rank phase A, candidate all-gather, resolve on every rank
(proxmox-backup_amd/shard.py).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size-gib 64] [--avg 4194304]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "proxmox-backup_amd"))

METRIC = "GiB/s chunked (device-resident), 4 MiB mean, 64 GiB stream; boundaries bit-exact"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
GEN = {"counter": 0, "random": 1, "vmimage": 2}
SEEDS = {"counter": 0, "random": 0x5EED0002, "vmimage": 0x5EED0003}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size-gib", type=float, default=64.0)
    ap.add_argument("--avg", type=int, default=4 * 1024 * 1024)
    ap.add_argument("--workload", choices=list(GEN), default="vmimage")
    ap.add_argument("--mode", choices=["streams", "sharded"], default="streams",
                    help="streams: one independent stream per GPU (config 4); "
                         "sharded: one stream split over the GPUs")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the CPU oracle timing")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-sample-mib", type=int, default=512)
    ap.add_argument("--host-inclusive-gib", type=float, default=4.0,
                    help="also time the host-buffer path (H2D + kernels + D2H) on this many GiB; 0 = skip")
    ap.add_argument("--digest", type=int, default=0,
                    help="also time the per-chunk SHA-256 stage (SURVEY 8(f)) over the stream's "
                         "chunks (GPU), with hashlib on the host cores beside it")
    ap.add_argument("--pipeline-gib", type=float, default=0.0,
                    help="also time the host-stream pipeline (copy -> chunk -> SHA-256 per chunk, "
                         "pbs_pipeline_host) over this many GiB of a pageable host copy of the "
                         "stream, with the oracle + hashlib on the host cores beside it")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per scan launch (written by profiles/collect_traffic.py)")
    return ap.parse_args()


def stream_seed(workload: str, rank: int) -> int:
    """Config 4: every GPU chunks its own independent stream (seed + rank)."""
    return SEEDS[workload] + rank


def aggregate(elapsed: float, nbytes: int, dist, device):
    """Whole-job numbers for N ranks: the slowest rank's time (MAX) and all ranks'
    bytes (SUM), one all-reduce each (RCCL on GPUs, gloo in the CPU tests)."""
    import torch

    if dist is None:
        return elapsed, float(nbytes)
    mx = torch.tensor([elapsed], dtype=torch.float64, device=device)
    tot = torch.tensor([float(nbytes)], dtype=torch.float64, device=device)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return float(mx.item()), float(tot.item())


def cpu_baseline(args, workload, seed, avg):
    """The oracle (faithful C restatement of chunker.rs) on the host cores, on a bounded
    sample of the same stream: `threads` threads each chunk their own sample slice."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle

    n = args.cpu_sample_mib * 1024 * 1024
    gen = {"counter": lambda o: oracle.gen_counter(n, o),
           "random": lambda o: oracle.gen_random(n, seed, o),
           "vmimage": lambda o: oracle.gen_vmimage(n, seed, o)}[workload]
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    bufs = [None] * threads

    def mk(t):
        bufs[t] = gen(t * n)

    ths = [threading.Thread(target=mk, args=(t,)) for t in range(threads)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    # single thread, one slice
    t0 = time.perf_counter()
    oracle.chunk_feed(avg, bufs[0])
    single = n / (1 << 30) / (time.perf_counter() - t0)
    # all threads, independent slices (ctypes releases the GIL)
    ths = [threading.Thread(target=oracle.chunk_feed, args=(avg, bufs[t])) for t in range(threads)]
    t0 = time.perf_counter()
    [t.start() for t in ths]
    [t.join() for t in ths]
    agg = threads * n / (1 << 30) / (time.perf_counter() - t0)
    cpu = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].split(":", 1)[-1].strip() \
        if os.path.exists("/proc/cpuinfo") else "unknown"
    del bufs
    return {"value": round(agg, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{threads} x {args.cpu_sample_mib} MiB slices of the same {workload} stream, "
                      f"whole-buffer scan loop (oracle/chunker_oracle.c, gcc -O2); "
                      f"1 thread: {single:.3f} GiB/s; host CPU: {cpu}"}


def digest_stage(args, buf, cuts, stream, reps: int = 3):
    """Per-chunk SHA-256 of the whole device-resident stream (one lane per chunk, longest
    chunks first), timed with HIP events on the launch stream; hashlib (OpenSSL) on the
    host cores over a bounded sample of the same chunks as the CPU reference point."""
    import hashlib

    import numpy as np
    import torch

    import pbschunk

    size = buf.numel()
    bounds = np.concatenate([[0], cuts]).astype(np.uint64)
    n = bounds.size - 1
    lens = np.diff(bounds.astype(np.int64))
    order = np.argsort(-lens, kind="stable").astype(np.int32)
    bd = torch.from_numpy(bounds.view(np.int64)).to(buf.device)
    od = torch.from_numpy(order).to(buf.device)
    out = torch.empty(n * 32, dtype=torch.uint8, device=buf.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    pbschunk.digest_chunks_async(buf.data_ptr(), size, bd.data_ptr(), od.data_ptr(), n,
                                 out.data_ptr(), hip_stream=stream.cuda_stream)  # warm-up
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        ev[0].record(stream)
        pbschunk.digest_chunks_async(buf.data_ptr(), size, bd.data_ptr(), od.data_ptr(), n,
                                     out.data_ptr(), hip_stream=stream.cuda_stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    t = min(ms) / 1e3
    # known-chunk test of the same digests (backup_writer.rs:677-697; no previous index:
    # repeats inside the stream, e.g. the zero chunks, are the known ones)
    flags = torch.empty(n, dtype=torch.uint8, device=buf.device)
    t0 = time.perf_counter()
    nknown = pbschunk.known_chunks_device(out.data_ptr(), n, 0, 0, flags.data_ptr(),
                                          hip_stream=stream.cuda_stream)
    known_ms = (time.perf_counter() - t0) * 1e3
    # host reference point: hashlib over the first chunks totalling ~1 GiB, 16 threads
    take = int(np.searchsorted(np.cumsum(lens), 1 << 30)) + 1
    take = max(1, min(n, take))
    host = buf[: int(bounds[take])].cpu().numpy()
    mv = memoryview(host)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    parts = [list(range(k, take, threads)) for k in range(threads)]

    def work(ix):
        for i in ix:
            hashlib.sha256(mv[int(bounds[i]):int(bounds[i + 1])]).digest()

    ths = [threading.Thread(target=work, args=(ix,)) for ix in parts]
    t0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu_gib_s = int(bounds[take]) / (1 << 30) / (time.perf_counter() - t0)
    crc = crc_stage(args, buf, bd, od, n, bounds, take, threads, stream, reps)
    return {"metric": "GiB/s SHA-256 digested (per chunk, device-resident)",
            "value": round(size / (1 << 30) / t, 3), "ms": round(t * 1e3, 3), "chunks": n,
            "max_chunk": int(lens.max()), "bound": "valu (one lane per chunk; serial per chunk)",
            "known_chunks": nknown, "known_ms": round(known_ms, 3),
            "cpu_baseline": {"value": round(cpu_gib_s, 3), "unit": "GiB/s", "cores": threads,
                             "kind": "hashlib (OpenSSL)",
                             "sample": f"first {take} chunks ({int(bounds[take]) >> 20} MiB)"},
            "blob_crc": crc}


def crc_stage(args, buf, bd, od, n, bounds, take, threads, stream, reps):
    """DataBlob::compute_crc (CRC-32) of every chunk on the device
    (256 lanes per chunk, HBM-bound), HIP events on the launch stream; zlib.crc32 (the
    same CRC-32) on the host cores over the digest stage's sample."""
    import zlib

    import torch

    import pbschunk

    size = buf.numel()
    out = torch.empty(n, dtype=torch.int32, device=buf.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    pbschunk.crc32_chunks_async(buf.data_ptr(), size, bd.data_ptr(), od.data_ptr(), n, out.data_ptr(),
                                hip_stream=stream.cuda_stream)  # warm-up
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        ev[0].record(stream)
        pbschunk.crc32_chunks_async(buf.data_ptr(), size, bd.data_ptr(), od.data_ptr(), n, out.data_ptr(),
                                    hip_stream=stream.cuda_stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    t = min(ms) / 1e3
    host = buf[: int(bounds[take])].cpu().numpy()
    mv = memoryview(host)
    parts = [list(range(k, take, threads)) for k in range(threads)]

    def work(ix):
        for i in ix:
            zlib.crc32(mv[int(bounds[i]):int(bounds[i + 1])])

    ths = [threading.Thread(target=work, args=(ix,)) for ix in parts]
    t0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu = int(bounds[take]) / (1 << 30) / (time.perf_counter() - t0)
    return {"metric": "GiB/s blob CRC-32 (per chunk, device-resident)",
            "value": round(size / (1 << 30) / t, 3), "ms": round(t * 1e3, 3),
            "roofline": {"bound": "hbm", "achieved": round(size / t / 1e9, 1), "peak": 8000.0,
                         "unit": "GB/s", "frac": round(size / t / 8e12, 4)},
            "cpu_baseline": {"value": round(cpu, 3), "unit": "GiB/s", "cores": threads,
                             "kind": "zlib.crc32 (same CRC-32 as crc32fast)",
                             "sample": f"first {take} chunks ({int(bounds[take]) >> 20} MiB)"}}


def pipeline_stage(args, buf, piece: int = 1 << 30):
    """a pageable host copy of the stream's first --pipeline-gib GiB
    through pbs_pipeline_host (copy thread -> HBM, chunker on CU-masked stream, per-chunk
    SHA-256 and blob CRC-32 on the other CUs, overlapped), end to end; the CPU path beside
    it: the oracle chunker + hashlib + zlib.crc32 per chunk on the host cores over a
    bounded sample."""
    import hashlib
    import zlib

    import numpy as np

    import pbschunk

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    n = int(args.pipeline_gib * (1 << 30)) // 8 * 8
    host = buf[:n].cpu().numpy()  # pageable, untimed
    pbschunk.pipeline_host(host[: 64 << 20], args.avg, piece=16 << 20, crc=True)  # warm-up
    t0 = time.perf_counter()
    ends, dig, crcs, t = pbschunk.pipeline_host(host, args.avg, piece=piece, crc=True)
    wall = time.perf_counter() - t0
    # CPU path: threads chunk their own slice and hash its chunks (hashlib/OpenSSL)
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    per = (256 << 20)

    def work(k):
        sl = host[k * per:(k + 1) * per]
        cuts = oracle.chunk_feed(args.avg, sl)
        b = np.concatenate([[0], cuts, [sl.size]]).astype(np.int64)
        mv = memoryview(sl)
        for i in range(b.size - 1):
            if b[i + 1] > b[i]:
                hashlib.sha256(mv[b[i]:b[i + 1]]).digest()
                zlib.crc32(mv[b[i]:b[i + 1]])

    nth = min(threads, max(1, n // per))
    ths = [threading.Thread(target=work, args=(k,)) for k in range(nth)]
    c0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu = nth * per / (1 << 30) / (time.perf_counter() - c0)
    return {"metric": "GiB/s host stream -> chunk boundaries + SHA-256 + blob CRC-32 per chunk (end to end)",
            "value": round(n / (1 << 30) / wall, 3), "bytes": n, "piece": piece,
            "chunks": int(ends.size), "timing_ms": {k: round(v, 2) for k, v in t.items()
                                                     if k.endswith("_ms")},
            "cpu_baseline": {"value": round(cpu, 3), "unit": "GiB/s", "cores": nth,
                             "kind": "port (oracle chunker) + hashlib + zlib.crc32",
                             "sample": f"{nth} x 256 MiB slices: chunk_feed then sha256 + crc32 per chunk"}}


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import pbschunk

    size = int(args.size_gib * (1 << 30)) // 8 * 8
    stream = torch.cuda.current_stream()
    ch = pbschunk.Chunker(args.avg)
    ch.set_stream(stream.cuda_stream)
    if args.mode == "sharded":
        import shard
        seed = SEEDS[args.workload]  # one stream; this rank generates its range of it
        base, local = shard.shard_ranges(size, world)[rank]
        buf = torch.empty(local, dtype=torch.uint8, device=dev)
        pbschunk.generate_device(buf.data_ptr(), local, GEN[args.workload], seed, base,
                                 stream.cuda_stream)
        torch.cuda.synchronize()
        ptr, tail = buf.data_ptr(), buf[max(0, local - shard.HALO):]

        def step():
            return shard.chunk_sharded(ch, ptr, local, base, size, tail, dist, rank, world, dev)
        work_bytes = local
    else:
        seed = stream_seed(args.workload, rank)
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        pbschunk.generate_device(buf.data_ptr(), size, GEN[args.workload], seed, 0,
                                 stream.cuda_stream)
        torch.cuda.synchronize()
        ptr = buf.data_ptr()

        def step():
            return ch.find_cuts_device(ptr, size, is_final=True)
        work_bytes = size

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scan_ms, ncuts, cand = [], 0, 0
    for _ in range(args.steps):
        cuts = step()
        t = ch.last_timing()
        scan_ms.append(t["scan_ms"])
        ncuts, cand = int(cuts.size), int(t["candidates"])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed, total_bytes = aggregate(elapsed, work_bytes, dist, dev)

    step_s = elapsed / max(1, args.steps)
    value = total_bytes * args.steps / (1 << 30) / elapsed
    avg_scan_s = float(np.mean(scan_ms)) / 1e3 if scan_ms else float("nan")
    achieved = work_bytes / avg_scan_s / 1e9  # algorithmic bytes (input read once) per launch
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if (tj.get("size") == work_bytes and tj.get("avg") == args.avg
                and tj.get("workload") == args.workload and args.mode == "streams"):
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    host_incl = None
    if rank == 0 and world == 1 and args.host_inclusive_gib > 0 and args.mode == "streams":
        hn = int(args.host_inclusive_gib * (1 << 30)) // 8 * 8
        hbuf = buf[:hn].cpu().numpy()  # pageable host copy of the stream prefix
        ch2 = pbschunk.Chunker(args.avg)
        ch2.find_cuts(hbuf[: 64 << 20], is_final=True)  # warm allocation
        t1 = time.perf_counter()
        ch2.find_cuts(hbuf, is_final=True)
        host_incl = hn / (1 << 30) / (time.perf_counter() - t1)
        ch2.close()
        del hbuf

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    default_cfg = (args.size_gib == 64.0 and args.avg == 4 * 1024 * 1024
                   and args.workload == "vmimage" and args.mode == "streams")
    metric = METRIC if default_cfg else (
        f"GiB/s chunked (device-resident), {args.avg >> 10} KiB mean, {args.size_gib:g} GiB "
        f"{args.workload} stream ({args.mode}); boundaries bit-exact")
    out = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "streams" else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic ({args.workload} generator, seed {hex(SEEDS[args.workload])}+rank, "
                f"generated in HBM before timing)",
        "config": {"workload": f"{args.workload}-{args.size_gib:g}GiB-avg{args.avg}",
                   "stream_bytes_per_gpu": work_bytes, "avg_chunk": args.avg,
                   "parallelism": (f"independent stream per GPU x{world}" if args.mode == "streams"
                                   else f"one stream sharded over {world} GPU(s)"),
                   "chunks_per_stream": ncuts, "candidates_per_stream": cand},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "scan_main_kernel", "avg_launch_ms": round(avg_scan_s * 1e3, 4)},
    }
    if host_incl is not None:
        out["host_inclusive_gib_s"] = round(host_incl, 3)
    if args.digest and args.mode == "streams":
        out["digest"] = digest_stage(args, buf, cuts, stream)
    if args.pipeline_gib > 0 and args.mode == "streams" and world == 1:
        out["pipeline"] = pipeline_stage(args, buf)
    if args.cpu_baseline and world == 1:
        del buf
        out["cpu_baseline"] = cpu_baseline(args, args.workload, SEEDS[args.workload], args.avg)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
