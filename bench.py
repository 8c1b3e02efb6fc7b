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

``--gpus N`` without a launcher (no WORLD_SIZE in the environment) starts N rank
processes itself (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set per child, 127.0.0.1) before
anything touches the GPU, and fails (exit 2) when fewer than N devices are visible or
when WORLD_SIZE disagrees with --gpus.  ``--cpu-standin`` runs the same launch,
barrier and MAX/SUM aggregation with gloo and the CPU oracle as the step (tests only:
its line says so and is never a GPU measurement).
"""
import argparse
import json
import os
import socket
import subprocess
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
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0 = nproc: every CPU this process may run on)")
    ap.add_argument("--cpu-sample-mib", type=int, default=512,
                    help="bytes each CPU-baseline thread chunks (windows of one shared sample)")
    ap.add_argument("--cpu-config1", type=int, default=1,
                    help="also time BASELINE config 1 on the CPU (1 GiB LE-u32 counter @ 64 KiB, "
                         "1 GiB random @ 4 MiB; 1 thread and nproc threads)")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="TEST ONLY: gloo + the CPU oracle as the step (exercises the N-rank "
                         "launcher and aggregation without a GPU)")
    ap.add_argument("--host-inclusive-gib", type=float, default=4.0,
                    help="also time the host-buffer path (H2D + kernels + D2H) on this many GiB; 0 = skip")
    ap.add_argument("--pinned-out", type=int, default=1,
                    help="1: the timed passes write the cut list into a pinned host array allocated "
                         "once; 0: a pageable array per call (the Python default, A/B)")
    ap.add_argument("--secondary-random", type=int, default=1,
                    help="after the headline, regenerate the same buffer as random data and "
                         "time the pass over it too (a secondary line: no zero extents)")
    ap.add_argument("--blobs", type=int, default=0,
                    help="also time the compressed DataBlob stage (zstd frames + CRC, SURVEY 8(f) rank 4) "
                         "over the stream's chunks, with libzstd level 1 + zlib on the host cores beside it")
    ap.add_argument("--digest", type=int, default=0,
                    help="also time the per-chunk SHA-256 stage (SURVEY 8(f)) over the stream's "
                         "chunks (GPU), with hashlib on the host cores beside it")
    ap.add_argument("--pipeline-gib", type=float, default=0.0,
                    help="also time the host-stream pipeline (copy -> chunk -> SHA-256 per chunk, "
                         "pbs_pipeline_host) over this many GiB of a pageable host copy of the "
                         "stream, with the oracle + hashlib on the host cores beside it")
    ap.add_argument("--upload-gib", type=float, default=0.0,
                    help="also time the client's upload path with compression (pbs_upload_stream_host: "
                         "copy -> chunk -> SHA-256 -> known-chunk test -> zstd blobs of the new chunks -> "
                         "blobs in host memory) over this many GiB, beside the host cores' oracle chunker + "
                         "hashlib + libzstd level 1 + zlib.crc32")
    ap.add_argument("--upload-corpus", choices=["stream", "text", "pxar"], default="stream",
                    help="the upload stage's bytes: the bench stream, or a seeded text-like / pxar-like "
                         "corpus (tests/corpus_gen.py, 32 MiB tiled)")
    ap.add_argument("--stages", type=int, default=-1,
                    help="the SURVEY 8(f) stages after the headline, each with its CPU path and its own "
                         "verification: digest + blob CRC over the 64 GiB stream, the host pipeline and the "
                         "compressing upload over its first --stage-gib GiB, the blob stage, zstd blobs of "
                         "1 GiB text-like and pxar-like corpora, the compressing upload of a 4 GiB text-like "
                         "corpus.  -1 (default): on for one GPU at the default config, off otherwise")
    ap.add_argument("--stage-gib", type=float, default=16.0,
                    help="bytes of the stream's host copy the pipeline and VM-image upload stages take")
    ap.add_argument("--verify", type=int, default=1,
                    help="1: after the timed region compare every rank's cut list (and the "
                         "secondary line's) with tests/golden/bench_cuts.json (oracle-made) and "
                         "exit 3 unless all match; 0: skip (streams without a golden entry)")
    ap.add_argument("--traffic-random-json", default=os.path.join(ROOT, "profiles", "traffic_random.json"),
                    help="the same for the secondary random-data line")
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


def cpu_info():
    """(CPUs this process may run on = nproc, cgroup CPU quota or None, CPU model)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = f.read().split("model name")[1].split("\n")[0].split(":", 1)[-1].strip()
    except (OSError, IndexError):
        pass
    return n, quota, model


def cpu_threads(args) -> int:
    """CPU-baseline threads: --cpu-threads, else the CPUs this process may use -- nproc,
    capped by the cgroup CPU quota where there is one (the GPU box: nproc 256 with a
    16-CPU quota; 256 threads there measured 9.4 GiB/s against ~15 at 16, the quota
    time-slicing them)."""
    if args.cpu_threads > 0:
        return args.cpu_threads
    n, quota, _ = cpu_info()
    return max(1, min(n, int(-(-quota // 1)))) if quota else n


def cpu_mhz():
    """Mean / min / max of the 'cpu MHz' lines of /proc/cpuinfo over the CPUs this process
    may run on (None where the file has none)."""
    try:
        allowed = os.sched_getaffinity(0)
        vals, cpu = [], None
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("processor"):
                    cpu = int(ln.split(":")[1])
                elif ln.startswith("cpu MHz") and cpu in allowed:
                    vals.append(float(ln.split(":")[1]))
        if vals:
            return {"mean": round(sum(vals) / len(vals)), "min": round(min(vals)), "max": round(max(vals)),
                    "cpus": len(vals)}
    except (OSError, ValueError, IndexError):
        pass
    return None


class MhzSampler:
    """cpu_mhz() sampled every 0.25 s on a thread while a CPU timing runs (the host's clock
    under that load: a core sharing its SMT sibling, or held below turbo, shows here)."""

    def __init__(self):
        self.samples, self._stop = [], threading.Event()
        self._th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            m = cpu_mhz()
            if m:
                self.samples.append(m["mean"])
            self._stop.wait(0.25)

    def __enter__(self):
        self._th.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._th.join()

    def summary(self):
        v = self.samples
        return {"mean": round(sum(v) / len(v)), "min": round(min(v)), "max": round(max(v)),
                "samples": len(v)} if v else None


def time_oracle(oracle, avg: int, sample, per: int, threads: int):
    """The oracle (gcc -O2 restatement of chunker.rs) on the host cores: one thread over
    sample[:per], then `threads` threads each over its own `per`-byte window of the
    shared read-only sample (windows start at different offsets: independent streams,
    bounded memory).  Returns (1-thread GiB/s, aggregate GiB/s, 1-thread CPU time / wall
    time: below 1 when the thread was preempted or waited)."""
    t0, c0 = time.perf_counter(), time.thread_time()
    oracle.chunk_feed(avg, sample[:per])
    wall = time.perf_counter() - t0
    single = per / (1 << 30) / wall
    cpu_frac = (time.thread_time() - c0) / wall
    span = sample.size - per
    offs = [(t * span // max(1, threads)) // 4096 * 4096 for t in range(threads)]
    ths = [threading.Thread(target=oracle.chunk_feed, args=(avg, sample[o:o + per])) for o in offs]
    t0 = time.perf_counter()
    [t.start() for t in ths]
    [t.join() for t in ths]  # ctypes releases the GIL
    agg = threads * per / (1 << 30) / (time.perf_counter() - t0)
    return single, agg, cpu_frac


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    return oracle


def cpu_baseline(args, workload, seed, avg):
    """The oracle on the host cores on a bounded sample of the same stream (bench's
    workload, seed, average): nproc threads by default (--cpu-threads)."""
    oracle = _oracle()
    per = args.cpu_sample_mib << 20
    gen = {"counter": lambda n: oracle.gen_counter(n, 0),
           "random": lambda n: oracle.gen_random(n, seed, 0),
           "vmimage": lambda n: oracle.gen_vmimage(n, seed, 0)}[workload]
    sample = gen(2 * per)
    threads = cpu_threads(args)
    with MhzSampler() as mhz:
        single, agg, cpu_frac = time_oracle(oracle, avg, sample, per, threads)
    n, quota, model = cpu_info()
    out = {"value": round(agg, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
           "sample": f"{threads} threads x {args.cpu_sample_mib} MiB windows of one "
                     f"{2 * args.cpu_sample_mib} MiB {workload} sample (seed {hex(seed)}), "
                     f"whole-buffer scan loop (oracle/chunker_oracle.c, gcc -O2); 1 thread: "
                     f"{single:.3f} GiB/s; nproc {n}, os.cpu_count {os.cpu_count()}, cgroup "
                     f"quota {quota if quota is not None else 'none'} CPUs; host CPU: {model}",
           "single_thread_gib_s": round(single, 3), "nproc": n, "cgroup_quota_cpus": quota,
           # what makes two runs' baselines comparable (the single-thread rate
           # moved 0.98 -> 1.61 GiB/s between round-end boxes with the same loop): the build,
           # the host's clock during the timing, and whether the timed thread had its CPU
           "oracle_build": oracle.build_info(), "cpu_mhz_during": mhz.summary(),
           "single_thread_cpu_over_wall": round(cpu_frac, 3)}
    if threads != n and args.cpu_threads <= 0:  # the same at nproc threads, for the record
        _, agg_n, _ = time_oracle(oracle, avg, sample, 64 << 20, n)
        out["nproc_threads"] = {"threads": n, "value": round(agg_n, 3),
                                "sample": f"{n} threads x 64 MiB windows of the same sample"}
    del sample
    return out


def cpu_config1(args):
    """BASELINE config 1 (CPU only): the reference's "pseudo-random" buffer -- 1 GiB
    LE-u32 counter, byte[4i+j] = (i >> 8j) & 0xff (examples/test_chunk_speed.rs:8-14) --
    at its 64 KiB average (:15), and 1 GiB seeded random at the 4 MiB default; the
    oracle with 1 thread over the whole GiB and nproc threads over 512 MiB windows."""
    oracle = _oracle()
    threads = cpu_threads(args)
    out = {"unit": "GiB/s", "threads": threads,
           "reference_published": "about 830MB/s: ChunkStream over 1 GiB of /dev/urandom at "
                                  "4 MiB (examples/test_chunk_speed2.rs:13)"}
    for name, mk, avg in (("counter_1GiB_avg64K", lambda: oracle.gen_counter(1 << 30, 0), 64 << 10),
                          ("random_1GiB_avg4M", lambda: oracle.gen_random(1 << 30, 0x5EED0001, 0), 4 << 20)):
        buf = mk()
        t0 = time.perf_counter()
        cuts = oracle.chunk_feed(avg, buf)
        one = buf.size / (1 << 30) / (time.perf_counter() - t0)
        _, agg, _ = time_oracle(oracle, avg, buf, 512 << 20, threads)
        out[name] = {"1_thread": round(one, 3), "aggregate": round(agg, 3), "chunks": int(cuts.size)}
        del buf
    return out


def traffic_record(path, workload, size, avg, streams=True):
    """(HBM bytes per launch, note) from a PMC traffic record (profiles/collect_traffic.py)
    when it is of this library build and this stream, else (None, why not)."""
    import pbschunk
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC record"
    bid = pbschunk.build_id()
    if tj.get("build_id") != bid:
        return None, f"PMC record is of build {tj.get('build_id')}, this is {bid}: not reported"
    if not (tj.get("size") == size and tj.get("avg") == avg and tj.get("workload") == workload and streams):
        return None, "PMC record is of another workload"
    return tj.get("hbm_bytes_per_launch"), f"rocprofv3 FETCH_SIZE x 1024 x 2, build {bid}"


def secondary_random(args, ch, buf, stream, steps: int = 3):
    """The same-size stream of random bytes (GEN_RANDOM, seed 0x5EED0002) through the same
    handle: every window hashes uniformly, so no zero extents shortcut anything; timed
    like the headline (synchronize around each pass) plus the kernel's HIP-event time."""
    import numpy as np
    import torch

    import pbschunk

    size = buf.numel()
    pbschunk.generate_device(buf.data_ptr(), size, GEN["random"], SEEDS["random"], 0, stream.cuda_stream)
    torch.cuda.synchronize()
    ch.find_cuts_device(buf.data_ptr(), size, is_final=True)  # warm-up
    torch.cuda.synchronize()
    wall, scan, fused, n = [], [], [], 0
    for _ in range(steps):
        t0 = time.perf_counter()
        cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        t = ch.last_timing()
        scan.append(t["scan_ms"])
        fused.append(pass_path(t))
        n = int(cuts.size)
    ms = float(np.mean(wall)) * 1e3
    sk = float(np.mean(scan))
    achieved = size / (sk / 1e3) / 1e9
    rec = {"chunks": n, **cut_record(cuts, keep=0)}
    if args.verify:
        verify_record(rec, "random", size, args.avg, SEEDS["random"])
    traffic, traffic_note = traffic_record(args.traffic_random_json, "random", size, args.avg)
    return {"workload": f"random-{args.size_gib:g}GiB-avg{args.avg}", "seed": hex(SEEDS["random"]),
            "value": round(size / (1 << 30) / (ms / 1e3), 3), "unit": "GiB/s", "steps": steps,
            "ms_per_step": round(ms, 3), **rec,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_note": traffic_note, "kernel": kernel_name(fused), "avg_launch_ms": round(sk, 4)}}


def blob_stage(args, buf, cuts, stream, reps: int = 2):
    """DataBlob::encode(chunk, None, compress = true) for every chunk of
    the device-resident stream (pbs_blob_encode_chunks_device: zstd frames of 64 KiB
    blocks, compressed-or-not per chunk, blob images + CRC), wall clock of the synchronous
    call; libzstd level 1 (the image's 1.4.8) + zlib.crc32 on the host cores over a bounded
    sample of the same chunks beside it, with both compressed sizes of that sample."""
    import zlib

    import numpy as np
    import torch

    import pbschunk

    oracle = _oracle()
    size = buf.numel()
    bounds = np.concatenate([[0], cuts]).astype(np.uint64)
    n = bounds.size - 1
    cap = pbschunk.blob_stream_bound(bounds)
    out = torch.empty(cap, dtype=torch.uint8, device=buf.device)
    pbschunk.blob_encode_chunks_device(buf.data_ptr(), size, bounds, out.data_ptr(), cap,
                                       hip_stream=stream.cuda_stream)  # warm-up (scratch allocation)
    best = None
    for _ in range(reps):
        offs, crcs, comp, tm = pbschunk.blob_encode_chunks_device(buf.data_ptr(), size, bounds, out.data_ptr(), cap,
                                                                  hip_stream=stream.cuda_stream)
        if best is None or tm["total_ms"] < best["total_ms"]:
            best = tm
    # host reference point: libzstd level 1 + crc32 over the first chunks (~1 GiB)
    lens = np.diff(bounds.astype(np.int64))
    take = max(1, min(n, int(np.searchsorted(np.cumsum(lens), 1 << 30)) + 1))
    host = buf[: int(bounds[take])].cpu().numpy()
    L = oracle.libzstd()
    threads = cpu_threads(args)
    sizes = np.zeros(take, dtype=np.int64)

    def work(ix):
        dst = np.empty(L.ZSTD_compressBound(int(lens.max())), dtype=np.uint8)
        for i in ix:
            a, b = int(bounds[i]), int(bounds[i + 1])
            r = L.ZSTD_compress(dst.ctypes.data, dst.size, host.ctypes.data + a, b - a, 1)
            sizes[i] = r
            zlib.crc32(memoryview(dst)[:r])

    parts = [list(range(k, take, threads)) for k in range(threads)]
    ths = [threading.Thread(target=work, args=(ix,)) for ix in parts]
    t0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu_gib_s = int(bounds[take]) / (1 << 30) / (time.perf_counter() - t0)
    ours = int(offs[take]) - 12 * take
    # the sample's blobs through DataBlob's load/decode check; the first two against the twin
    import hashlib
    img = out[: int(offs[take])].cpu().numpy().tobytes()
    ok = True
    for i in range(take):
        ch = host[int(bounds[i]):int(bounds[i + 1])].tobytes()
        blob = img[int(offs[i]):int(offs[i + 1])]
        ok &= oracle.blob_load_decode(blob, hashlib.sha256(ch).digest(), read_sizes=(1 << 17,)) == ch
        ok &= int.from_bytes(blob[8:12], "little") == int(crcs[i])
        if i < 2:
            ok &= blob == oracle.blob_compressed(ch)
    del out
    pbschunk.blob_encode_release()
    return {"metric": "GiB/s chunks -> compressed DataBlob images (zstd frames + CRC, device-resident)",
            "value": round(size / (1 << 30) / (best["total_ms"] / 1e3), 3), "ms": round(best["total_ms"], 3),
            "kernel_ms": {k: round(best[k], 3) for k in ("compress_ms", "assemble_ms", "crc_ms")},
            "chunks": n, "blocks": int(best["blocks"]), "compressed_chunks": int(best["compressed_chunks"]),
            "bytes_in": int(best["bytes_in"]), "bytes_out": int(best["bytes_out"]),
            "ratio_out_in": round(best["bytes_out"] / max(1, best["bytes_in"]), 4),
            "sample_payload_bytes": {"ours": ours, "libzstd_level1": int(sizes.sum()),
                                     "sample": f"first {take} chunks ({int(bounds[take]) >> 20} MiB)"},
            "unit": "GiB/s", "verified": bool(ok),
            "verify_note": f"the first {take} chunks' blobs load + decode (oracle.blob_load_decode) to their "
                           "chunks with the CRCs returned; the first 2 byte-equal to the host twin",
            "parity": "frames decode with libzstd to the chunks (tests); bytes are not libzstd's: unpinned",
            "cpu_baseline": {"value": round(cpu_gib_s, 3), "unit": "GiB/s", "cores": threads,
                             "kind": f"libzstd {L.ZSTD_versionNumber()} level 1 + zlib.crc32 (ctypes)",
                             "sample": f"first {take} chunks ({int(bounds[take]) >> 20} MiB)"}}


def digest_stage(args, buf, cuts, stream, ch=None, reps: int = 3):
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
    # where the GPU-only time goes: each chunk-length class launched alone (HIP events)
    classes = []
    edges = [0, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 12 << 20, 16 << 20, max(int(lens.max()) + 1, (16 << 20) + 1)]
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = order[(lens[order] >= lo) & (lens[order] < hi)]
        if sel.size == 0:
            continue
        oc = torch.from_numpy(sel.astype(np.int32)).to(buf.device)
        ev[0].record(stream)
        pbschunk.digest_chunks_async(buf.data_ptr(), size, bd.data_ptr(), oc.data_ptr(), int(sel.size),
                                     out.data_ptr(), hip_stream=stream.cuda_stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        classes.append({"lo_mib": lo / (1 << 20), "hi_mib": hi / (1 << 20), "chunks": int(sel.size),
                        "gib": round(float(lens[sel].sum()) / (1 << 30), 3),
                        "ms": round(ev[0].elapsed_time(ev[1]), 3)})
    # hybrid: the longest chunks on the host cores (SHA extensions), zero chunks once per
    # length, the rest on the GPU; wall clock of the synchronous call, digests on the host
    threads = cpu_threads(args)
    ref = out.view(n, 32).cpu().numpy()
    hyb = []
    for _ in range(reps):
        dg, tm = pbschunk.digest_chunks_hybrid(buf.data_ptr(), size, bounds, threads=threads,
                                               hip_stream=stream.cuda_stream)
        hyb.append(tm)
    if not np.array_equal(dg, ref):
        raise RuntimeError("hybrid digests differ from the GPU-only digests")
    hb = min(hyb, key=lambda x: x["total_ms"])
    hybrid = {"ms": round(hb["total_ms"], 3), "GiB/s": round(size / (1 << 30) / (hb["total_ms"] / 1e3), 3),
              "sha_ni": pbschunk.sha256_host_uses_ni(),
              **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in hb.items()}}
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
    parts = [list(range(k, take, threads)) for k in range(threads)]

    def work(ix):
        for i in ix:
            hashlib.sha256(mv[int(bounds[i]):int(bounds[i + 1])]).digest()

    ths = [threading.Thread(target=work, args=(ix,)) for ix in parts]
    t0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu_gib_s = int(bounds[take]) / (1 << 30) / (time.perf_counter() - t0)
    # the GPU's digests of the sample's chunks (and the last chunk) against hashlib
    last = buf[int(bounds[n - 1]):int(bounds[n])].cpu().numpy()
    dig_ok = all(bytes(ref[i]) == hashlib.sha256(mv[int(bounds[i]):int(bounds[i + 1])]).digest() for i in range(take))
    dig_ok = dig_ok and bytes(ref[n - 1]) == hashlib.sha256(last).digest()
    crc = crc_stage(args, buf, bd, od, n, bounds, take, threads, stream, reps)
    best = min(t, hb["total_ms"] / 1e3)
    # chunk + digest makespan from HBM (backup_writer.rs:671-678: every chunk of the stream
    # digested): the chunker pass, the chunks ordered longest first, the GPU digest launch,
    # one sync -- the digests must equal the ones above
    span = None
    if ch is not None:
        cut_out = torch.empty(ch.cuts_bound(size), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
        spans, hspans = [], []
        for _ in range(reps):
            # GPU only
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c2 = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=cut_out)
            b2 = np.concatenate([[0], c2]).astype(np.uint64)
            l2 = np.diff(b2.astype(np.int64))
            o2 = np.argsort(-l2, kind="stable").astype(np.int32)
            bd2 = torch.from_numpy(b2.view(np.int64)).to(buf.device, non_blocking=True)
            od2 = torch.from_numpy(o2).to(buf.device, non_blocking=True)
            pbschunk.digest_chunks_async(buf.data_ptr(), size, bd2.data_ptr(), od2.data_ptr(), int(o2.size),
                                         out.data_ptr(), hip_stream=stream.cuda_stream)
            torch.cuda.synchronize()
            spans.append(time.perf_counter() - t0)
            # hybrid: the same pass, then the longest chunks on the host cores (from HBM
            # through the pinned ring) beside the GPU share
            t0 = time.perf_counter()
            c3 = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=cut_out)
            b3 = np.concatenate([[0], c3]).astype(np.uint64)
            dg3, _ = pbschunk.digest_chunks_hybrid(buf.data_ptr(), size, b3, threads=threads,
                                                   hip_stream=stream.cuda_stream)
            hspans.append(time.perf_counter() - t0)
        if not np.array_equal(out.view(n, 32).cpu().numpy(), ref):
            raise RuntimeError("chunk+digest digests differ from the digest stage's")
        if not np.array_equal(dg3, ref):
            raise RuntimeError("chunk+hybrid digest digests differ from the digest stage's")
        best_span = min(min(spans), min(hspans))
        span = {"ms": round(best_span * 1e3, 3), "GiB/s": round(size / (1 << 30) / best_span, 3),
                "gpu_only_ms": round(min(spans) * 1e3, 3), "hybrid_ms": round(min(hspans) * 1e3, 3),
                "what": "find_cuts_device (pinned cut list), then the digests of every chunk, one sync: "
                        "GPU only (longest-first lanes; floor = the pass + the longest chunk's serial SHA "
                        "chain) or hybrid (the longest chunks copied to host cores); ms = the faster"}
    return {"metric": "GiB/s SHA-256 digested (per chunk, device-resident)",
            "value": round(size / (1 << 30) / best, 3), "unit": "GiB/s", "ms": round(best * 1e3, 3), "chunks": n,
            "verified": bool(dig_ok and crc["verified"]),
            "verify_note": f"GPU digests of the first {take} chunks and the last vs hashlib; the hybrid's and "
                           "chunk+digest's equal to the GPU's (else the stage raises); blob CRCs vs zlib",
            "gpu_only": {"ms": round(t * 1e3, 3), "GiB/s": round(size / (1 << 30) / t, 3),
                         "classes": classes},
            "hybrid": hybrid, "chunk_and_digest": span,
            "max_chunk": int(lens.max()), "bound": "valu (GPU: one lane per chunk, serial per chunk); PCIe D2H (hybrid host share)",
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
    got = out[:take].cpu().numpy().view("<u4")
    ok = all(int(got[i]) == zlib.crc32(mv[int(bounds[i]):int(bounds[i + 1])]) for i in range(take))
    return {"metric": "GiB/s blob CRC-32 (per chunk, device-resident)",
            "value": round(size / (1 << 30) / t, 3), "unit": "GiB/s", "ms": round(t * 1e3, 3),
            "verified": bool(ok), "verify_note": f"the first {take} chunks' CRCs vs zlib.crc32",
            "roofline": {"bound": "hbm", "achieved": round(size / t / 1e9, 1), "peak": 8000.0,
                         "unit": "GB/s", "frac": round(size / t / 8e12, 4)},
            "cpu_baseline": {"value": round(cpu, 3), "unit": "GiB/s", "cores": threads,
                             "kind": "zlib.crc32 (same CRC-32 as crc32fast)",
                             "sample": f"first {take} chunks ({int(bounds[take]) >> 20} MiB)"}}


def pipeline_stage(args, buf, piece: int = 1 << 30, host=None):
    """a pageable host copy of the stream's first --pipeline-gib GiB
    through pbs_pipeline_host (copy thread -> HBM, chunker on CU-masked stream, per-chunk
    SHA-256 and blob CRC-32 on the other CUs, overlapped), end to end; the CPU path beside
    it: the oracle chunker + hashlib + zlib.crc32 per chunk on the host cores over a
    bounded sample."""
    import hashlib
    import zlib

    import numpy as np

    import pbschunk

    oracle = _oracle()

    if host is None:
        n = int(args.pipeline_gib * (1 << 30)) // 8 * 8
        host = buf[:n].cpu().numpy()  # pageable, untimed
    n = host.size
    # warm-up at full size: the first call also allocates the device work area (kept
    # between calls), reported as first_call; the timed call is the steady state
    t0 = time.perf_counter()
    cold = pbschunk.pipeline_host(host, args.avg, piece=piece, crc=True)
    cold_wall = time.perf_counter() - t0
    t0 = time.perf_counter()
    ends, dig, crcs, t = pbschunk.pipeline_host(host, args.avg, piece=piece, crc=True)
    wall = time.perf_counter() - t0
    same = all(np.array_equal(a, b) for a, b in zip(cold[:3], (ends, dig, crcs)))
    del cold
    cuts = verify_record({"chunks": int(ends.size), **cut_record(ends, keep=0)}, args.workload, n, args.avg,
                         SEEDS[args.workload])
    # CPU path: threads chunk their own slice and hash its chunks (hashlib/OpenSSL)
    threads = cpu_threads(args)
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
    # digests and CRCs of a sample of chunks (the first 32 and the last) against hashlib / zlib
    bnd = np.concatenate([[0], ends]).astype(np.int64)
    pick = list(range(min(32, ends.size))) + [int(ends.size) - 1]
    mv = memoryview(host)
    sample_ok = all(bytes(dig[i]) == hashlib.sha256(mv[bnd[i]:bnd[i + 1]]).digest() and
                    int(crcs[i]) == zlib.crc32(mv[bnd[i]:bnd[i + 1]]) for i in pick)
    return {"metric": "GiB/s host stream -> chunk boundaries + SHA-256 + blob CRC-32 per chunk (end to end)",
            "verified": bool(cuts["verified"] is True and sample_ok and same),
            "verify_note": "cut list vs tests/golden/bench_cuts.json (oracle); digests + CRCs of "
                           f"{len(pick)} chunks vs hashlib / zlib; same result as the first call",
            "value": round(n / (1 << 30) / wall, 3), "bytes": n, "piece": piece,
            "first_call": {"value": round(n / (1 << 30) / cold_wall, 3),
                           "note": "same stream, first call: includes allocating the device work area",
                           "same_result": same},
            "chunks": int(ends.size), "cuts": cuts, "timing_ms": {k: round(v, 2) for k, v in t.items()
                                                     if k.endswith("_ms")},
            "host_share": {"chunks": t["host_chunks"], "gib": round(t["host_bytes"] / (1 << 30), 3),
                           "threads": t["host_threads"],
                           "routing": (f"fixed: chunks >= {os.environ['PBS_PIPE_HOST_MIN']} B"
                                       if "PBS_PIPE_HOST_MIN" in os.environ else
                                       "deadline: the GPU when its SHA-256 chain ends before the copy does")},
            "digest_queue": {"gpu_jobs": t["gpu_jobs"], "claimed": t["gpu_claimed"],
                             "launches": t["queue_launches"], "gpu_done_ms": round(t["gpu_done_ms"], 2),
                             "host_work_ms": round(t["host_work_ms"], 2)},
            "cpu_baseline": {"value": round(cpu, 3), "unit": "GiB/s", "cores": nth,
                             "kind": "port (oracle chunker) + hashlib + zlib.crc32",
                             "sample": f"{nth} x 256 MiB slices: chunk_feed then sha256 + crc32 per chunk"}}


def corpus_host(name: str, n: int, base=None):
    """A seeded text-like / pxar-like corpus (tests/corpus_gen.py, 32 MiB) tiled to n bytes;
    every 4 KiB page of every tile but the first stamped with its page number (8 bytes at
    the page start): the tiles stop repeating each other's chunks, so the known-chunk test
    finds no duplicates and every chunk is compressed, at ~0.2 % of the bytes."""
    import numpy as np

    if base is None:
        base = corpus_base(name)
    host = np.tile(base, -(-n // base.size))[:n]
    pages = host[base.size:].reshape(-1)[: (n - base.size) // 4096 * 4096].reshape(-1, 4096)
    pages[:, :8] = np.arange(1, pages.shape[0] + 1, dtype="<u8").view(np.uint8).reshape(-1, 8)
    return host, (f"{name}-like corpus (tests/corpus_gen.py seed {CORPUS_SEEDS[name]}, 32 MiB tiled, every later "
                  f"4 KiB page stamped with its number)")


CORPUS_SEEDS = {"text": 21, "pxar": 22}


def corpus_base(name: str):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import corpus_gen
    return {"text": corpus_gen.text, "pxar": corpus_gen.pxar}[name](32 << 20, CORPUS_SEEDS[name])


def upload_stage(args, host, what: str, piece: int = 1 << 30, golden=None):
    """backup_writer.rs:631-706 with compress = true (proxmox-backup-client main.rs:1011-1016)
    from a pageable host buffer to the new chunks' blobs in (pinned) host memory, through
    pbs_upload_stream_host; the CPU path beside it over a bounded sample: the oracle
    chunker, hashlib SHA-256, libzstd level 1 (the reference's compressor, data_blob.rs:151;
    the image's 1.4.8) and zlib.crc32 per chunk on the host cores.  Verified after the
    timing: the cut list (against `golden` = (workload, seed) of tests/golden/bench_cuts.json,
    else against the oracle run over the same bytes), the first new chunks' blobs against
    the host twin's, their zstd payloads through libzstd and DataBlob's load/decode check
    (oracle.blob_load_decode) with the upload's own digests."""
    import hashlib
    import zlib

    import numpy as np
    import torch

    import pbschunk

    oracle = _oracle()
    n = host.size
    cap = n // max(args.avg >> 2, 65) + 4
    blobs = torch.empty(12 * cap + n, dtype=torch.uint8, pin_memory=True).numpy()
    cold = pbschunk.upload_stream_host(host, args.avg, piece=piece, blobs_out=blobs)  # allocations
    t0 = time.perf_counter()
    out = pbschunk.upload_stream_host(host, args.avg, piece=piece, blobs_out=blobs)
    wall = time.perf_counter() - t0
    same = (np.array_equal(cold["ends"], out["ends"]) and np.array_equal(cold["digests"], out["digests"])
            and np.array_equal(cold["blob_offsets"], out["blob_offsets"]))
    del cold
    rec = {"chunks": int(out["ends"].size), **cut_record(out["ends"], keep=0)}
    if golden is not None:
        cuts = verify_record(rec, golden[0], n, args.avg, golden[1])
    else:  # the oracle over the same bytes (every cut, the tail appended as find_cuts does)
        ref = oracle.chunk_feed(args.avg, host)
        if ref.size == 0 or int(ref[-1]) != n:
            ref = np.append(ref, np.uint64(n))
        cuts = {**rec, "verified": bool(np.array_equal(ref, out["ends"])),
                "verify_note": "against oracle.chunk_feed over the same host bytes"}
    # the first new chunks' blobs against the host twin's (oracle.blob_compressed), and the
    # reference's own check of a blob (load: magic + CRC; decode; digest)
    checked, blobs_ok = 0, True
    offs = out["blob_offsets"]
    for i in np.flatnonzero(out["known"] == 0)[:3]:
        s0 = int(out["ends"][i - 1]) if i else 0
        chunk = host[s0:int(out["ends"][i])].tobytes()
        blob = out["blobs"][int(offs[i]):int(offs[i + 1])].tobytes()
        blobs_ok &= blob == oracle.blob_compressed(chunk)
        blobs_ok &= bytes(out["digests"][i]) == hashlib.sha256(chunk).digest()
        blobs_ok &= oracle.blob_load_decode(blob, bytes(out["digests"][i]), read_sizes=(1 << 17,)) == chunk
        checked += 1
    t = out["timing"]
    # CPU path: every thread chunks its own slice, then SHA-256 + libzstd-1 + CRC per chunk
    L = oracle.libzstd()
    threads = cpu_threads(args)
    per = 128 << 20
    nth = min(threads, max(1, n // per))

    def work(k):
        sl = np.ascontiguousarray(host[k * per:(k + 1) * per])
        cc = oracle.chunk_feed(args.avg, sl)
        b = np.concatenate([[0], cc, [sl.size]]).astype(np.int64)
        mv = memoryview(sl)
        dst = np.empty(L.ZSTD_compressBound(int(np.diff(b).max())), np.uint8)
        for i in range(b.size - 1):
            if b[i + 1] > b[i]:
                hashlib.sha256(mv[b[i]:b[i + 1]]).digest()
                r = L.ZSTD_compress(dst.ctypes.data, dst.size, sl.ctypes.data + int(b[i]), int(b[i + 1] - b[i]), 1)
                zlib.crc32(memoryview(dst)[:r])

    ths = [threading.Thread(target=work, args=(k,)) for k in range(nth)]
    c0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu = nth * per / (1 << 30) / (time.perf_counter() - c0)
    st = out["stats"]
    return {"metric": "GiB/s host stream -> chunks + SHA-256 + known-chunk test + compressed blobs of the new "
                      "chunks in host memory (end to end, backup_writer.rs:631-706 with compress = true)",
            "value": round(n / (1 << 30) / wall, 3), "unit": "GiB/s", "wall_ms": round(wall * 1e3, 2), "bytes": n,
            "data": what, "piece": piece,
            "verified": bool(cuts["verified"] is True and blobs_ok and same),
            "chunks": int(out["ends"].size), "cuts": cuts, "same_result_as_first_call": same,
            "blobs_checked_against_twin_and_decoded": checked,
            "upload_stats": st, "compressed_over_new": round(st["size_compressed"] / max(1, st["size"] - st["size_reused"]), 4),
            "compressed_chunks": t["compressed_chunks"],
            "pipeline_detail_ms": {k: (round(v, 2) if isinstance(v, float) else v) for k, v in t["pipe"].items()},
            "timing_ms": {"total": round(t["total_ms"], 2), "pipeline": round(t["pipe"]["total_ms"], 2),
                          "h2d": round(t["pipe"]["h2d_ms"], 2), "known": round(t["known_ms"], 2),
                          "encode": round(t["encode_ms"], 2), "blobs_d2h": round(t["d2h_ms"], 2),
                          "zstd_blocks": round(t["blob"]["compress_ms"], 2)},
            "cpu_baseline": {"value": round(cpu, 3), "unit": "GiB/s", "cores": nth,
                             "kind": "port (oracle chunker) + hashlib + libzstd level 1 + zlib.crc32",
                             "libzstd_version": int(L.ZSTD_versionNumber()),
                             "sample": f"{nth} x {per >> 20} MiB slices: chunk_feed then sha256 + zstd-1 + crc32 per chunk"}}


def zstd_stage(args, name: str, base, gib: float = 1.0, reps: int = 3):
    """SURVEY 8(f) rank 4 on compressible data: DataBlob::encode(chunk, None, true)
    (data_blob.rs:139-176; zstd level 1 in the reference, :151) of every chunk of a
    seeded text-like / pxar-like corpus (32 MiB tiled to `gib` GiB in HBM, a chunk's
    window never reaches a neighbouring tile), cut by the GPU chunker; wall clock of the
    synchronous pbs_blob_encode_chunks_device, best of `reps`.  Beside it libzstd level 1
    + zlib.crc32 over every chunk on the host cores.  Verified: the payloads within 10 %
    of libzstd-1's over the first 64 MiB of chunks, the first two blobs byte-equal to the
    host twin's, and every blob of that sample through DataBlob's load/decode check."""
    import hashlib
    import zlib

    import numpy as np
    import torch

    import pbschunk

    oracle = _oracle()
    n = int(gib * (1 << 30)) // base.size * base.size
    host = np.tile(base, n // base.size)
    dev = torch.from_numpy(host).to("cuda")
    with pbschunk.Chunker(args.avg) as c:
        ends = c.find_cuts_device(dev.data_ptr(), n, is_final=True)
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    cap = pbschunk.blob_stream_bound(bounds)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)  # warm-up
    best = None
    for _ in range(reps):
        offs, crcs, comp, tm = pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)
        if best is None or tm["total_ms"] < best["total_ms"]:
            best = tm
    L = oracle.libzstd()
    take = max(1, int(np.searchsorted(bounds, 64 << 20)))
    img = out[: int(offs[take])].cpu().numpy().tobytes()
    ours = int(offs[take]) - 12 * take
    ref, ok = 0, True
    for i in range(take):
        ch = np.ascontiguousarray(host[int(bounds[i]):int(bounds[i + 1])])
        dst = np.empty(L.ZSTD_compressBound(ch.size), np.uint8)
        ref += L.ZSTD_compress(dst.ctypes.data, dst.size, ch.ctypes.data, ch.size, 1)
        blob = img[int(offs[i]):int(offs[i + 1])]
        ok &= oracle.blob_load_decode(blob, hashlib.sha256(ch).digest(), read_sizes=(1 << 17,)) == ch.tobytes()
        ok &= struct_crc(blob) == int(crcs[i])
        if i < 2:
            ok &= blob == oracle.blob_compressed(ch.tobytes())
    nb = int(bounds.size - 1)
    threads = cpu_threads(args)
    lens = np.diff(bounds.astype(np.int64))

    def work(ix):
        dst = np.empty(L.ZSTD_compressBound(int(lens.max())), np.uint8)
        for i in ix:
            a0, b0 = int(bounds[i]), int(bounds[i + 1])
            r = L.ZSTD_compress(dst.ctypes.data, dst.size, host.ctypes.data + a0, b0 - a0, 1)
            zlib.crc32(memoryview(dst)[:r])

    ths = [threading.Thread(target=work, args=(list(range(k, nb, threads)),)) for k in range(threads)]
    h0 = time.perf_counter()
    [x.start() for x in ths]
    [x.join() for x in ths]
    cpu = n / (1 << 30) / (time.perf_counter() - h0)
    del dev, out
    pbschunk.blob_encode_release()
    ratio = ours / max(1, ref)
    return {"metric": f"GiB/s chunks -> compressed DataBlob images (zstd frames + CRC, device-resident), {name}-like corpus",
            "value": round(n / (1 << 30) / (best["total_ms"] / 1e3), 3), "unit": "GiB/s", "bytes": n,
            "data": f"{name}-like corpus (tests/corpus_gen.py seed {CORPUS_SEEDS[name]}, 32 MiB tiled)",
            "chunks": nb, "ms": {k: round(best[k], 3) for k in ("total_ms", "compress_ms", "assemble_ms", "crc_ms")},
            "out_in": round(best["bytes_out"] / n, 4),
            "sample_payload": {"ours": ours, "libzstd_level1": ref, "ratio": round(ratio, 4), "chunks": take},
            "verified": bool(ok and ratio <= 1.10),
            "verify_note": f"the first {take} chunks' blobs load + decode to their chunks (DataBlob load/decode, "
                           "oracle.blob_load_decode) with the CRCs returned; the first 2 byte-equal to the host twin; "
                           "payload <= 1.10 x libzstd level 1 over them",
            "cpu_baseline": {"value": round(cpu, 3), "unit": "GiB/s", "cores": threads,
                             "kind": f"libzstd {L.ZSTD_versionNumber()} level 1 + zlib.crc32 (ctypes)",
                             "sample": f"all {nb} chunks of the corpus"}}


def struct_crc(blob: bytes) -> int:
    return int.from_bytes(blob[8:12], "little")


def free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def kfd_gpu_count():
    """GPUs visible to this process, counted without any HIP/torch call: the KFD topology
    nodes with SIMDs (CPU nodes have simd_count 0), narrowed by the *_VISIBLE_DEVICES
    lists the ROCm runtime honours.  None when the topology is not readable (the rank
    processes then check for themselves)."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(root, node, "properties")) as f:
                props = dict(ln.split(None, 1) for ln in f if ln.strip() and len(ln.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: N rank processes of this script (one per GPU),
    started before anything touches the GPU -- this parent makes no HIP or torch.cuda
    call at all (the GPU count comes from the KFD topology in sysfs, and every rank
    checks its own device again); returns the job's exit code.  A rank that fails ends
    the others (they would wait in the barrier)."""
    n = args.gpus
    share = os.environ.get("PBS_BENCH_SHARE_GPU") == "1"
    if not args.cpu_standin and not share:
        have = kfd_gpu_count()
        if have is not None and have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if args.cpu_standin or share:  # gloo on the loopback device (the hostname may not resolve)
            env.setdefault("GLOO_SOCKET_IFNAME", "lo")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:
                    q.kill()  # our own children, by PID
        time.sleep(0.1)
    return rc


def pass_path(t: dict) -> str:
    """Which path a pass took (last_timing): the one-launch fused pass, the scan pass
    (scan_fused_kernel without resolver waves + gather + multi-kernel resolve) or the
    multi-launch path (scan_main_kernel + scan_exact + sort + resolve)."""
    if t["bytes"] > 0 and t["scan_pass"] == t["bytes"]:
        return "scan_pass"
    if t["bytes"] > 0 and t["fused"] == t["bytes"]:
        return "fused"
    return "multi"


def kernel_name(paths) -> str:
    """The dominant kernel of the timed passes (the roofline's kernel)."""
    if paths and all(p == "fused" for p in paths):
        return "scan_fused_kernel"
    if paths and all(p == "scan_pass" for p in paths):
        return "scan_fused_kernel (scan pass)"
    return "scan_main_kernel"


def timed_steps(step, args, dist, sync, after=None):
    """W untimed warm-up steps, then exactly K steps bracketed by a barrier + device sync
    on both sides.  Returns (this rank's elapsed seconds, last step's result)."""
    for _ in range(args.warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
        if after:
            after(res)
    sync()
    if dist:
        dist.barrier()
    return time.perf_counter() - t0, res


def cut_record(cuts, keep: int = 8192) -> dict:
    """A rank's cut list (chunk END offsets, the stream end included) for the per-rank
    record: its SHA-256 over the u64 LE values, and the list itself when it is short (the
    multi-rank tests diff each rank's list against the oracle)."""
    import hashlib

    import numpy as np

    c = np.ascontiguousarray(np.asarray(cuts, dtype=np.uint64))
    out = {"cuts_sha256": hashlib.sha256(c.astype("<u8").tobytes()).hexdigest()}
    if c.size <= keep:
        out["cuts"] = [int(x) for x in c]
    return out


# PBS_BENCH_GOLDEN: another golden file (tests: a corrupted copy must fail verification)
GOLDEN = os.environ.get("PBS_BENCH_GOLDEN", os.path.join(ROOT, "tests", "golden", "bench_cuts.json"))
_golden = None


def golden_entry(workload: str, size: int, avg: int, seed: int):
    """The oracle-made record of this stream (tests/golden/make_bench_golden.py), or None."""
    global _golden
    if _golden is None:
        try:
            with open(GOLDEN) as f:
                _golden = json.load(f)["streams"]
        except (OSError, ValueError, KeyError):
            _golden = {}
    return _golden.get(f"{workload}:{size}:{avg}:{seed:#x}")


def verify_record(rec: dict, workload: str, size: int, avg: int, seed: int) -> dict:
    """Compares a timed cut list's record (cut_record) with the golden one: adds
    "verified" True / False, or None with "verify_note" when no golden entry exists."""
    g = golden_entry(workload, size, avg, seed)
    if g is None:
        rec["verified"] = None
        rec["verify_note"] = (f"no golden entry for {workload}:{size}:{avg}:{seed:#x} in "
                              f"tests/golden/bench_cuts.json")
    else:
        rec["verified"] = bool(g["cuts_sha256"] == rec["cuts_sha256"] and g["chunks"] == rec["chunks"])
        if not rec["verified"]:
            rec["verify_note"] = (f"cut list differs from the oracle's: {rec['chunks']} chunks, sha "
                                  f"{rec['cuts_sha256'][:16]} vs {g['chunks']}, {g['cuts_sha256'][:16]}")
    return rec


def verdict(recs, extra=()) -> bool:
    """True when every rank's (and every extra line's) cut list equals its golden one."""
    return all(r.get("verified") is True for r in list(recs) + list(extra))


def device_identity(torch, dev) -> dict:
    """The GPU a rank ran on, as the runtime names it: PCI domain:bus:device, UUID, name --
    an 8-rank line shows on its own that 8 distinct devices did the work."""
    p = torch.cuda.get_device_properties(dev)
    out = {"index": dev.index, "name": p.name, "arch": getattr(p, "gcnArchName", None)}
    if hasattr(p, "pci_bus_id"):
        out["pci"] = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}"
    if hasattr(p, "uuid"):
        out["uuid"] = str(p.uuid)
    return out


def per_rank_records(rec: dict, dist, world: int):
    if dist is None:
        return [rec]
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out


def base_line(args, metric, value, world, elapsed, scaling, dtype, data, config):
    return {"metric": metric, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": dtype, "data": data, "config": config}


def standin_main(args, world: int, rank: int):
    """TEST ONLY (--cpu-standin): the launcher, barrier and MAX/SUM aggregation of the GPU
    path with gloo, every rank chunking its own stream (seed + rank) with the CPU oracle."""
    import torch

    oracle = _oracle()
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    size = int(args.size_gib * (1 << 30)) // 8 * 8
    seed = stream_seed(args.workload, rank)
    buf = {"counter": lambda: oracle.gen_counter(size, 0),
           "random": lambda: oracle.gen_random(size, seed, 0),
           "vmimage": lambda: oracle.gen_vmimage(size, seed, 0)}[args.workload]()
    import numpy as np

    def step():  # find_cuts(..., is_final=True)'s list: the stream end when the tail is non-empty
        c = oracle.chunk_feed(args.avg, buf)
        return np.append(c, np.uint64(size)) if size and (c.size == 0 or int(c[-1]) != size) else c
    elapsed, cuts = timed_steps(step, args, dist, lambda: None)
    import socket
    rec = {"rank": rank, "seed": seed, "elapsed_s": elapsed, "bytes": size, "world_size": world,
           "device": {"kind": "cpu-standin", "host": socket.gethostname(), "pid": os.getpid()},
           "avg_launch_ms": round(elapsed / max(1, args.steps) * 1e3, 4),  # (an oracle pass)
           "chunks": int(cuts.size), **cut_record(cuts)}
    if args.verify:
        verify_record(rec, args.workload, size, args.avg, seed)
    recs = per_rank_records(rec, dist, world)
    mx, total = aggregate(elapsed, size, dist, torch.device("cpu"))
    if rank == 0:
        out = base_line(args, "STAND-IN (CPU oracle over gloo, not a GPU measurement): GiB/s chunked",
                        total * args.steps / (1 << 30) / mx, world, mx, "weak", "u8",
                        f"synthetic ({args.workload}, seed {hex(SEEDS[args.workload])}+rank)",
                        {"workload": f"{args.workload}-{args.size_gib:g}GiB-avg{args.avg}",
                         "stream_bytes_per_rank": size})
        out["stand_in"] = True
        out["per_rank"] = recs
        if args.verify:
            out["verified"] = verdict(recs)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if args.verify and not verdict(recs):
        sys.exit(3)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu_standin:
        standin_main(args, world, rank)
        return
    import numpy as np
    import torch

    # TEST ONLY (PBS_BENCH_SHARE_GPU=1): every rank on GPU 0 and gloo instead of RCCL -- a
    # rehearsal of the N-rank GPU path on a one-GPU box (the ranks share one HBM, so the
    # line is not a scaling measurement and says so)
    share = world > 1 and os.environ.get("PBS_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0  # (--mode sharded stages its all-gathers through host memory: shard.py)
    if torch.cuda.device_count() < (1 if share else max(world, local + 1)):
        print(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible",
              file=sys.stderr)
        sys.exit(2)
    dist = None
    # TEST ONLY (PBS_BENCH_DIST_WORLD1=1, under torch.distributed.run): a one-rank job still
    # creates its RCCL group, so the device-tensor barrier / all-reduce / all-gather path of
    # the multi-GPU run executes on a one-GPU box (tests/test_dist.py)
    if world > 1 or (world == 1 and env_world is not None and os.environ.get("PBS_BENCH_DIST_WORLD1") == "1"):
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    red_dev = torch.device("cpu") if share else dev  # gloo reduces CPU tensors

    import pbschunk

    size = int(args.size_gib * (1 << 30)) // 8 * 8
    stream = torch.cuda.current_stream()
    ch = pbschunk.Chunker(args.avg)
    ch.set_stream(stream.cuda_stream)
    if args.mode == "sharded":
        import shard
        seed = SEEDS[args.workload]  # one stream; this rank generates its range of it
        base, local_len = shard.shard_ranges(size, world)[rank]
        buf = torch.empty(local_len, dtype=torch.uint8, device=dev)
        pbschunk.generate_device(buf.data_ptr(), local_len, GEN[args.workload], seed, base,
                                 stream.cuda_stream)
        torch.cuda.synchronize()
        ptr, tail = buf.data_ptr(), buf[max(0, local_len - shard.HALO):]

        def step():
            return shard.chunk_sharded(ch, ptr, local_len, base, size, tail, dist, rank, world, dev)
        work_bytes = local_len
    else:
        seed = stream_seed(args.workload, rank)
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        pbschunk.generate_device(buf.data_ptr(), size, GEN[args.workload], seed, 0,
                                 stream.cuda_stream)
        torch.cuda.synchronize()
        ptr = buf.data_ptr()
        # the cut list lands in a pinned host array allocated once (DMA straight into it; a
        # pageable one is staged through a bounce buffer and then copied: ~6 MB per pass
        # at 64 KiB averages)
        cut_out = None
        if args.pinned_out:
            cut_out = torch.empty(ch.cuts_bound(size), dtype=torch.int64,
                                  pin_memory=True).numpy().view(np.uint64)

        def step():
            return ch.find_cuts_device(ptr, size, is_final=True, out=cut_out)
        work_bytes = size

    scan_ms, last, fused = [], {}, []

    def after(cuts):
        t = ch.last_timing()
        scan_ms.append(t["scan_ms"])
        fused.append(pass_path(t))
        last.update(t, ncuts=int(cuts.size))

    elapsed, cuts = timed_steps(step, args, dist, torch.cuda.synchronize, after)
    # after the timed region: this rank's last timed cut list against the oracle's golden
    # record of the same stream (tests/golden/bench_cuts.json)
    rec = {"rank": rank, "seed": seed, "elapsed_s": round(elapsed, 6), "bytes": work_bytes,
           "world_size": dist.get_world_size() if dist is not None else 1,
           "device": device_identity(torch, dev),
           # this rank's own kernel time (HIP events around the pass's launch), beside the
           # line's roofline, which is rank 0's
           "avg_launch_ms": round(float(np.mean(scan_ms)), 4) if scan_ms else None,
           "chunks": int(cuts.size), **cut_record(cuts)}
    if args.verify:
        verify_record(rec, args.workload, size, args.avg, seed)
    recs = per_rank_records(rec, dist, world)
    elapsed, total_bytes = aggregate(elapsed, work_bytes, dist, red_dev)

    value = total_bytes * args.steps / (1 << 30) / elapsed
    avg_scan_s = float(np.mean(scan_ms)) / 1e3 if scan_ms else float("nan")
    achieved = work_bytes / avg_scan_s / 1e9  # algorithmic bytes (input read once) per launch
    traffic, traffic_note = traffic_record(args.traffic_json, args.workload, work_bytes, args.avg,
                                           args.mode == "streams")
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
        if args.verify and not verdict(recs):
            sys.exit(3)
        return
    default_cfg = (args.size_gib == 64.0 and args.avg == 4 * 1024 * 1024
                   and args.workload == "vmimage" and args.mode == "streams")
    metric = METRIC if default_cfg and not share else ("REHEARSAL (ranks share one GPU, gloo): " if share else "") + (
        f"GiB/s chunked (device-resident), {args.avg >> 10} KiB mean, {args.size_gib:g} GiB "
        f"{args.workload} stream ({args.mode}); boundaries bit-exact")
    out = base_line(
        args, metric, value, world, elapsed, "weak" if args.mode == "streams" else "strong", "u8",
        f"synthetic ({args.workload} generator, seed {hex(SEEDS[args.workload])}+rank, "
        f"generated in HBM before timing)",
        {"workload": f"{args.workload}-{args.size_gib:g}GiB-avg{args.avg}",
         "stream_bytes_per_gpu": work_bytes, "avg_chunk": args.avg,
         "parallelism": (f"independent stream per GPU x{world}" if args.mode == "streams"
                         else f"one stream sharded over {world} GPU(s)"),
         "chunks_per_stream": last.get("ncuts", 0),
         "candidates_per_stream": int(last.get("candidates", 0))})
    out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                       "traffic_note": traffic_note,
                       "kernel": kernel_name(fused),
                       "avg_launch_ms": round(avg_scan_s * 1e3, 4)}
    out["build_id"] = pbschunk.build_id()
    if share:
        out["rehearsal"] = "TEST ONLY: all ranks on GPU 0 over gloo; not a scaling measurement"
    out["per_rank"] = recs
    if dist is not None:
        out["backend"] = dist.get_backend()
    if host_incl is not None:
        out["host_inclusive_gib_s"] = round(host_incl, 3)
    stages = args.stages if args.stages >= 0 else int(default_cfg and world == 1 and not share)
    if stages and (world != 1 or args.mode != "streams"):
        stages = 0  # the f-stages are one-GPU measurements
    if stages:
        out["stages_note"] = ("SURVEY 8(f) stages after the headline's timed region, each with its CPU path "
                              "and its own verification; none of them changes value / roofline / cpu_baseline")
    if (args.digest or stages) and args.mode == "streams":
        out["digest"] = digest_stage(args, buf, cuts, stream, ch=ch if args.mode == "streams" else None)
    stage_host = None
    if stages:  # one pageable host copy of the stream's prefix for the pipeline and the upload
        stage_host = buf[: int(args.stage_gib * (1 << 30)) // 8 * 8].cpu().numpy()
    if (args.pipeline_gib > 0 or stages) and args.mode == "streams" and world == 1:
        out["pipeline"] = pipeline_stage(args, buf, host=stage_host)  # before the blob stage's 64 GiB scratch
    if stages:
        pbschunk.pipeline_release()
        out["upload_vm"] = upload_stage(args, stage_host, f"{args.workload} stream prefix (seed "
                                        f"{hex(SEEDS[args.workload])})", golden=(args.workload, SEEDS[args.workload]))
        del stage_host
        pbschunk.pipeline_release()
    if (args.blobs or stages) and args.mode == "streams":
        out["blobs"] = blob_stage(args, buf, cuts, stream)
    if args.secondary_random and args.mode == "streams" and world == 1 and args.workload != "random":
        out["secondary_random"] = secondary_random(args, ch, buf, stream)
    if stages:
        ch.close()
        del buf
        torch.cuda.empty_cache()
        bases = {}
        for name in ("text", "pxar"):
            bases[name] = corpus_base(name)
            out[f"zstd_{name}"] = zstd_stage(args, name, bases[name])
            torch.cuda.empty_cache()
        host, what = corpus_host("text", 4 << 30, bases["text"])
        out["upload_text"] = upload_stage(args, host, what)
        del host, bases
        pbschunk.pipeline_release()
    elif args.upload_gib > 0 and args.mode == "streams" and world == 1:
        # (the last GPU stage: a 64 GiB upload holds the stream copy, the blob slots and the
        # blobs in HBM at once, so the bench stream goes first)
        n = int(args.upload_gib * (1 << 30)) // 8 * 8
        if args.upload_corpus == "stream":
            host, what, golden = buf[:n].cpu().numpy(), f"{args.workload} stream (seed {hex(SEEDS[args.workload])})", \
                (args.workload, SEEDS[args.workload])
        else:
            (host, what), golden = corpus_host(args.upload_corpus, n), None
        buf.set_()
        torch.cuda.empty_cache()
        pbschunk.blob_encode_release()
        pbschunk.pipeline_release()
        out["upload"] = upload_stage(args, host, what, golden=golden)
        del host
    if args.cpu_baseline:  # (rank 0 only: the other ranks have returned; after every timed region)
        buf = None
        out["cpu_baseline"] = cpu_baseline(args, args.workload, SEEDS[args.workload], args.avg)
        if args.cpu_config1:
            out["cpu_config1"] = cpu_config1(args)
    extra = [out["secondary_random"]] if "secondary_random" in out else []
    if "pipeline" in out and out["pipeline"]["cuts"]["verified"] is not None:  # a golden stream length
        extra.append(out["pipeline"]["cuts"])
    for k in ("upload", "upload_vm", "upload_text"):
        if k in out and out[k]["cuts"]["verified"] is not None:
            extra.append(out[k]["cuts"])
    # every stage's own verification (digests, CRCs, blobs, cut lists)
    for k in ("digest", "pipeline", "upload_vm", "blobs", "zstd_text", "zstd_pxar", "upload_text"):
        if k in out and out[k].get("verified") is not True:
            extra.append({"verified": out[k].get("verified"), "stage": k})
    if args.verify:
        # every timed cut list (each rank's, the secondary line's) equals the oracle's
        out["verified"] = verdict(recs, extra)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if args.verify and not out["verified"]:
        print("bench.py: a timed cut list is not verified against tests/golden/bench_cuts.json "
              "(see per_rank / secondary_random verify_note; --verify 0 for streams without a "
              "golden entry)", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
