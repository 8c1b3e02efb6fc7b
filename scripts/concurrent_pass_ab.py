"""Does another thread's blob encoding slow a fused pass on its own stream?  One process:
a chunker handle runs fused passes over a 16 GiB VM-image stream (4 MiB average) on stream
A while a second thread encodes compressed blobs (zstd + CRC) of a 2 MiB text/pxar stream
and CRCs its chunks on stream B, in a loop.  Modes, alternated: alone (no second thread),
steady (the work areas kept between calls: no hipMalloc / hipFree, csrc/dev_arena.h) and
churn (pbs_blob_encode_release after every call, so every call allocates and frees its
device buffers again, as before round 4).  Per mode: pass ms (median / p90 / max), the
second thread's calls (paced: one every --side-interval-ms, so both modes do the same
work unless a mode cannot keep the pace), and both results checked.

    python scripts/concurrent_pass_ab.py [--reps 3] [--passes 20]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "proxmox-backup_amd"), os.path.join(ROOT, "tests")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--side-interval-ms", type=float, default=8.0,
                    help="the second thread starts a call every this many ms (the same work in both modes)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import pbschunk
    import corpus_gen

    size = int(a.gib * (1 << 30)) // 8 * 8
    buf = torch.empty(size, dtype=torch.uint8, device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    pbschunk.generate_device(buf.data_ptr(), size, bench.GEN["vmimage"], bench.SEEDS["vmimage"], 0, sa.cuda_stream)
    torch.cuda.synchronize()
    ch = pbschunk.Chunker(4 << 20)
    ch.set_stream(sa.cuda_stream)
    out = torch.empty(ch.cuts_bound(size), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
    ref = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out).copy()
    side = np.concatenate([corpus_gen.text(1 << 20, 7), corpus_gen.pxar(1 << 20, 8)])
    with pbschunk.Chunker(256 << 10) as c2:
        sb_ends = c2.find_cuts(side, is_final=True)
    bounds = np.concatenate([[0], sb_ends]).astype(np.uint64)
    dside = torch.from_numpy(side).to("cuda")
    cap = pbschunk.blob_stream_bound(bounds)
    bout = torch.empty(cap, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ref_blob = pbschunk.blob_encode_chunks_device(dside.data_ptr(), side.size, bounds, bout.data_ptr(), cap,
                                                  hip_stream=sb.cuda_stream)
    ref_img = bout[: int(ref_blob[0][-1])].cpu().numpy().tobytes()
    ref_crc = pbschunk.crc32_chunks_device(dside.data_ptr(), side.size, bounds, hip_stream=sb.cuda_stream)

    def run(mode):
        stop = threading.Event()
        calls, errs = [0], []

        def second():
            try:
                t_next = time.perf_counter()
                while not stop.is_set():
                    t_next += a.side_interval_ms / 1e3
                    dt = t_next - time.perf_counter()
                    if dt > 0:
                        time.sleep(dt)
                    offs, crcs, comp, _ = pbschunk.blob_encode_chunks_device(
                        dside.data_ptr(), side.size, bounds, bout.data_ptr(), cap, hip_stream=sb.cuda_stream)
                    if not np.array_equal(offs, ref_blob[0]) or not np.array_equal(crcs, ref_blob[1]):
                        raise AssertionError("blob result changed")
                    cr = pbschunk.crc32_chunks_device(dside.data_ptr(), side.size, bounds, hip_stream=sb.cuda_stream)
                    if not np.array_equal(cr, ref_crc):
                        raise AssertionError("crc result changed")
                    if mode == "churn":
                        pbschunk.blob_encode_release()
                    calls[0] += 1
            except BaseException as e:  # noqa: BLE001
                errs.append(e)

        th = threading.Thread(target=second) if mode != "alone" else None
        if th:
            th.start()
            time.sleep(0.05)
        ms = []
        for _ in range(a.passes):
            t0 = time.perf_counter()
            got = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
            ms.append((time.perf_counter() - t0) * 1e3)
            assert np.array_equal(got, ref), "cut list changed"
        if th:
            stop.set()
            th.join(timeout=60)
        if errs:
            raise errs[0]
        return ms, calls[0]

    res = {}
    for _ in range(a.reps):
        for mode in ("alone", "steady", "churn"):
            ms, calls = run(mode)
            r = res.setdefault(mode, {"ms": [], "calls": 0})
            r["ms"] += ms
            r["calls"] += calls
    allocs = pbschunk.debug_arena_allocs()
    for mode, r in res.items():
        v = np.array(r["ms"])
        print(json.dumps({"mode": mode, "passes": int(v.size), "median_ms": round(float(np.median(v)), 3),
                          "p90_ms": round(float(np.percentile(v, 90)), 3), "max_ms": round(float(v.max()), 3),
                          "second_thread_calls": r["calls"]}), flush=True)
    print(json.dumps({"arena_allocs_total": allocs, "cuts": int(ref.size), "blob_bytes": len(ref_img)}), flush=True)


if __name__ == "__main__":
    main()
