"""Where a scan pass's time goes beyond its kernel (small averages): per pass
the wall time of find_cuts_device into a pinned cut array, the scan kernel, the gather and
the resolve (HIP events, pbs_timing), for the given averages x kinds at 64 GiB.

    python scripts/scan_pass_split.py [--kinds vmimage,random] [--avgs 65536,131072,262144]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proxmox-backup_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="vmimage,random")
    ap.add_argument("--avgs", default="65536,131072,262144")
    ap.add_argument("--size-gib", type=float, default=64.0)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    import numpy as np
    import torch
    import pbschunk

    size = int(a.size_gib * (1 << 30)) // 8 * 8
    buf = torch.empty(size, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    for kind in a.kinds.split(","):
        pbschunk.generate_device(buf.data_ptr(), size, bench.GEN[kind], bench.SEEDS[kind], 0, stream.cuda_stream)
        torch.cuda.synchronize()
        for avg in [int(x) for x in a.avgs.split(",")]:
            ch = pbschunk.Chunker(avg)
            ch.set_stream(stream.cuda_stream)
            out = torch.empty(ch.cuts_bound(size), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
            for _ in range(3):
                ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
            torch.cuda.synchronize()
            rows = []
            for _ in range(a.steps):
                t0 = time.perf_counter()
                cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
                wall = (time.perf_counter() - t0) * 1e3
                t = ch.last_timing()
                rows.append((wall, t["scan_ms"], t["exact_ms"], t["resolve_ms"], t.get("total_ms", 0.0)))
            m = np.median(np.array(rows), axis=0)
            print(json.dumps({"kind": kind, "avg": avg, "path": bench.pass_path(t), "chunks": int(cuts.size),
                              "candidates": int(t["candidates"]), "wall_ms": round(m[0], 3),
                              "scan_ms": round(m[1], 3), "gather_ms": round(m[2], 3), "resolve_ms": round(m[3], 3),
                              "rest_ms": round(m[0] - m[1] - m[2] - m[3], 3), "timing": {k: round(v, 3) if isinstance(v, float) else v for k, v in t.items()}}),
                  flush=True)
            ch.close()


if __name__ == "__main__":
    main()
