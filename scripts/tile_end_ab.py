"""A/B of an environment knob read when a chunker handle is created, one process, settings
alternated, 64 GiB per stream: median scan-kernel ms and wall ms per pass, and whether each
setting's cut list still equals the golden record.  Round 4 ran it with PBS_FUSED_DBG (a
temporary switch of the scan pass's tile ends, since removed; `profiles/r04/scanpass/
tileend.log`) and with PBS_FUSED_MIN_AVG (the scan pass forced up to 4 MiB, `r04p_*.log`).

    python scripts/tile_end_ab.py --env PBS_FUSED_MIN_AVG --dbg 262144,8388608 [--kinds vmimage] [--avgs ...]
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
    ap.add_argument("--avgs", default="65536,131072")
    ap.add_argument("--dbg", default="262144,8388608", help="the knob's values, comma-separated")
    ap.add_argument("--env", default="PBS_FUSED_MIN_AVG")
    ap.add_argument("--size-gib", type=float, default=64.0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
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
            res = {}
            for _ in range(a.reps):
                for d in a.dbg.split(","):
                    os.environ[a.env] = d
                    ch = pbschunk.Chunker(avg)
                    ch.set_stream(stream.cuda_stream)
                    out = torch.empty(ch.cuts_bound(size), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
                    ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
                    torch.cuda.synchronize()
                    for _ in range(a.steps):
                        t0 = time.perf_counter()
                        cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
                        wall = (time.perf_counter() - t0) * 1e3
                        t = ch.last_timing()
                        res.setdefault(d, []).append((wall, t["scan_ms"], bench.pass_path(t)))
                    rec = {"chunks": int(cuts.size), **bench.cut_record(cuts, keep=0)}
                    bench.verify_record(rec, kind, size, avg, bench.SEEDS[kind])
                    res.setdefault(d + "v", []).append(rec["verified"])
                    ch.close()
            os.environ.pop(a.env, None)
            for d in a.dbg.split(","):
                v = np.array([(w, s) for w, s, _ in res[d]])
                m = np.median(v, axis=0)
                print(json.dumps({"kind": kind, "avg": avg, a.env: d, "path": res[d][-1][2],
                                  "wall_ms": round(m[0], 3), "scan_ms": round(m[1], 3),
                                  "verified": res[d + "v"]}), flush=True)


if __name__ == "__main__":
    main()
