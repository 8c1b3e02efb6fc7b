"""every average the datastore accepts (pbs-datastore/src/chunk_store.rs:33-48:
64 KiB .. 4 MiB) x {VM image, random}, 64 GiB each, one build, one box, one process.

Per cell: W warm-up passes, then K passes timed like bench.py (sync, K x find_cuts_device
into a pinned cut array, sync) -> pass GiB/s; the scan kernel's HIP-event time -> kernel
roofline fraction; the path the passes took; the cut list's SHA-256 checked against
tests/golden/bench_cuts.json (oracle-made); board power / GFX clock sampled with amd-smi
while the passes run back to back for --power-s seconds.

    python scripts/avg_table.py [--kinds vmimage,random] [--avgs 65536,...] [--steps 10]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proxmox-backup_amd"))

import bench  # noqa: E402  (cut_record, verify_record, pass_path, SEEDS, GEN)

AVGS = [64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20]


class PowerSampler:
    """amd-smi metric -p -c (SOCKET_POWER, GFX_0 clock) every ~0.25 s in a thread."""

    def __init__(self):
        self.samples, self._stop, self._th, self.raw = [], threading.Event(), None, None

    def _run(self):
        while not self._stop.is_set():
            try:
                p = subprocess.run(["amd-smi", "metric", "-p", "-c", "-g", "0"], capture_output=True,
                                   text=True, timeout=10)
                txt = p.stdout
                if self.raw is None:
                    self.raw = txt[:4000]
                pw = re.search(r"SOCKET_POWER:\s*([\d.]+)", txt)
                ck = re.search(r"GFX_0:\s*\n\s*CLK:\s*([\d.]+)", txt)
                self.samples.append((float(pw.group(1)) if pw else None, float(ck.group(1)) if ck else None))
            except Exception as e:  # noqa: BLE001 -- sampling is best effort
                self.samples.append((None, None))
                if self.raw is None:
                    self.raw = repr(e)
            self._stop.wait(0.25)

    def __enter__(self):
        self._th = threading.Thread(target=self._run, daemon=True)
        self._th.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._th.join(timeout=15)

    def summary(self):
        pw = sorted(p for p, _ in self.samples if p is not None)
        ck = sorted(c for _, c in self.samples if c is not None)
        med = lambda v: v[len(v) // 2] if v else None  # noqa: E731
        return {"n": len(self.samples), "power_w_median": med(pw), "power_w_max": pw[-1] if pw else None,
                "gfx_mhz_median": med(ck), "gfx_mhz_min": ck[0] if ck else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="vmimage,random")
    ap.add_argument("--avgs", default=",".join(str(a) for a in AVGS))
    ap.add_argument("--size-gib", type=float, default=64.0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--power-s", type=float, default=2.0, help="0 = no power sampling")
    a = ap.parse_args()

    import numpy as np
    import torch
    import pbschunk

    size = int(a.size_gib * (1 << 30)) // 8 * 8
    buf = torch.empty(size, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    rows = []
    print(json.dumps({"build_id": pbschunk.build_id(), "size": size}), flush=True)
    for kind in a.kinds.split(","):
        seed = bench.SEEDS[kind]
        pbschunk.generate_device(buf.data_ptr(), size, bench.GEN[kind], seed, 0, stream.cuda_stream)
        torch.cuda.synchronize()
        for avg in [int(x) for x in a.avgs.split(",")]:
            ch = pbschunk.Chunker(avg)
            ch.set_stream(stream.cuda_stream)
            out = torch.empty(ch.cuts_bound(size), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
            for _ in range(a.warmup):
                ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
            torch.cuda.synchronize()
            scan, paths = [], []
            t0 = time.perf_counter()
            for _ in range(a.steps):
                cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
                t = ch.last_timing()
                scan.append(t["scan_ms"])
                paths.append(bench.pass_path(t))
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            rec = {"chunks": int(cuts.size), **bench.cut_record(cuts, keep=0)}
            bench.verify_record(rec, kind, size, avg, seed)
            power = None
            if a.power_s > 0:
                with PowerSampler() as ps:
                    t1 = time.perf_counter()
                    k = 0
                    while time.perf_counter() - t1 < a.power_s:
                        ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
                        k += 1
                    torch.cuda.synchronize()
                    pms = (time.perf_counter() - t1) / k * 1e3
                power = {**ps.summary(), "passes": k, "ms_per_pass": round(pms, 3)}
                if ps.raw and not ps.summary()["power_w_median"]:
                    power["raw"] = ps.raw[:600]
            sk = float(np.mean(scan))
            row = {"kind": kind, "avg": avg, "gib_s": round(size / (1 << 30) / (ms / 1e3), 1),
                   "ms_per_pass": round(ms, 3), "kernel_ms": round(sk, 3),
                   "frac": round(size / (sk / 1e3) / 8e12, 4), "path": paths[-1],
                   "candidates": int(t["candidates"]), "verified": rec["verified"], **rec, "power": power}
            rows.append(row)
            print(json.dumps(row), flush=True)
            ch.close()
            del out
    print("\n| kind | avg | pass GiB/s | ms/pass | kernel ms | frac | path | candidates | verified | W (med) | MHz (med) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        p = r["power"] or {}
        print(f"| {r['kind']} | {r['avg'] >> 10} KiB | {r['gib_s']} | {r['ms_per_pass']} | {r['kernel_ms']} | "
              f"{r['frac']} | {r['path']} | {r['candidates']} | {r['verified']} | {p.get('power_w_median')} | "
              f"{p.get('gfx_mhz_median')} |")
    ok = all(r["verified"] is True for r in rows)
    print("ALL VERIFIED" if ok else "NOT ALL VERIFIED", flush=True)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
