"""The headline's roofline fraction recomputed from a rocprofv3 kernel trace of the SAME
process that printed the bench line: the scan kernel's launches in
launch order, the warm-up ones (the first --warmup) dropped, the next --steps averaged, and
frac = algorithmic bytes per launch / that average / the HBM peak -- the line's own formula
(bench.py `roofline`), so the two agree when the trace and the HIP events agree.

    python scripts/frac_from_trace.py <run_results.db | kernel_trace.csv> --bench <bench line file>
"""
import argparse
import csv
import glob
import json
import os
import sqlite3


def launches(path: str, kernel: str):
    """(start_ns, end_ns) of every launch of `kernel`, in launch order."""
    out = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        t = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
        kd = [x for x in t if x.startswith("rocpd_kernel_dispatch")][0]
        ks = [x for x in t if x.startswith("rocpd_info_kernel_symbol")][0]
        for n, a, b in c.execute(f"select s.kernel_name, d.start, d.end from {kd} d join {ks} s on d.kernel_id = s.id"
                                 f" order by d.start"):
            if kernel in n:
                out.append((int(a), int(b)))
    else:
        for r in csv.DictReader(open(path)):
            if kernel in r.get("Kernel_Name", ""):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        out.sort()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", help="rocpd results .db, kernel_trace.csv, or a directory holding one")
    ap.add_argument("--bench", required=True, help="file holding the bench JSON line of the same process")
    ap.add_argument("--kernel", default="scan_fused_kernel")
    a = ap.parse_args()
    path = a.trace
    if os.path.isdir(path):
        found = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) or \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = found[0]
    line = None
    for s in open(a.bench):
        if s.startswith("{") and '"metric"' in s:
            line = json.loads(s)
    roof = line["roofline"]
    w, k = int(line["warmup"]), int(line["steps"])
    bytes_per_launch = roof["achieved"] * 1e9 * roof["avg_launch_ms"] / 1e3  # GB/s x s
    L = launches(path, a.kernel)
    dur = [(e - s) / 1e6 for s, e in L]
    timed = dur[w:w + k]
    avg = sum(timed) / len(timed)
    frac = bytes_per_launch / (avg / 1e3) / (roof["peak"] * 1e9)
    rec = {"trace": os.path.relpath(path), "kernel": a.kernel, "launches_in_trace": len(dur),
           "first_launches_ms": [round(x, 4) for x in dur[:w + k + 2]],
           "warmup_dropped": w, "timed_launches": len(timed), "warm_avg_ms": round(avg, 4),
           "min_ms": round(min(timed), 4), "bytes_per_launch": int(round(bytes_per_launch)),
           "frac_from_trace": round(frac, 4), "frac_fastest": round(bytes_per_launch / (min(timed) / 1e3) /
                                                                    (roof["peak"] * 1e9), 4),
           "line": {"value": line["value"], "ms_per_step": line["ms_per_step"], "avg_launch_ms": roof["avg_launch_ms"],
                    "frac": roof["frac"]}}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
