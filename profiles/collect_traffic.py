"""Derive HBM read bytes per scan_main_kernel launch from a rocprofv3 --pmc FETCH_SIZE
run of bench.py and write profiles/traffic_latest.json (read by bench.py).

The record carries the library's build id (pbs_build_id, a digest of its sources):
bench.py reports the traffic only for the same build.

FETCH_SIZE is in KiB; on gfx950 it reports exactly half the bytes of a wide coalesced
streaming read (MI355X_MICROARCH.md "HBM"), so bytes = FETCH_SIZE * 1024 * 2.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
        python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --host-inclusive-gib 0
    python profiles/collect_traffic.py gpurun_out/pmc_fetch --size-gib 64 --avg 4194304 --workload vmimage
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "proxmox-backup_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("--size-gib", type=float, default=64.0)
ap.add_argument("--avg", type=int, default=4 * 1024 * 1024)
ap.add_argument("--workload", default="vmimage")
ap.add_argument("--kernel", default="scan_fused_kernel",
                help="kernel-name substring (scan_fused_kernel, scan_main_kernel, crc32_chunks_kernel)")
ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic_latest.json"))
a = ap.parse_args()

files = glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True)
per_dispatch = {}
for f in files:
    for row in csv.DictReader(open(f)):
        if a.kernel not in row.get("Kernel_Name", "") or row.get("Counter_Name") != "FETCH_SIZE":
            continue
        key = (f, row.get("Dispatch_Id"))
        per_dispatch[key] = per_dispatch.get(key, 0.0) + float(row["Counter_Value"])
vals = sorted(per_dispatch.values())
if not vals:
    raise SystemExit(f"no {a.kernel} FETCH_SIZE rows found")
kib = statistics.median(vals)
size = int(a.size_gib * (1 << 30)) // 8 * 8
import pbschunk  # noqa: E402  (the library the PMC run loaded: no device call)

out = {"build_id": pbschunk.build_id(), "kernel": a.kernel, "size": size, "avg": a.avg, "workload": a.workload, "dispatches": len(vals),
       "fetch_size_kib_median": kib, "hbm_bytes_per_launch": int(kib * 1024 * 2),
       "ratio_to_algorithmic": kib * 1024 * 2 / size,
       "note": "FETCH_SIZE x 1024 x 2 (gfx950 half-count correction), median over dispatches"}
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps(out))
