"""Per-input-byte PMC table from rocprofv3 --pmc runs (one directory per counter group,
named <build>_<workload>_<first counter>, each beside a <same>.log whose 'bytes_per_call N'
or bench JSON line gives the bytes per dispatch).  Prints a JSON record per (build,
workload): counters per dispatch and per input byte, wave-cycle shares and the clock
(GRBM_GUI_ACTIVE / 8 XCDs / kernel ms when a duration is given).

    python scripts/pmc_per_byte.py gpurun_out/pmc_zstd --kernel zstd_block_kernel
    python scripts/pmc_per_byte.py gpurun_out/pmc_scan --kernel scan_fused_kernel --bytes 68719476736
"""
import argparse
import csv
import glob
import json
import os
import re  # noqa: F401
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--bytes", type=int, default=0, help="bytes per dispatch (else read from the logs)")
    a = ap.parse_args()
    groups = defaultdict(dict)
    nbytes = {}
    for d in sorted(glob.glob(os.path.join(a.root, "*"))):
        if not os.path.isdir(d):
            continue
        base = os.path.basename(d)
        toks = base.split("_")
        first = next((i for i, t in enumerate(toks) if t.isupper()), None)  # the counter's first token
        if first is None or first == 0:
            continue
        pre = toks[:first]
        key = ("_".join(pre[:-1]) or "cur", pre[-1])
        per, disp = defaultdict(float), defaultdict(set)
        dur = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if a.kernel not in r["Kernel_Name"]:
                    continue
                per[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
                if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # ms
        for c, v in per.items():
            groups[key][c] = v / max(1, len(disp[c]))
        if dur and "GRBM_GUI_ACTIVE" in per:
            ms = sum(dur.values()) / len(dur)
            groups[key]["_kernel_ms"] = ms
            groups[key]["_clock_ghz"] = per["GRBM_GUI_ACTIVE"] / max(1, len(disp["GRBM_GUI_ACTIVE"])) / 8 / (ms * 1e6)
        log = d + ".log"
        if os.path.exists(log) and key not in nbytes:
            t = open(log, errors="replace").read()
            mb = re.search(r"bytes_per_call (\d+)", t)
            if mb:
                nbytes[key] = int(mb.group(1))
    for key, cs in sorted(groups.items()):
        nb = a.bytes or nbytes.get(key, 0)
        rec = {"build": key[0], "workload": key[1], "bytes_per_dispatch": nb,
               "per_dispatch": {c: round(v) for c, v in sorted(cs.items()) if not c.startswith("_")}}
        if "_clock_ghz" in cs:
            rec["kernel_ms_in_grbm_pass"] = round(cs["_kernel_ms"], 3)
            rec["clock_ghz"] = round(cs["_clock_ghz"], 3)
        if nb:
            rec["per_byte"] = {c: round(v / nb, 4) for c, v in sorted(cs.items())
                               if c.startswith("SQ_INSTS") or c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "FETCH_SIZE")}
        wc = cs.get("SQ_WAVE_CYCLES")
        if wc:
            rec["wave_cycle_shares"] = {c: round(cs[c] / wc, 3) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                           "SQ_ACTIVE_INST_ANY") if c in cs}
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
