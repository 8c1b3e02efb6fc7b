"""Sum rocprofv3 --pmc counter values per kernel (and per dispatch count) from the
*_counter_collection.csv files under the given directories.

    python scripts/pmc_summary.py gpurun_out/r03j/pmc_icache [more dirs] [--kernel zstd_block]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = None
    if "--kernel" in sys.argv:
        filt = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != filt]
    tot = defaultdict(float)
    disp = defaultdict(set)
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if filt and filt not in k:
                    continue
                k = k.split("(")[0][-60:]
                tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    for (k, c), v in sorted(tot.items()):
        n = len(disp[k])
        print(f"{k:60s} {c:32s} total {v:16.0f}  per-dispatch {v / n:14.0f}  (dispatches {n})")


if __name__ == "__main__":
    main()
