"""Per-kernel totals from a rocprofv3 results database (rocpd sqlite): name, launches,
sum and average ms; with --seq the durations in launch order (filter by substring)."""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    t = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [x for x in t if x.startswith("rocpd_kernel_dispatch")][0]
    ks = [x for x in t if x.startswith("rocpd_info_kernel_symbol")][0]
    rows = list(c.execute(f"select s.kernel_name, d.start, d.end from {kd} d join {ks} s on d.kernel_id = s.id "
                          f"order by d.start"))
    agg = collections.defaultdict(list)
    for n, a, b in rows:
        agg[n.split("(")[0]].append((b - a) / 1e6)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if flt in k:
            print(f"{k[-60:]:60s} n={len(v):5d} sum={sum(v):9.3f} ms avg={sum(v) / len(v):8.4f} ms")


if __name__ == "__main__":
    main()
