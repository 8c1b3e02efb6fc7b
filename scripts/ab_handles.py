"""Same-process A/B of chunker settings read at handle creation (PBS_* knobs): one handle
per mode, created with that mode's environment, passes alternating over the same
device-resident stream; cut lists must agree.  Pass time as bench.py measures it (sync,
find_cuts_device into a pinned array, sync) and the scan kernel's HIP-event time.

    python scripts/ab_handles.py <kind> <GiB> <avg> <mode> [<mode> ...]
    mode = name[:VAR=value[,VAR=value...]]   e.g. fused  scan:PBS_FUSED_MIN_AVG=524288
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proxmox-backup_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import pbschunk  # noqa: E402


def main():
    kind, gib, avg = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    modes = sys.argv[4:]
    reps = int(os.environ.get("AB_REPS", "10"))
    size = int(gib * (1 << 30)) // 8 * 8
    st = torch.cuda.current_stream()
    buf = torch.empty(size, dtype=torch.uint8, device="cuda")
    pbschunk.generate_device(buf.data_ptr(), size, bench.GEN[kind], bench.SEEDS[kind], 0, st.cuda_stream)
    torch.cuda.synchronize()
    hs = {}
    for m in modes:
        name, _, envs = m.partition(":")
        saved = {}
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        ch = pbschunk.Chunker(avg)
        ch.set_stream(st.cuda_stream)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        out = torch.empty(ch.cuts_bound(size), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
        hs[name] = (ch, out, [], [], [])
    ref = None
    for rep in range(reps + 2):
        for name, (ch, out, wall, scan, path) in hs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True, out=out)
            torch.cuda.synchronize()
            w = (time.perf_counter() - t0) * 1e3
            t = ch.last_timing()
            if ref is None:
                ref = cuts.copy()
            assert np.array_equal(cuts, ref), f"cut lists differ ({name})"
            if rep >= 2:
                wall.append(w)
                scan.append(t["scan_ms"])
                path.append(bench.pass_path(t))
    rec = {"chunks": int(ref.size), **bench.cut_record(ref, keep=0)}
    bench.verify_record(rec, kind, size, avg, bench.SEEDS[kind])
    print(f"{kind} {gib:g} GiB avg {avg}: {ref.size} cuts, verified {rec['verified']}")
    for name, (ch, out, wall, scan, path) in hs.items():
        w, s = sorted(wall), sorted(scan)
        print(f"  {name:>12}: pass ms min {w[0]:.3f} med {w[len(w) // 2]:.3f} -> {size / (1 << 30) / (w[len(w) // 2] / 1e3):.1f}"
              f" GiB/s | kernel ms min {s[0]:.3f} med {s[len(s) // 2]:.3f} (frac {size / (s[len(s) // 2] / 1e3) / 8e12:.4f})"
              f" | path {set(path)}", flush=True)


if __name__ == "__main__":
    main()
