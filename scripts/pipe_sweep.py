"""Host-stream pipeline (pbs_pipeline_host) over one pageable 64 GiB host copy of the VM-image
stream, for several routing settings in one process (the PBS_PIPE_* knobs are read per call):
total, drain after the last piece, host share, digest-queue jobs; digests checked against the
first run's (and the cut list against the golden record).

    python scripts/pipe_sweep.py [--gib 64] "SLACK_MS=40" "SLACK_MS=120,HOST_THREADS=15" ...

(a name starting with PBS_ is taken as it is, e.g. "PBS_SHA_HOST_LANES=1")
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=64.0)
    ap.add_argument("--piece-mib", type=int, default=1024)
    ap.add_argument("settings", nargs="*", default=["SLACK_MS=40"])
    a = ap.parse_args()
    n = int(a.gib * (1 << 30)) // 8 * 8
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    pbschunk.generate_device(dev.data_ptr(), n, bench.GEN["vmimage"], bench.SEEDS["vmimage"], 0,
                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = dev.cpu().numpy()
    del dev
    torch.cuda.empty_cache()
    pbschunk.pipeline_host(host[: 64 << 20], 4 << 20, piece=16 << 20, crc=True)  # warm-up
    ref = None
    for st in a.settings:
        name = lambda k: k if k.startswith("PBS_") else f"PBS_PIPE_{k}"  # noqa: E731
        keys = [name(kv.split("=")[0]) for kv in st.split(",") if kv]
        for kv in filter(None, st.split(",")):
            k, v = kv.split("=", 1)
            os.environ[name(k)] = v
        t0 = time.perf_counter()
        ends, dig, crcs, t = pbschunk.pipeline_host(host, 4 << 20, piece=a.piece_mib << 20, crc=True)
        wall = time.perf_counter() - t0
        for k in keys:
            os.environ.pop(k, None)
        if ref is None:
            rec = {"chunks": int(ends.size), **bench.cut_record(ends, keep=0)}
            bench.verify_record(rec, "vmimage", n, 4 << 20, bench.SEEDS["vmimage"])
            ref = (ends, dig, crcs)
            same = f"cuts verified {rec['verified']}"
        else:
            same = "same as the first" if (np.array_equal(ends, ref[0]) and np.array_equal(dig, ref[1])
                                           and np.array_equal(crcs, ref[2])) else "DIFFERENT"
        print(f"{st:40s}: {n / (1 << 30) / wall:6.2f} GiB/s  total {t['total_ms']:.1f} h2d {t['h2d_ms']:.1f} "
              f"drain {t['drain_ms']:.1f} ms | host {t['host_chunks']} chunks {t['host_bytes'] / (1 << 30):.2f} GiB "
              f"host work done {t['host_work_ms']:.1f} gpu done {t['gpu_done_ms']:.1f} | queue jobs {t['gpu_jobs']} claimed {t['gpu_claimed']} "
              f"launches {t['queue_launches']} | {same}", flush=True)


if __name__ == "__main__":
    main()
