"""Same-box A/B of the GPU blob stage on the zstd corpora: one process per library (the
library under test through PBS_LIBPBSCHUNK_AB, else the in-tree build), best of --reps
encodes of --gib GiB per corpus, one JSON line per corpus.  Used with scripts/gpu_runs/zstd_ab.sh,
which alternates the libraries.

    python scripts/zstd_ab.py [--corpus text,pxar] [--gib 1] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "proxmox-backup_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--corpus", default="text,pxar")
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--avg", type=int, default=4 << 20)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch

    import corpus_gen
    import pbschunk

    torch.cuda.set_device(0)
    for name in a.corpus.split(","):
        base = {"text": lambda: corpus_gen.text(32 << 20, 21), "pxar": lambda: corpus_gen.pxar(32 << 20, 22)}[name]()
        n = int(a.gib * (1 << 30)) // base.size * base.size
        dev = torch.from_numpy(np.tile(base, n // base.size)).to("cuda")
        with pbschunk.Chunker(a.avg) as c:
            ends = c.find_cuts_device(dev.data_ptr(), n, is_final=True)
        bounds = np.concatenate([[0], ends]).astype(np.uint64)
        cap = pbschunk.blob_stream_bound(bounds)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        offs = pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)[0]  # warm-up
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"corpus": name, "lib": os.environ.get("PBS_LIBPBSCHUNK_AB", "tree"),
                          "build": pbschunk.build_id(), "GiB/s": round(n / min(ts) / 2**30, 2),
                          "ms": [round(t * 1e3, 2) for t in ts], "out_bytes": int(offs[-1])}),
              flush=True)
        del dev, out


if __name__ == "__main__":
    main()
