"""Workload for the zstd block kernel's PMC passes (profiles/r05/pmc_zstd/): a seeded
text-like or pxar-like corpus (tests/corpus_gen.py, 32 MiB tiled to --mib MiB) cut by the
GPU chunker at 4 MiB, then --reps calls of pbs_blob_encode_chunks_device.  Prints the
bytes encoded per call so the counters can be divided per input byte.

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS ... -- python scripts/zstd_pmc_run.py --corpus text
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "proxmox-backup_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--corpus", default="text")
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch

    import corpus_gen
    import pbschunk
    base = {"text": lambda: corpus_gen.text(32 << 20, 21), "pxar": lambda: corpus_gen.pxar(32 << 20, 22)}[a.corpus]()
    n = (a.mib << 20) // base.size * base.size
    torch.cuda.set_device(0)
    dev = torch.from_numpy(np.tile(base, n // base.size)).to("cuda")
    with pbschunk.Chunker(4 << 20) as c:
        ends = c.find_cuts_device(dev.data_ptr(), n, is_final=True)
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    cap = pbschunk.blob_stream_bound(bounds)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    for _ in range(a.reps):
        offs, _, _, tm = pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)
    print(f"corpus {a.corpus} bytes_per_call {n} calls {a.reps} out {int(offs[-1])} compress_ms {tm['compress_ms']:.2f}",
          flush=True)


if __name__ == "__main__":
    main()
