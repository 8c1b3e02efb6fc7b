"""Debug: one find_cuts_device pass over a generated stream in HBM, its cut list against the
oracle's two-phase restatement, with whatever PBS_* switches the environment sets.

    python scripts/debug/fused_check.py [gib] [kind 1=random 2=vm] [avg]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "proxmox-backup_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    import pbschunk
    import oracle
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    avg = int(sys.argv[3]) if len(sys.argv) > 3 else 4 << 20
    n = int(gib * (1 << 30))
    seed = 0x5EED0002 if kind == 1 else 0x5EED0003
    dev = torch.empty((n + 7) // 8 * 8, dtype=torch.uint8, device="cuda")
    pbschunk.generate_device(dev.data_ptr(), dev.numel(), kind, seed, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ch = pbschunk.Chunker(avg)
    got = ch.find_cuts_device(dev.data_ptr(), n, is_final=False)
    t = ch.last_timing()
    host = dev[:n].cpu().numpy()
    cand = oracle.candidates(avg, host)
    ref = oracle.resolve(avg, cand, n)
    ok = np.array_equal(got, ref)
    print({k: t[k] for k in ("fused", "scan_pass", "candidates", "cuts") if k in t}, "ref cuts", ref.size,
          "got", got.size, "cand", cand.size, "OK" if ok else "MISMATCH", got[:4], ref[:4], flush=True)


if __name__ == "__main__":
    main()
