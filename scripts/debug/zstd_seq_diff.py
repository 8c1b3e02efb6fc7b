"""Diagnostics: the first zstd block whose GPU frame bytes differ from the twin's, and the
first sequence where the GPU parse (PBS_ZSTD_DEBUG_ITEM dump) and the twin's parse
(zstd_twin_parse) part.  Runs on the GPU box.

    python scripts/debug/zstd_seq_diff.py [--kind vm|text|pxar] [--mib 4]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "proxmox-backup_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
KIB = 1024


def blocks(frame):
    """(offset, size) of each block of a single-segment frame"""
    fhd = frame[4]
    fcs = {0: 1, 1: 2, 2: 4, 3: 8}[fhd >> 6]
    o = 5 + fcs
    out = []
    while True:
        h = frame[o] | frame[o + 1] << 8 | frame[o + 2] << 16
        t, sz = (h >> 1) & 3, h >> 3
        body = 1 if t == 1 else sz
        out.append((o, 3 + body))
        o += 3 + body
        if h & 1:
            return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="vm")
    ap.add_argument("--mib", type=int, default=4)
    ap.add_argument("--item", type=int, default=-1)
    a = ap.parse_args()
    import corpus_gen
    import gen_np
    import oracle
    n = a.mib << 20
    data = {"vm": lambda: gen_np.gen_vmimage(n, 0x5EED0003, 0), "text": lambda: corpus_gen.text(n, 3),
            "pxar": lambda: corpus_gen.pxar(n, 4)}[a.kind]()
    if a.item < 0:  # find the first differing block, then rerun this script for its dump
        import torch
        import pbschunk
        torch.cuda.set_device(0)
        dev = torch.from_numpy(data).to("cuda")
        bounds = np.array([0, n], np.uint64)
        cap = pbschunk.blob_stream_bound(bounds)
        out = torch.empty(cap, dtype=torch.uint8, device="cuda")
        offs, _, _, _ = pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)
        torch.cuda.synchronize()
        g = out[12:int(offs[1])].cpu().numpy().tobytes()
        t = oracle.zstd_twin_frame(data.tobytes())
        if g == t:
            print("frames equal")
            return
        gb, tb = blocks(g), blocks(t)
        for j, (x, y) in enumerate(zip(gb, tb)):
            if g[x[0]:x[0] + x[1]] != t[y[0]:y[0] + y[1]]:
                print(f"first differing block {j}: gpu {x[1]} bytes, twin {y[1]} bytes")
                env = dict(os.environ, PBS_ZSTD_DEBUG_ITEM=str(j), PBS_ZSTD_DEBUG_OUT="/tmp/zdbg.bin")
                subprocess.run([sys.executable] + sys.argv + ["--item", str(j)], env=env, check=True)
                return
        print("block lists differ in length", len(gb), len(tb))
        return
    # the dump of item a.item: rerun the encode with the env set, then diff
    import torch
    import pbschunk
    torch.cuda.set_device(0)
    dev = torch.from_numpy(data).to("cuda")
    bounds = np.array([0, n], np.uint64)
    cap = pbschunk.blob_stream_bound(bounds)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    pbschunk.blob_encode_chunks_device(dev.data_ptr(), n, bounds, out.data_ptr(), cap)
    torch.cuda.synchronize()
    dump = np.fromfile("/tmp/zdbg.bin", dtype=np.uint32)
    per = dump.size // 8
    gseq = []
    for w in range(8):
        cnt = int(dump[w * per])
        rec = dump[w * per + 1: w * per + 1 + 3 * cnt].reshape(-1, 3)
        gseq += [tuple(int(v) for v in r) + (w,) for r in rec]
    j = a.item
    off = j * 64 * KIB
    blk = np.ascontiguousarray(data[off: off + 64 * KIB])
    L = oracle._twin_lib()
    L.zstd_twin_parse.restype = ctypes.c_uint64
    L.zstd_twin_parse.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    buf = np.ascontiguousarray(data)
    o = np.empty(3 * 20000, np.uint32)
    k = L.zstd_twin_parse(buf.ctypes.data + off, blk.size, off, o.ctypes.data, 20000)
    tseq = [tuple(int(v) for v in o[3 * i: 3 * i + 3]) for i in range(k)]
    print(f"item {j}: gpu {len(gseq)} sequences, twin {len(tseq)}")
    for i, (x, y) in enumerate(zip(gseq, tseq)):
        if x[:3] != y:
            print(f"first difference at sequence {i} (gpu sub-block {x[3]}): gpu {x[:3]} twin {y}")
            for q in range(max(0, i - 3), min(len(tseq), i + 4)):
                print("  ", q, "gpu", gseq[q] if q < len(gseq) else None, "twin", tseq[q])
            return
    print("sequence lists agree on their common prefix")


if __name__ == "__main__":
    main()
