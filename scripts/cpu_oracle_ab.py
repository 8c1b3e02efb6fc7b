"""CPU baseline stability: the round-3 and round-5 builds of the oracle
(oracle/chunker_oracle.c at commits 2558058 and HEAD, both `gcc -O2 -fPIC -std=c11`, and both
again with `-falign-loops=64 -falign-functions=64`, built into scripts/ab_libs/) timed alternately on one core over the same 512 MiB VM-image sample
(ora_chunk_feed, 4 MiB average), with the CPU clock beside it.  Equal rates = the build did
not move the baseline; the host did.

    python scripts/cpu_oracle_ab.py
"""
import ctypes
import os
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mhz():
    try:
        v = [float(l.split(":")[1]) for l in open("/proc/cpuinfo") if l.startswith("cpu MHz")]
        return round(sum(v) / len(v)) if v else None
    except OSError:
        return None


def main():
    n = 512 << 20
    names = ("r03", "r05", "r03_aligned", "r05_aligned")
    libs = {v: ctypes.CDLL(os.path.join(ROOT, "scripts", "ab_libs", f"liboracle_{v}.so")) for v in names}
    for L in libs.values():
        L.ora_chunk_feed.restype = ctypes.c_int64
        L.ora_chunk_feed.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_uint64]
    buf = np.empty(n, np.uint8)
    libs["r05"].ora_gen_vmimage(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(n),
                                ctypes.c_uint64(0x5EED0003), ctypes.c_uint64(0))
    out = np.empty(n // 65536 + 16, np.uint64)
    res = {}
    for _ in range(3):
        for v in names + names[::-1]:
            t0 = time.perf_counter()
            k = libs[v].ora_chunk_feed(4 << 20, buf.ctypes.data, n, 0, out.ctypes.data, out.size)
            dt = time.perf_counter() - t0
            res.setdefault(v, []).append(n / dt / 2**30)
            print(f"{v} chunks {k} GiB/s {n / dt / 2**30:.3f} cpu_mhz {mhz()}", flush=True)
    for v, r in res.items():
        print(f"{v} median GiB/s {sorted(r)[len(r) // 2]:.3f}")


if __name__ == "__main__":
    main()
