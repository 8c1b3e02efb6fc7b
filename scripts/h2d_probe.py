"""H2D copy rates into HBM from a pageable host buffer vs the same buffer registered
(hipHostRegister, in 1 GiB pieces as a pipeline would do ahead of its copy) vs a pinned
allocation, and the cost of registering/unregistering -- for the host-stream pipeline
(pbs_pipeline.cpp), whose floor is this copy.

    python scripts/h2d_probe.py [--gib 8]
"""
import argparse
import ctypes
import time

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=8)
    a = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    n = a.gib << 30
    piece = 1 << 30
    host = np.empty(n, np.uint8)
    host[::4096] = 1  # touch every page
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()

    def copy(label):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for off in range(0, n, piece):
            hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr() + off), ctypes.c_void_p(host.ctypes.data + off),
                               piece, 1, ctypes.c_void_p(st.cuda_stream))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{label}: {n / dt / 1e9:.1f} GB/s ({dt * 1e3:.1f} ms for {a.gib} GiB)", flush=True)

    copy("pageable warm-up")
    copy("pageable")
    t0 = time.perf_counter()
    rcs = [hip.hipHostRegister(ctypes.c_void_p(host.ctypes.data + off), piece, 0) for off in range(0, n, piece)]
    reg = time.perf_counter() - t0
    print(f"hipHostRegister of {a.gib} x 1 GiB: {reg * 1e3:.1f} ms ({reg / a.gib * 1e3:.1f} ms per GiB), rc {set(rcs)}",
          flush=True)
    copy("registered")
    copy("registered again")
    t0 = time.perf_counter()
    for off in range(0, n, piece):
        hip.hipHostUnregister(ctypes.c_void_p(host.ctypes.data + off))
    print(f"hipHostUnregister: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    del host
    pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pin[::4096] = 1
    host = pin.numpy()
    copy("pinned (hipHostMalloc)")


def sha_rates():
    """Host SHA-256 (the library's SHA-extension code) on 16 MiB chunks: 1 and N threads."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
    import pbschunk
    data = np.random.default_rng(1).integers(0, 256, 2 << 30, dtype=np.uint8)
    bounds = np.arange(0, data.size + 1, 16 << 20, dtype=np.uint64)
    for th in (1, 8, 14, 16):
        t0 = time.perf_counter()
        pbschunk.digest_chunks_host(data, bounds, threads=th)
        dt = time.perf_counter() - t0
        print(f"host SHA-256 {th} threads: {data.size / dt / 1e9:.2f} GB/s (ni {pbschunk.sha256_host_uses_ni()})",
              flush=True)




def contention(gib: int = 8, hash_threads: int = 14):
    """Host SHA-256 threads beside a running H2D copy: the copy from a pageable buffer
    (the runtime stages it through the CPU) vs from the same buffer registered."""
    import os
    import resource
    import sys
    import threading
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
    import pbschunk
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    n = gib << 30
    piece = 1 << 30
    src = np.empty(n, np.uint8)
    src[::4096] = 1
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    data = np.random.default_rng(2).integers(0, 256, 2 << 30, dtype=np.uint8)
    bounds = np.arange(0, data.size + 1, 16 << 20, dtype=np.uint64)
    for mode in ("pageable", "registered"):
        if mode == "registered":
            for off in range(0, n, piece):
                hip.hipHostRegister(ctypes.c_void_p(src.ctypes.data + off), piece, 0)
        stop = threading.Event()
        copied = [0]

        def copier():
            while not stop.is_set():
                for off in range(0, n, piece):
                    hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr() + off), ctypes.c_void_p(src.ctypes.data + off),
                                       piece, 1, ctypes.c_void_p(s.cuda_stream))
                hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream))
                copied[0] += n

        r0 = resource.getrusage(resource.RUSAGE_SELF)
        th = threading.Thread(target=copier)
        t0 = time.perf_counter()
        th.start()
        hashed = 0
        while time.perf_counter() - t0 < 3.0:
            pbschunk.digest_chunks_host(data, bounds, threads=hash_threads)
            hashed += data.size
        dt = time.perf_counter() - t0
        stop.set()
        th.join()
        dt2 = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
        print(f"contention {mode}: SHA {hashed / dt / 1e9:.1f} GB/s on {hash_threads} threads beside the copy "
              f"at {copied[0] / dt2 / 1e9:.1f} GB/s; process CPU {cpu / dt2:.1f} cores", flush=True)
        if mode == "registered":
            for off in range(0, n, piece):
                hip.hipHostUnregister(ctypes.c_void_p(src.ctypes.data + off))


if __name__ == "__main__":
    main()
    sha_rates()
    contention()
