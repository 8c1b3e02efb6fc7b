"""Model of the host-stream pipeline's tail (pbs_pipeline.cpp): when does the last chunk
digest finish, for a given split of the chunks between the GPU (one lane per chunk, a
serial SHA-256 chain at ~r_gpu per lane) and the host threads (SHA extensions), given
the cut list of the 64 GiB stream?  Used to choose the routing rule before building it.

    python scripts/pipe_sim.py cuts.npy [--piece-mib 1024] [--copy-gbs 56.2] ...
"""
import argparse
import heapq

import numpy as np


def simulate(ends, zero, piece, copy_bps, r_gpu, r_host, threads, policy, slack_ms, launch):
    n = ends.size
    starts = np.concatenate([[0], ends[:-1]])
    lens = ends - starts
    total = int(ends[-1])
    t_copy_end = total / copy_bps * 1e3
    # chunk c is known once the piece holding its end is resident (+ the pass, ~0.3 ms)
    piece_idx = (ends - 1) // piece
    t_known = ((piece_idx + 1) * piece).clip(max=total) / copy_bps * 1e3 + 0.3
    deadline = t_copy_end + slack_ms
    gpu_done, host_jobs = 0.0, []
    seen_zero = set()
    # "eft": deadline first, else whichever side finishes the chunk first -- the host side
    # modelled as the workers' free times, FIFO (the pool is fed in stream order)
    model = [0.0] * threads
    heapq.heapify(model)
    for c in range(n):
        L = int(lens[c])
        if zero[c]:
            if L in seen_zero:
                continue
            seen_zero.add(L)
        g = L / r_gpu * 1e3
        if launch == "quarter":  # launches when a quarter of the stream is chunked
            q = min(3, int(ends[c] * 4 // total))
            t_launch = (q + 1) * total / 4 / copy_bps * 1e3 + 0.3
        else:  # a persistent kernel takes the chunk as soon as it is known
            t_launch = t_known[c]
        if policy == "eft":
            to_gpu = t_launch + g <= deadline
            if not to_gpu:
                h_end = max(model[0], t_known[c]) + L / r_host * 1e3
                to_gpu = t_launch + g < h_end
                if not to_gpu:
                    heapq.heapreplace(model, h_end)
        else:
            to_gpu = {"fixed8": L < (8 << 20), "deadline": t_launch + g <= deadline,
                      "gpu": True}[policy]
        if to_gpu:
            gpu_done = max(gpu_done, t_launch + g)
        else:
            host_jobs.append((t_known[c], L))
    # host pool: FIFO by arrival, `threads` workers
    host_jobs.sort()
    free = [0.0] * threads
    heapq.heapify(free)
    host_done, host_bytes = 0.0, 0
    for t, L in host_jobs:
        w = heapq.heappop(free)
        s = max(w, t)
        e = s + L / r_host * 1e3
        heapq.heappush(free, e)
        host_done = max(host_done, e)
        host_bytes += L
    end = max(t_copy_end + 0.3, gpu_done, host_done)
    return {"end_ms": round(end, 1), "copy_end_ms": round(t_copy_end, 1), "gpu_done": round(gpu_done, 1),
            "host_done": round(host_done, 1), "host_gib": round(host_bytes / (1 << 30), 2),
            "host_chunks": len(host_jobs), "GiB/s": round(total / (1 << 30) / (end / 1e3), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cuts")
    ap.add_argument("--piece-mib", type=int, default=1024)
    ap.add_argument("--copy-gbs", type=float, default=56.2)
    ap.add_argument("--r-gpu-mbs", type=float, default=35.0)
    ap.add_argument("--r-host-mbs", type=float, default=1500.0)
    ap.add_argument("--threads", type=int, default=14)
    a = ap.parse_args()
    ends = np.load(a.cuts).astype(np.int64)
    # zero chunks: the VM image's 64 MiB zero extent per GiB (slot from the seed) holds them
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
    import oracle
    seed = 0x5EED0003
    starts = np.concatenate([[0], ends[:-1]])
    zero = np.zeros(ends.size, bool)
    for c in range(ends.size):
        s, e = int(starts[c]), int(ends[c])
        g = s >> 30
        if (e - 1) >> 30 != g:
            continue
        slot = (oracle.splitmix64(seed ^ 0x4558544E54000000 ^ g) & 15) << 26
        base = (g << 30) + slot
        zero[c] = s >= base and e <= base + (1 << 26)
    print(f"{ends.size} chunks, {zero.sum()} zero (in the extents)")
    for piece in (a.piece_mib, 256, 64):
        for launch in ("quarter", "persistent"):
            for policy, slack in (("fixed8", 0), ("gpu", 0), ("deadline", 0), ("deadline", 20), ("deadline", 60),
                                  ("eft", 0), ("eft", 20)):
                r = simulate(ends, zero, piece << 20, a.copy_gbs * 1e9, a.r_gpu_mbs * 1e6, a.r_host_mbs * 1e6,
                             a.threads, policy, slack, launch)
                print(f"piece {piece:5d} MiB {launch:10s} {policy:8s} slack {slack:3d}: {r}")


if __name__ == "__main__":
    main()
