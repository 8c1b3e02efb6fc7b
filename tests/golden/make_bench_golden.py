"""Golden cut lists of every stream bench.py may time (tests/golden/bench_cuts.json).

TEST INFRASTRUCTURE: the expected results come from the CPU oracle's streaming
restatement of Chunker::scan (oracle/chunker_oracle.c, ora_chunk_generated: the stream
is generated 16 MiB at a time and fed through the ChunkStream caller loop around the
chunker.rs:112-168 scan), never from the GPU.  bench.py compares each rank's timed cut
list against these entries after its timed region and prints "verified" per rank.

Each entry is keyed ``<workload>:<bytes>:<avg>:<seed>`` and holds the number of chunks
and the SHA-256 of the cut list exactly as bench.py's ``cut_record`` hashes it: chunk
END offsets as u64 little-endian, the stream end included when the tail is non-empty
(find_cuts(..., is_final=True)).

Streams (bench.py's generators, seeds as in bench.SEEDS / stream_seed):
  * vmimage 64 GiB, seeds 0x5EED0003..0x5EED000A (config 3 = rank 0, config 4 = ranks
    0-7), 4 MiB -- one independent stream per GPU (proxmox-backup-client/src/main.rs:200-211);
  * vmimage and random 64 GiB at every average verify_chunk_size accepts
    (pbs-datastore/src/chunk_store.rs:33-48: 64 KiB .. 4 MiB; config 5 = vmimage 256 KiB;
    random 4 MiB = bench.py's secondary line);
  * random 8 GiB, 4 MiB (config 2);
  * vmimage 16 GiB, 4 MiB: the first 16 GiB of config 3's stream (bench.py's pipeline and
    upload stages);
  * the small streams tests/test_dist.py runs bench.py on.

    python tests/golden/make_bench_golden.py [--threads 8] [--only SUBSTR] [--check]

``--check`` recomputes only the entries under 1 GiB and compares them with the file.
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

GiB = 1 << 30
KiB = 1 << 10
MiB = 1 << 20
AVERAGES = [64 * KiB, 128 * KiB, 256 * KiB, 512 * KiB, 1 * MiB, 2 * MiB, 4 * MiB]
SEED_RANDOM, SEED_VM = 0x5EED0002, 0x5EED0003
OUT = os.path.join(HERE, "bench_cuts.json")


def stream_bytes(gib: float) -> int:
    """bench.py's stream length for --size-gib (whole 8-byte words)."""
    return int(gib * GiB) // 8 * 8


def key(workload: str, size: int, avg: int, seed: int) -> str:
    return f"{workload}:{size}:{avg}:{seed:#x}"


def streams():
    """(workload, bytes, avg, seed) of every golden entry."""
    out = []
    big = stream_bytes(64)
    for r in range(8):
        out.append(("vmimage", big, 4 * MiB, SEED_VM + r))
    for avg in AVERAGES:
        if avg != 4 * MiB:
            out.append(("vmimage", big, avg, SEED_VM))
        out.append(("random", big, avg, SEED_RANDOM))
    out.append(("random", stream_bytes(8), 4 * MiB, SEED_RANDOM))
    # bench.py's f-stages: the host pipeline and the compressing upload over the first
    # --stage-gib (16) GiB of the config-3 stream
    out.append(("vmimage", stream_bytes(16), 4 * MiB, SEED_VM))
    # tests/test_dist.py: 2 ranks of 0.25 GiB (4 MiB) and of 0.01 GiB (4 MiB, 64 KiB)
    for gib, avg in ((0.25, 4 * MiB), (0.01, 4 * MiB), (0.01, 64 * KiB)):
        for r in range(2):
            out.append(("vmimage", stream_bytes(gib), avg, SEED_VM + r))
    return out


def cuts_sha256(cuts) -> str:
    import numpy as np
    c = np.ascontiguousarray(np.asarray(cuts, dtype=np.uint64))
    return hashlib.sha256(c.astype("<u8").tobytes()).hexdigest()


def record(workload: str, size: int, avg: int, seed: int) -> dict:
    import oracle
    cuts = oracle.chunk_generated(workload, seed, avg, size)
    return {"workload": workload, "bytes": size, "avg": avg, "seed": hex(seed),
            "chunks": int(cuts.size), "cuts_sha256": cuts_sha256(cuts),
            "last_cuts": [int(x) for x in cuts[-3:]]}


def run(todo, threads: int, log=print) -> dict:
    res, lock = {}, threading.Lock()
    todo = sorted(todo, key=lambda s: -s[1])  # longest first
    it = iter(todo)

    def worker():
        while True:
            with lock:
                s = next(it, None)
            if s is None:
                return
            t0 = time.time()
            rec = record(*s)
            with lock:
                res[key(*s)] = rec
                log(f"{key(*s)}: {rec['chunks']} chunks, {time.time() - t0:.0f} s "
                    f"({len(res)}/{len(todo)})", flush=True)

    ths = [threading.Thread(target=worker) for _ in range(threads)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--only", default="", help="only the entries whose key contains this")
    ap.add_argument("--check", action="store_true", help="recompute the < 1 GiB entries and compare")
    a = ap.parse_args()
    if a.check:
        have = json.load(open(OUT))["streams"]
        todo = [s for s in streams() if s[1] < GiB]
        got = run(todo, a.threads)
        bad = [k for k in got if have.get(k) != got[k]]
        print("check:", "OK" if not bad else f"MISMATCH {bad}")
        sys.exit(1 if bad else 0)
    todo = [s for s in streams() if a.only in key(*s)]
    old = json.load(open(OUT))["streams"] if os.path.exists(OUT) else {}
    res = run(todo, a.threads)
    old.update(res)
    doc = {"about": "Golden cut lists of bench.py's streams: chunk END offsets as u64 LE (stream "
                    "end included), SHA-256 + count, from the CPU oracle's streaming restatement "
                    "of Chunker::scan (oracle/chunker_oracle.c ora_chunk_generated). Made by "
                    "tests/golden/make_bench_golden.py.",
           "streams": dict(sorted(old.items()))}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"wrote {len(old)} entries to {OUT}")


if __name__ == "__main__":
    main()
