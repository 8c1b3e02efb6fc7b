"""Generate the golden cut-list fixtures in tests/golden/ with the CPU oracle.

Inputs are NOT stored: each case names a generator (oracle/chunker_oracle.c,
DESIGN.md "Inputs") with its seed, offset and length; the fixture holds the chunk
END offsets the oracle's streaming restatement of chunker.rs:112-168 produces when
the whole buffer is fed at once (test_chunker1's "test2" loop, chunker.rs:246-257),
plus, for a few cases, the phase-A candidate positions.

Provenance: the reference (Rust) cannot be built in this image; the oracle is pinned
by the table digest, test_chunker1's feed invariance and the SURVEY.md section 0.6
vector (an independent transliteration).  See DESIGN.md "Parity".

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

KiB, MiB = 1024, 1024 * 1024

CASES = [
    # name, generator, seed, offset, length, avg, store_candidates
    ("counter_1M_64K", "counter", 0, 0, 1 * MiB, 64 * KiB, True),
    ("counter_80M_64K", "counter", 0, 0, 80 * MiB, 64 * KiB, False),
    ("random_64M_4M", "random", 0x5EED0002, 0, 64 * MiB, 4 * MiB, True),
    ("random_32M_256K", "random", 0x5EED0002, 0, 32 * MiB, 256 * KiB, True),
    ("random_16M_64K", "random", 0x5EED0001, 0, 16 * MiB, 64 * KiB, False),
    ("random_16M_512K", "random", 0x5EED0001, 0, 16 * MiB, 512 * KiB, False),
    ("vm_96M_4M_extent", "vmimage", 0x5EED0003, 496 * MiB, 96 * MiB, 4 * MiB, True),
    ("vm_48M_256K_off", "vmimage", 0x5EED0003, 1270 * MiB + 4096 + 8, 48 * MiB, 256 * KiB, False),
    ("random_64K_avg1", "random", 7, 0, 64 * KiB, 1, False),
    ("random_64K_avg2", "random", 7, 0, 64 * KiB, 2, True),
    ("random_64K_avg16", "random", 7, 0, 64 * KiB, 16, True),
    ("random_64K_avg64", "random", 7, 0, 64 * KiB, 64, True),
    ("random_256K_avg128", "random", 8, 0, 256 * KiB, 128, True),
    ("random_1M_avg4096", "random", 9, 0, 1 * MiB, 4096, True),
    ("zeros_40M_4M", "zeros", 0, 0, 40 * MiB, 4 * MiB, False),
    ("random_100_64", "random", 3, 0, 100, 64, True),
    ("random_63_64", "random", 3, 0, 63, 64, True),
]


def make_input(gen: str, seed: int, offset: int, length: int) -> np.ndarray:
    if gen == "counter":
        return oracle.gen_counter(length, offset)
    if gen == "random":
        return oracle.gen_random(length, seed, offset)
    if gen == "vmimage":
        return oracle.gen_vmimage(length, seed, offset)
    if gen == "zeros":
        return np.zeros(length, dtype=np.uint8)
    raise ValueError(gen)


def main():
    manifest = []
    for name, gen, seed, offset, length, avg, store_cand in CASES:
        data = make_input(gen, seed, offset, length)
        cuts = oracle.chunk_feed(avg, data, 0)
        np.save(os.path.join(HERE, f"{name}.cuts.npy"), cuts.astype("<u8"), allow_pickle=False)
        entry = dict(name=name, generator=gen, seed=seed, offset=offset, length=length, avg=avg,
                     ncuts=int(cuts.size), tail=int(length - (int(cuts[-1]) if cuts.size else 0)))
        if store_cand:
            cand = oracle.candidates(avg, data)
            np.save(os.path.join(HERE, f"{name}.cand.npy"), cand.astype("<u8"), allow_pickle=False)
            entry["ncand"] = int(cand.size)
        manifest.append(entry)
        print(name, entry["ncuts"], entry.get("ncand"))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator_script": "tests/golden/make_golden.py",
                   "oracle": "oracle/chunker_oracle.c",
                   "cuts": "chunk END offsets (exclusive), whole-buffer feed; tail not a cut",
                   "cases": manifest}, f, indent=1)


if __name__ == "__main__":
    main()
