"""CPU tests of the oracle (test infrastructure) against the reference's own test,
the table digest, the SURVEY.md section 0 properties and the golden fixtures.

Reference: pbs-datastore/src/chunker.rs (table :35-68, new :75-106, scan :112-168,
shall_break :172-186, test_chunker1 :202-271)."""
import hashlib
import json
import os

import numpy as np
import pytest

import gen_np

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KiB, MiB = 1024, 1024 * 1024


def _table_from_oracle_header():
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "oracle", "buzhash_table_oracle.h")).read()
    body = src[src.index("{") + 1: src.index("};")]
    return np.array([int(x, 16) for x in re.findall(r"0x[0-9a-f]+", body)], dtype="<u4")


def test_table_digest(oracle):
    t = _table_from_oracle_header()
    assert t.size == 256 and t[0] == 0x458BE752 and t[255] == 0xD95DDF11
    assert hashlib.sha256(t.tobytes()).hexdigest() == oracle.TABLE_SHA256


def test_ctor_rejects_non_power_of_two(oracle):
    for avg in (0, 3, 100, 64 * KiB + 1, 3 * MiB):
        with pytest.raises(ValueError, match="not a power of two"):
            oracle.Chunker(avg)
    oracle.Chunker(1)
    oracle.Chunker(1 << 40)


def test_chunker1_feed_invariance(oracle):
    """test_chunker1 (chunker.rs:202-271): 1 MiB LE-u32 counter at 64 KiB; feeding single
    bytes gives the same (offset, len) list as feeding the remaining buffer."""
    buf = oracle.gen_counter(1 * MiB)
    c = oracle.Chunker(64 * KiB)
    chunks1, last = [], 0
    for pos in range(buf.size):  # test1: single bytes
        if c.scan(buf[pos:pos + 1]) != 0:
            chunks1.append((last, pos + 1 - last))
            last = pos + 1
    chunks1.append((last, buf.size - last))
    c = oracle.Chunker(64 * KiB)
    chunks2, pos = [], 0
    while pos < buf.size:  # test2: whole remaining buffer
        k = c.scan(buf[pos:])
        if k == 0:
            break
        chunks2.append((pos, k))
        pos += k
    chunks2.append((pos, buf.size - pos))
    assert chunks1 == chunks2
    assert sum(n for _, n in chunks1) == 1 * MiB


def test_survey_vector(oracle):
    """SURVEY.md section 0.6 (independent transliteration): cuts at 143377, 405521,
    667665, 929809, tail 118767."""
    cuts = oracle.chunk_feed(64 * KiB, oracle.gen_counter(1 * MiB))
    assert cuts.tolist() == [143377, 405521, 667665, 929809]
    assert 1 * MiB - int(cuts[-1]) == 118767


@pytest.mark.parametrize("gen", ["counter", "random", "vmimage"])
def test_generators_match_numpy(oracle, gen):
    for off, n in ((0, 4096), (8, 1000), (5, 777), ((1 << 30) - 64 * MiB * 0 + 123, 5000),
                   (512 * MiB - 100, 300)):
        if gen == "counter":
            a, b = oracle.gen_counter(n, off), gen_np.gen_counter(n, off)
        elif gen == "random":
            a, b = oracle.gen_random(n, 0x5EED0002, off), gen_np.gen_random(n, 0x5EED0002, off)
        else:
            a, b = oracle.gen_vmimage(n, 0x5EED0003, off), gen_np.gen_vmimage(n, 0x5EED0003, off)
        assert np.array_equal(a, b), (gen, off, n)
        # the word-at-a-time generator of the long golden streams writes the same bytes
        seed = {"counter": 0, "random": 0x5EED0002, "vmimage": 0x5EED0003}[gen]
        assert np.array_equal(a, oracle.gen_block(gen, n, seed, off)), (gen, off, n)
    # page and extent edges of the VM image in word steps
    for off, n in (((1 << 30) - 5 * 4096 - 3, 11 * 4096 + 7), (512 * MiB - 4096 - 5, 3 * 4096 + 11)):
        assert np.array_equal(oracle.gen_vmimage(n, 0x5EED0003, off),
                              oracle.gen_block("vmimage", n, 0x5EED0003, off))


def test_vmimage_has_zero_pages_and_extent(oracle):
    d = oracle.gen_vmimage(8 * MiB, 0x5EED0003, 512 * MiB - 4 * MiB)
    pages = d.reshape(-1, 4096)
    zero = (pages == 0).all(axis=1)
    assert zero[:1024].mean() > 0.25 and zero[:1024].mean() < 0.55  # 40 % zero pages
    assert zero[1024:].all()  # the forced 64 MiB extent starts at 512 MiB for this seed


def test_window_hash_purity(oracle):
    """SURVEY.md section 0 property 1: after the fill, the rolling h at p equals the
    direct 64-term XOR of rotl(T[b[p-k]], k mod 32); checked via the candidate set."""
    data = oracle.gen_random(64 * KiB, 11)
    rng = np.random.default_rng(1)
    table = _table_from_oracle_header().astype(np.uint64)

    def direct(p):
        h = 0
        for k in range(64):
            t = int(table[data[p - k]])
            r = k & 31
            h ^= ((t << r) | (t >> (32 - r))) & 0xFFFFFFFF if r else t
        return h

    for p in rng.integers(63, data.size, 200).tolist() + [63, data.size - 1]:
        assert oracle.window_hash(data, p) == direct(p)


def test_constant_data_never_hash_cuts(oracle):
    """Property 2: constant windows hash to 0, so only max-size cuts happen."""
    for val in (0, 0x55, 0xFF):
        d = np.full(3 * 256 * KiB + 100, val, dtype=np.uint8)
        assert oracle.candidates(64 * KiB, d).size == 0
        cuts = oracle.chunk_feed(64 * KiB, d)
        assert np.array_equal(cuts, np.arange(1, cuts.size + 1, dtype=np.uint64) * 256 * KiB)


def test_first_test_at_65(oracle):
    """Property 3: the fill phase never tests, so tiny averages cut every 65 bytes."""
    for avg in (1, 2, 4, 8, 16):
        cuts = oracle.chunk_feed(avg, oracle.gen_random(10000, 5))
        assert np.all(np.diff(np.concatenate([[0], cuts])) == 65), avg


INPUTS = [("counter", lambda n: gen_np.gen_counter(n)),
          ("random", lambda n: gen_np.gen_random(n, 0x5EED0002)),
          ("vm", lambda n: gen_np.gen_vmimage(n, 0x5EED0003, 512 * MiB - (n // 2)))]


@pytest.mark.parametrize("name,mk", INPUTS, ids=[i[0] for i in INPUTS])
@pytest.mark.parametrize("avg", [16, 64, 128, 256, 4096, 64 * KiB, 256 * KiB, 4 * MiB])
def test_two_phase_equivalence(oracle, name, mk, avg):
    """Property 4: candidates + min/max resolve == streaming scan, for any feed."""
    n = 8 * MiB if avg >= 64 * KiB else 512 * KiB
    data = mk(n)
    ref = oracle.chunk_feed(avg, data, 0)
    two = oracle.resolve(avg, oracle.candidates(avg, data), data.size)
    assert np.array_equal(ref, two)


@pytest.mark.parametrize("feed", [1, 7, 65, 4096, 256 * KiB - 3])
def test_feed_granularity(oracle, feed):
    avg = 4096 if feed < 64 else 64 * KiB
    n = 256 * KiB if feed < 64 else 4 * MiB
    data = gen_np.gen_random(n, 0x5EED0001)
    assert np.array_equal(oracle.chunk_feed(avg, data, feed), oracle.chunk_feed(avg, data, 0))


def _golden_cases():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


def _golden_input(case):
    gen = case["generator"]
    if gen == "counter":
        return gen_np.gen_counter(case["length"], case["offset"])
    if gen == "random":
        return gen_np.gen_random(case["length"], case["seed"], case["offset"])
    if gen == "vmimage":
        return gen_np.gen_vmimage(case["length"], case["seed"], case["offset"])
    return np.zeros(case["length"], dtype=np.uint8)


@pytest.mark.parametrize("case", _golden_cases(), ids=lambda c: c["name"])
def test_golden_fixtures(oracle, case):
    data = _golden_input(case)
    cuts = np.load(os.path.join(GOLDEN, case["name"] + ".cuts.npy"), allow_pickle=False)
    assert np.array_equal(oracle.chunk_feed(case["avg"], data, 0), cuts)
    assert cuts.size == case["ncuts"]
    if "ncand" in case:
        cand = np.load(os.path.join(GOLDEN, case["name"] + ".cand.npy"), allow_pickle=False)
        assert np.array_equal(oracle.candidates(case["avg"], data), cand)
