"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle and the
golden fixtures.  Bit-exact comparison of candidate positions and cut lists.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import json
import os
import threading

import numpy as np
import pytest

import gen_np

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KiB, MiB, GiB = 1024, 1024 * 1024, 1024 * 1024 * 1024


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


# ---------------------------------------------------------------- phase A (candidates)

def _holes(n: int, seed: int, max_run: int = 20000) -> np.ndarray:
    """Random bytes punched with zero runs of random length and alignment (the scan
    kernel skips all-zero 128-byte blocks that follow an all-zero block)."""
    rng = np.random.default_rng(seed)
    d = gen_np.gen_random(n, seed)
    pos = 0
    while pos < n:
        pos += int(rng.integers(1, 3000))
        ln = int(rng.choice([int(rng.integers(1, max_run)), 64, 127, 128, 129, 255, 256, 257]))
        d[pos:pos + ln] = 0
        pos += ln
    return d


CAND_CASES = [
    # (name, maker, avg) -- sizes cover exact-only (< 1 MiB wave tile), several wave tiles
    # plus a ragged tail, and dense candidates (tiny averages) that overflow the first
    # suspect/candidate capacity estimate.
    ("random_3M+77_64K", lambda: gen_np.gen_random(3 * MiB + 77, 0x5EED0002), 64 * KiB),
    ("random_3M+77_16", lambda: gen_np.gen_random(3 * MiB + 77, 0x5EED0002), 16),
    ("random_2M+5_128", lambda: gen_np.gen_random(2 * MiB + 5, 3), 128),
    ("random_700K_4096", lambda: gen_np.gen_random(700 * KiB + 1, 4), 4096),
    ("random_40M+3_256K", lambda: gen_np.gen_random(40 * MiB + 3, 5), 256 * KiB),
    ("counter_20M_64K", lambda: gen_np.gen_counter(20 * MiB), 64 * KiB),
    ("vm_64M_4M", lambda: gen_np.gen_vmimage(64 * MiB, 0x5EED0003, 500 * MiB), 4 * MiB),
    ("zeros_5M_64K", lambda: np.zeros(5 * MiB, np.uint8), 64 * KiB),
    ("tiny_100_64", lambda: gen_np.gen_random(100, 1), 64),
    ("empty_64", lambda: np.zeros(0, np.uint8), 64),
    ("random_4M_avg2", lambda: gen_np.gen_random(4 * MiB, 9), 2),
    ("random_1M_avg1", lambda: gen_np.gen_random(1 * MiB, 9), 1),
    ("holes_8M_256", lambda: _holes(8 * MiB + 5, 31), 256),
    ("holes_24M_4096", lambda: _holes(24 * MiB, 32, 200000), 4096),
    ("holes_6M_64", lambda: _holes(6 * MiB + 1, 33, 1000), 64),
]


@pytest.mark.parametrize("name,mk,avg", CAND_CASES, ids=[c[0] for c in CAND_CASES])
def test_candidates_match_oracle(gpu, oracle, name, mk, avg):
    data = mk()
    got = gpu.candidates_host(data, avg)
    ref = oracle.candidates(avg, data)
    assert np.array_equal(got, ref), (name, got.size, ref.size)


def test_candidates_golden(gpu):
    for case in _golden_cases():
        if "ncand" not in case:
            continue
        data = _golden_input(case)
        ref = np.load(os.path.join(GOLDEN, case["name"] + ".cand.npy"), allow_pickle=False)
        assert np.array_equal(gpu.candidates_host(data, case["avg"]), ref), case["name"]


# ---------------------------------------------------------------- cut lists

@pytest.mark.parametrize("case", _golden_cases(), ids=lambda c: c["name"])
def test_find_cuts_golden(gpu, case):
    data = _golden_input(case)
    ref = np.load(os.path.join(GOLDEN, case["name"] + ".cuts.npy"), allow_pickle=False)
    with gpu.Chunker(case["avg"]) as c:
        got = c.find_cuts(data, is_final=False)
    assert np.array_equal(got, ref), (case["name"], got[:5], ref[:5])


def test_find_cuts_final_tail(gpu, oracle):
    data = gen_np.gen_random(5 * MiB + 11, 77)
    ref = oracle.chunk_feed(256 * KiB, data)
    with gpu.Chunker(256 * KiB) as c:
        got = c.find_cuts(data, is_final=True)
        assert np.array_equal(got[:-1], ref) and int(got[-1]) == data.size
        assert c.stream_offset == 0  # handle restarted
        again = c.find_cuts(data, is_final=True)  # a fresh stream gives the same cuts
    assert np.array_equal(again, got)


@pytest.mark.parametrize("avg", [64, 4096, 64 * KiB, 4 * MiB])
def test_find_cuts_split_calls(gpu, oracle, avg):
    """State carried across calls (carry bytes, open chunk, pending candidates)."""
    n = 24 * MiB if avg >= 64 * KiB else 1 * MiB
    data = gen_np.gen_vmimage(n, 0x5EED0003, 512 * MiB - n // 3)
    ref = oracle.chunk_feed(avg, data)
    rng = np.random.default_rng(avg)
    cuts = np.concatenate([[0], np.sort(rng.choice(np.arange(1, n), 12, replace=False)), [n]])
    got = []
    with gpu.Chunker(avg) as c:
        for a, b in zip(cuts[:-1], cuts[1:]):
            got.append(c.find_cuts(data[a:b]))
            assert c.stream_offset == b
    got = np.concatenate(got)
    assert np.array_equal(got, ref)


def test_find_cuts_device(gpu, oracle):
    import torch
    n = 48 * MiB + 8
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n, gpu.GEN_VMIMAGE, 0x5EED0003, 480 * MiB)
    host = dev.cpu().numpy()
    assert np.array_equal(host, oracle.gen_vmimage(n, 0x5EED0003, 480 * MiB))
    ref = oracle.chunk_feed(1 * MiB, host)
    with gpu.Chunker(1 * MiB) as c:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        half = 20 * MiB + 3
        g1 = c.find_cuts_device(dev.data_ptr(), half)
        g2 = c.find_cuts_device(dev.data_ptr() + half, n - half, is_final=True)
        t = c.last_timing()
    got = np.concatenate([g1, g2])
    assert np.array_equal(got[:-1], ref) and int(got[-1]) == n
    assert t["bytes"] == n - half and t["total_ms"] > 0


def test_find_cuts_device_into_pinned_out(gpu, oracle):
    """find_cuts_device(out=...) as bench.py times it: the cut list DMA'd into a pinned
    host array (64 KiB averages: a long list), the oracle's cuts, and a too-small or
    wrongly typed array refused."""
    import torch
    n = 40 * MiB + 8  # the generator writes whole 8-byte words
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n, gpu.GEN_RANDOM, 0x5EED0002, 0)
    host = dev.cpu().numpy()
    ref = oracle.chunk_feed(64 * KiB, host)
    with gpu.Chunker(64 * KiB) as c:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        out = torch.empty(c.cuts_bound(n), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
        for _ in range(2):  # the same array reused
            got = c.find_cuts_device(dev.data_ptr(), n, is_final=True, out=out)
            assert np.array_equal(got[:-1], ref) and int(got[-1]) == n
        with pytest.raises(ValueError):
            c.find_cuts_device(dev.data_ptr(), n, is_final=True, out=out[:8])
        with pytest.raises(ValueError):
            c.find_cuts_device(dev.data_ptr(), n, is_final=True, out=out.view(np.int64))
        ro = np.frombuffer(bytes(8 * c.cuts_bound(n)), dtype=np.uint64)  # read-only
        with pytest.raises(ValueError):
            c.find_cuts_device(dev.data_ptr(), n, is_final=True, out=ro)


def _zebra(n_runs: int, zero_run: int, rand_run: int, seed: int) -> np.ndarray:
    """Zero runs (no candidates -> long forced-cut runs) between random runs."""
    r = gen_np.gen_random(n_runs * rand_run, seed)
    out = np.zeros(n_runs * (zero_run + rand_run), np.uint8)
    for i in range(n_runs):
        a = i * (zero_run + rand_run) + zero_run
        out[a:a + rand_run] = r[i * rand_run:(i + 1) * rand_run]
    return out


# The resolve runs in one workgroup up to 16384 - 2 candidates (pending + new) and in the
# multi-kernel sort + pointer-doubling path above that: sizes straddle the switch (random
# bytes at avg 256 give ~3/512 candidates per byte), and forced-cut runs of >= 256 cuts
# per node exercise the block-filled list, including more than its 64 entries.
RESOLVE_CASES = [
    ("random_2.5M_256", lambda: gen_np.gen_random(2 * MiB + 512 * KiB, 21), 256),
    ("random_2.75M_256", lambda: gen_np.gen_random(2 * MiB + 768 * KiB + 13, 22), 256),
    ("random_2.9M_256", lambda: gen_np.gen_random(2 * MiB + 920 * KiB, 23), 256),
    ("random_6M_256", lambda: gen_np.gen_random(6 * MiB + 1, 24), 256),
    ("zeros_1M_64", lambda: np.zeros(1 * MiB, np.uint8), 64),
    ("zeros_9M_4096", lambda: np.zeros(9 * MiB + 3, np.uint8), 4096),
    ("zebra_100x128K_64", lambda: _zebra(100, 128 * KiB, 4 * KiB, 25), 64),
    ("zebra_30x8M_4096", lambda: _zebra(30, 8 * MiB, 64 * KiB, 26), 4096),
]


@pytest.mark.parametrize("name,mk,avg", RESOLVE_CASES, ids=[c[0] for c in RESOLVE_CASES])
def test_resolve_paths(gpu, oracle, name, mk, avg):
    data = mk()
    ref = oracle.chunk_feed(avg, data)
    if ref.size == 0 or int(ref[-1]) != data.size:  # the EOF tail chunk, if any
        ref = np.append(ref, np.uint64(data.size))
    with gpu.Chunker(avg) as c:
        got = c.find_cuts(data, is_final=True)
        t = c.last_timing()
    assert np.array_equal(got, ref), (name, t["candidates"], got.size, ref.size)
    # split in two calls: the open chunk's candidates come back as pending
    h = data.size // 2 + 7
    with gpu.Chunker(avg) as c:
        got2 = np.concatenate([c.find_cuts(data[:h]), c.find_cuts(data[h:], is_final=True)])
    assert np.array_equal(got2, got), name


# Batches of <= 1 MiB take the small-input path (block scan + one-workgroup resolve, one
# sync); more than ~16K candidates in such a batch (avg 16/64) falls back to the
# regular path; 1 MiB + 1 is the first size on the regular path.
@pytest.mark.parametrize("avg,piece", [(4 * MiB, 256 * KiB), (64 * KiB, 64 * KiB + 3),
                                       (256, 1 * MiB), (64, 1 * MiB), (16, 300 * KiB),
                                       (4096, 1 * MiB + 1), (1 * MiB, 7)])
def test_small_batches(gpu, oracle, avg, piece):
    n = 6 * MiB + 11 if piece > 64 else 64 * KiB
    data = gen_np.gen_vmimage(n, 0x5EED0003, 300 * MiB + 4093)
    ref = oracle.chunk_feed(avg, data)
    got = []
    with gpu.Chunker(avg) as c:
        for a in range(0, n, piece):
            got.append(c.find_cuts(data[a:a + piece], is_final=a + piece >= n))
    got = np.concatenate(got)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("kind,n,avg", [("vmimage", 192 * MiB + 5, 64 * KiB), ("random", 96 * MiB, 64 * KiB),
                                        ("random", 40 * MiB + 3, 64 * KiB), ("vmimage", 160 * MiB + 3, 128 * KiB),
                                        ("random", 72 * MiB, 128 * KiB), ("random", 200 * MiB + 7, 256 * KiB),
                                        ("vmimage", 256 * MiB, 256 * KiB)])
def test_scan_pass(gpu, oracle, kind, n, avg):
    """64, 128 and 256 KiB averages: scan_fused_kernel without resolver waves, the records' candidates
    gathered in stream order, the multi-kernel resolve -- whole, and split into three calls
    (pending candidates of the open chunk carried over), against the oracle."""
    import torch
    n8 = (n + 7) // 8 * 8  # (the generator fills whole 8-byte words; n itself is ragged)
    dev = torch.empty(n8, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n8, gpu.GEN_VMIMAGE if kind == "vmimage" else gpu.GEN_RANDOM,
                        0x5EED0003, 7 * GiB)
    host = dev[:n].cpu().numpy()
    ref = oracle.chunk_feed(avg, host)
    with gpu.Chunker(avg) as c:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        got = c.find_cuts_device(dev.data_ptr(), n, is_final=True)
        t = c.last_timing()
    assert t["scan_pass"] == t["fused"] == t["bytes"] == n, t  # the scan pass served the whole stream
    assert np.array_equal(got[:-1], ref) and int(got[-1]) == n
    cuts = [n // 3 + 1, 2 * n // 3 + 4093]
    parts = []
    with gpu.Chunker(avg) as c:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        for a, b in zip([0] + cuts, cuts + [n]):
            parts.append(c.find_cuts_device(dev.data_ptr() + a, b - a, is_final=b == n))
    assert np.array_equal(np.concatenate(parts), got)
    # into a pinned cut array, as bench.py times it: the resolve writes the cuts there
    # itself (and the open chunk's candidates to mapped memory), whole and split
    with gpu.Chunker(avg) as c:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        out = torch.empty(c.cuts_bound(n), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
        out[:] = 7
        assert np.array_equal(c.find_cuts_device(dev.data_ptr(), n, is_final=True, out=out), got)
        parts = [c.find_cuts_device(dev.data_ptr(), cuts[0], out=out).copy()]
        parts.append(c.find_cuts_device(dev.data_ptr() + cuts[0], cuts[1] - cuts[0], out=out).copy())
        parts.append(c.find_cuts_device(dev.data_ptr() + cuts[1], n - cuts[1], is_final=True, out=out).copy())
    assert np.array_equal(np.concatenate(parts), got)


def test_small_batches_device(gpu, oracle):
    import torch
    n, avg = 5 * MiB + 24, 256 * KiB
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n, gpu.GEN_VMIMAGE, 0x5EED0003, 96 * MiB)
    ref = oracle.chunk_feed(avg, dev.cpu().numpy())
    got = []
    with gpu.Chunker(avg) as c:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        for a in range(0, n, 777 * KiB + 5):  # unaligned device pieces
            b = min(n, a + 777 * KiB + 5)
            got.append(c.find_cuts_device(dev.data_ptr() + a, b - a))
    assert np.array_equal(np.concatenate(got), ref)


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_device_generator_matches_oracle(gpu, oracle, kind):
    import torch
    n, off = 3 * MiB + 8, 1 * GiB - 1 * MiB
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n, kind, 0x5EED0002, off)
    host = dev.cpu().numpy()
    ref = [oracle.gen_counter(n, off), oracle.gen_random(n, 0x5EED0002, off),
           oracle.gen_vmimage(n, 0x5EED0002, off)][kind]
    assert np.array_equal(host, ref)


# ---------------------------------------------------------------- scan() drop-in surface

@pytest.mark.parametrize("feed,avg,n", [(1, 1024, 24 * KiB), (7, 256, 64 * KiB),
                                        (65, 4096, 256 * KiB), (4096, 64 * KiB, 3 * MiB),
                                        (256 * KiB, 64 * KiB, 12 * MiB),
                                        # scan server passes (8 KiB): ragged multi-pass
                                        # requests, dense hits, the largest request, and a
                                        # request with more hits than the mailbox holds
                                        (12345, 64, 1 * MiB), (8192, 2, 256 * KiB),
                                        (1 * MiB, 2 * KiB, 5 * MiB + 17), (8192, 4 * MiB, 24 * MiB),
                                        (64 * KiB, 2, 512 * KiB)])
def test_scan_feed_granularity(gpu, oracle, feed, avg, n):
    """test_chunker1 (chunker.rs:202-271) style: same cuts for any feed size."""
    data = gen_np.gen_random(n, feed)
    ref = oracle.chunk_feed(avg, data, feed)
    assert np.array_equal(ref, oracle.chunk_feed(avg, data, 0))
    got = []
    with gpu.Chunker(avg) as c:
        for piece in range(0, n, feed):
            p = data[piece:piece + feed]
            off = 0
            while off < p.size:
                k = c.scan(p[off:])
                if k == 0:
                    break
                off += k
                got.append(piece + off)
    assert np.array_equal(np.array(got, dtype=np.uint64), ref)


SERVER_MODES = {  # PBS_SERVER_VRAM, PBS_SERVER_VRAM_MAX, PBS_SERVER_WGS
    "vram": ("1", None, None),             # default: BAR-written slot, requests split over 16 WGs
    "vram-host-slot": ("1", "131072", None),  # requests over 128 KiB split, read from the pinned slot
    "vram-one-wg": ("1", None, "1"),       # the one-workgroup server
    "pinned": ("0", None, None),           # record + slot in pinned host memory (one workgroup)
}


@pytest.mark.parametrize("mode", list(SERVER_MODES))
@pytest.mark.parametrize("feed,avg", [(8192, 64 * KiB), (256 * KiB + 3, 64 * KiB),
                                      (1 * MiB, 64 * KiB), (1 * MiB, 1 * KiB)])
def test_scan_server_request_placement(gpu, oracle, monkeypatch, mode, feed, avg):
    """scan() per read with the server's request record + slot in BAR-written VRAM (default),
    long requests in the pinned slot, one workgroup, and everything in pinned host memory
    (PBS_SERVER_VRAM=0): the oracle's cuts every way, over many requests that reuse the
    same slots (stale lines would show here); avg 1 KiB puts hundreds of candidates of
    one request in every workgroup's range (each workgroup's own region of the array)."""
    for var, val in zip(("PBS_SERVER_VRAM", "PBS_SERVER_VRAM_MAX", "PBS_SERVER_WGS"), SERVER_MODES[mode]):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, val)
    n = 6 * MiB + 333
    data = gen_np.gen_random(n, 0x5EED0011)
    ref = oracle.chunk_feed(avg, data, 0)
    got = []
    with gpu.Chunker(avg) as c:
        for piece in range(0, n, feed):
            p = data[piece:piece + feed]
            off = 0
            while off < p.size:
                k = c.scan(p[off:])
                if k == 0:
                    break
                off += k
                got.append(piece + off)
    assert np.array_equal(np.array(got, dtype=np.uint64), ref)


@pytest.mark.parametrize("wgs,minpass", [(None, None), ("3", None), ("32", "1")])
@pytest.mark.parametrize("avg", [4 * KiB, 64 * KiB])
def test_scan_server_ragged_reads(gpu, oracle, monkeypatch, wgs, minpass, avg):
    """scan() over reads of seeded ragged sizes (1 byte to 1.5 MiB, many just around the
    server's pass and split sizes), so requests split over the workgroups end at every
    kind of boundary -- also split one pass per workgroup over up to 32 of them; the
    oracle's cuts (chunker.rs:127-181 driven like a reader loop)."""
    for var, val in (("PBS_SERVER_WGS", wgs), ("PBS_SERVER_MINPASS", minpass)):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, val)
    rng = np.random.default_rng(0x5EED0012 + avg)
    n = 12 * MiB + 77
    data = gen_np.gen_random(n, 0x5EED0013)
    ref = oracle.chunk_feed(avg, data, 0)
    sizes = []
    while sum(sizes) < n:
        kind = rng.integers(0, 4)
        if kind == 0:
            sizes.append(int(rng.integers(1, 64)))
        elif kind == 1:
            base = int(rng.choice([4096, 8192, 16384, 65536, 131072, 262144]))
            sizes.append(max(1, base + int(rng.integers(-65, 66))))
        else:
            sizes.append(int(rng.integers(1, 3 * MiB // 2)))
    got, pos = [], 0
    with gpu.Chunker(avg) as c:
        for s in sizes:
            p = data[pos:pos + s]
            off = 0
            while off < p.size:
                k = c.scan(p[off:])
                if k == 0:
                    break
                off += k
                got.append(pos + off)
            pos += p.size
    assert np.array_equal(np.array(got, dtype=np.uint64), ref)


def test_chunker1_whole_buffer(gpu):
    """test_chunker1's test2 loop on its own 1 MiB counter buffer (chunker.rs:246-257)."""
    buf = gen_np.gen_counter(1 * MiB)
    with gpu.Chunker(64 * KiB) as c:
        chunks, pos = [], 0
        while pos < buf.size:
            k = c.scan(buf[pos:])
            if k == 0:
                break
            chunks.append((pos, k))
            pos += k
    assert [p + k for p, k in chunks] == [143377, 405521, 667665, 929809]
    assert buf.size - pos == 118767


def test_test_chunk_speed_loop(gpu, oracle):
    """examples/test_chunk_speed.rs: 5 passes over an 80 MiB counter at 64 KiB with the
    chunker state carried across passes (the chunker is never reset)."""
    buf = oracle.gen_counter(80 * MiB)
    ref_c = oracle.Chunker(64 * KiB)
    with gpu.Chunker(64 * KiB) as c:
        for _ in range(2):
            pos = 0
            while pos < buf.size:
                k = c.scan(buf[pos:])
                r = ref_c.scan(buf[pos:])
                assert k == r
                if k == 0:
                    break
                pos += k


@pytest.mark.parametrize("min_scan", [0, 4 * MiB])
def test_chunk_stream_and_writer(gpu, oracle, min_scan):
    data = gen_np.gen_vmimage(20 * MiB + 5, 0x5EED0003, 510 * MiB)
    ref = oracle.chunk_feed(1 * MiB, data)
    pieces = [data[i:i + 256 * KiB].tobytes() for i in range(0, data.size, 256 * KiB)]
    cs = gpu.ChunkStream(pieces, 1 * MiB)
    cs.min_scan = min_scan
    chunks = list(cs)
    ends = np.cumsum([len(ch) for ch in chunks])
    assert b"".join(chunks) == data.tobytes()
    assert np.array_equal(ends[:-1], ref) and ends[-1] == data.size
    got = []
    w = gpu.DynamicChunkWriter(lambda end, b: got.append(end), 1 * MiB)
    for i in range(0, data.size, 64 * KiB):
        w.write_all(data[i:i + 64 * KiB].tobytes())
    w.close()
    assert np.array_equal(np.array(got[:-1], dtype=np.uint64), ref) and got[-1] == data.size


def test_invalid_arguments(gpu):
    with pytest.raises(ValueError):
        gpu.Chunker(12345)
    with gpu.Chunker(4 * MiB) as c:
        assert c.scan(b"") == 0
        assert c.find_cuts(b"").size == 0


# ---------------------------------------------------------------- full-size (config 2)

def _oracle_two_phase_parallel(oracle, data: np.ndarray, avg: int, threads: int = 16):
    """Multi-threaded oracle: phase-A candidates per segment (63-byte overlap; ctypes
    releases the GIL), then the oracle's resolve.  Equivalent to the streaming oracle
    (tests/test_oracle.py::test_two_phase_equivalence)."""
    n = data.size
    seg = (n + threads - 1) // threads
    parts = [None] * threads

    def work(t):
        a, b = t * seg, min(n, (t + 1) * seg)
        if a >= b:
            parts[t] = np.zeros(0, np.uint64)
            return
        lo = max(0, a - 63)
        c = oracle.candidates(avg, data[lo:b]).astype(np.uint64) + np.uint64(lo)
        parts[t] = c[c >= a]

    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    cand = np.concatenate(parts)
    return cand, oracle.resolve(avg, cand, n)


@pytest.mark.slow
@pytest.mark.parametrize("gib,kind,avg,dyn,fused",
                         [(8, 1, 4 * MiB, None, None), (6, 2, 256 * KiB, None, None),
                          (3, 1, 64 * KiB, None, None), (64, 2, 4 * MiB, None, None),
                          (64, 2, 256 * KiB, None, None),
                          (6, 2, 4 * MiB, "1", None), (3, 1, 64 * KiB, "1", None),
                          (1.5, 2, 1 * MiB, "1", None),
                          (8, 1, 4 * MiB, None, "0"), (8, 1, 4 * MiB, None, "1"),
                          (5.5, 2, 256 * KiB, None, "1"), (16.25, 1, 1 * MiB, None, "1")],
                         ids=["config2-8GiB-random-4M", "6GiB-vm-256K", "3GiB-random-64K",
                              "config3-64GiB-vm-4M", "config5-64GiB-vm-256K",
                              "6GiB-vm-4M-dynamic", "3GiB-random-64K-dynamic",
                              "1.5GiB+ragged-vm-1M-dynamic",
                              "config2-8GiB-random-4M-multi-launch",
                              "config2-8GiB-random-4M-fused-static",
                              "5.5GiB+ragged-vm-256K-fused-static",
                              "16.25GiB+ragged-random-1M-fused-static"])
def test_full_size_in_hbm(gpu, oracle, monkeypatch, gib, kind, avg, dyn, fused):
    """BASELINE config 2 (8 GiB random already in HBM, 4 MiB average), the headline
    config 3 (64 GiB VM image, 4 MiB: 16 KiB segments in the dynamic tile order), and
    sizes that select the other scan_main segment lengths (16 KiB, 8 KiB) in both tile
    orders (PBS_SCAN_DYN forces the dynamic one), and the one-launch pass in the static
    tile order (PBS_FUSED=1: runtime segment lengths, one block longer for the first
    tiles, 1-3 tiles per scanner wave, an 8 KiB tail) against the multi-launch path
    (PBS_FUSED=0): the full cut list is diffed against the (multi-threaded two-phase)
    oracle."""
    import torch
    if dyn is not None:
        monkeypatch.setenv("PBS_SCAN_DYN", dyn)
    if fused is not None:
        monkeypatch.setenv("PBS_FUSED", fused)
    n = int(gib * GiB) + (12345 if gib != int(gib) else 0)  # ragged: the tail after the small tiles
    seed = 0x5EED0002 if kind == 1 else 0x5EED0003
    n8 = (n + 7) // 8 * 8  # the generator writes whole words
    dev = torch.empty(n8, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n8, kind, seed, 0)
    with gpu.Chunker(avg) as c:
        got = c.find_cuts_device(dev.data_ptr(), n, is_final=False)
        t = c.last_timing()
    host = dev[:n].cpu().numpy()
    del dev
    cand, ref = _oracle_two_phase_parallel(oracle, host, avg)
    assert t["candidates"] == cand.size
    assert np.array_equal(got, ref)
    # spot-check against the streaming oracle on the first 256 MiB
    head = oracle.chunk_feed(avg, host[:256 * MiB])
    assert np.array_equal(got[:head.size], head)


# ---------------------------------------------------------------- dense periodic input

def _passing_pattern(oracle, period: int, avg: int) -> np.ndarray:
    """Random bytes of length `period` whose periodic continuation has a window hash that
    passes the cut test at some phase (then every period-th byte is a candidate)."""
    mask = 2 * avg - 1
    for seed in range(1, 1 << 20):
        pat = gen_np.gen_random(period, seed)
        buf = np.tile(pat, 64 // period + 3)
        if any((oracle.window_hash(buf, 63 + k) & mask) >= mask - 2 for k in range(period)):
            return pat
    raise AssertionError("no passing pattern")


def test_periodic_dense_candidates(gpu, oracle):
    """A period-7 stream whose window hash passes the test makes every 7th byte a
    candidate: 153 M candidates in 1 GiB, more than one batch may hold (the scan redoes
    it as shorter batches; 64-bit candidate counters), at a 4 KiB average whose chunks
    are ~1 KiB.  The cut list equals the oracle's."""
    import torch
    pat = _passing_pattern(oracle, 7, 4096)
    n = (1 << 30) + 13
    host = np.tile(pat, n // 7 + 1)[:n]
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    with gpu.Chunker(4096) as c:
        got = c.find_cuts_device(dev.data_ptr(), n, is_final=True)
        t = c.last_timing()
    del dev
    ref = oracle.chunk_feed(4096, host)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert t["candidates"] > (1 << 27) // 4  # dense: the batches were shrunk
    assert np.array_equal(got, ref)


def test_scan_pass_dense_falls_back(gpu, oracle):
    """At 64 KiB averages a period-7 stream whose window hash passes makes every 128-byte
    block a flagged one: every tile of the scan pass overflows its four records, and the
    batch goes through the multi-launch path instead -- same cuts as the oracle."""
    import torch
    pat = _passing_pattern(oracle, 7, 64 * KiB)
    n = 48 * MiB + 5
    host = np.tile(pat, n // 7 + 1)[:n]
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    with gpu.Chunker(64 * KiB) as c:
        got = c.find_cuts_device(dev.data_ptr(), n, is_final=True)
        t = c.last_timing()
    del dev
    ref = oracle.chunk_feed(64 * KiB, host)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert t["fused"] == 0 and t["scan_pass"] == 0, t  # the scan pass stood down
    assert np.array_equal(got, ref)


# ---------------------------------------------------------------- fused pass (scan_fused.h)

FUSED_CASES = [
    # (name, maker, avg, pieces): batches > 1 MiB at avg >= 128 KiB take the one-launch
    # pass; pieces carry the open chunk's candidates and the 63-byte history across calls
    ("vm_40M+77_128K", lambda: gen_np.gen_vmimage(40 * MiB + 77, 0x5EED0003, 700 * MiB), 128 * KiB, 1),
    ("random_33M_256K_x5", lambda: gen_np.gen_random(33 * MiB + 5, 41), 256 * KiB, 5),
    ("holes_48M_1M_x3", lambda: _holes(48 * MiB + 3, 42, 3 * MiB), 1 * MiB, 3),
    ("zebra_8x3M_4M", lambda: _zebra(8, 3 * MiB, 512 * KiB, 43), 4 * MiB, 2),
    ("counter_24M_128K", lambda: gen_np.gen_counter(24 * MiB), 128 * KiB, 1),
    ("zeros_70M_4M_x2", lambda: np.zeros(70 * MiB + 1, np.uint8), 4 * MiB, 2),
    # forced-cut runs between candidate runs, candidates packed near the 64-block limit
    ("zebra_64x(600K+200K)_128K", lambda: _zebra(64, 600 * KiB, 200 * KiB, 45), 128 * KiB, 3),
    ("vm_300M_128K", lambda: gen_np.gen_vmimage(300 * MiB, 0x5EED0003, 3 * GiB), 128 * KiB, 1),
    ("random_200M_256K_x7", lambda: gen_np.gen_random(200 * MiB + 9, 46), 256 * KiB, 7),
    # 64 KiB averages forced through the one-launch pass (the product serves them with the
    # scan pass; random bytes make it stand down: > 64 flagged blocks per tile)
    ("vm_96M+5_64K_x3", lambda: gen_np.gen_vmimage(96 * MiB + 5, 0x5EED0003, 9 * GiB), 64 * KiB, 3),
    ("random_72M+3_64K_x2", lambda: gen_np.gen_random(72 * MiB + 3, 47), 64 * KiB, 2),
    ("holes_64M_64K_x4", lambda: _holes(64 * MiB + 11, 48, 2 * MiB), 64 * KiB, 4),
]


@pytest.mark.parametrize("name,mk,avg,pieces", FUSED_CASES, ids=[c[0] for c in FUSED_CASES])
def test_fused_pass(gpu, oracle, monkeypatch, name, mk, avg, pieces):
    """The one-launch pass (scan + exact + resolve in scan_fused_kernel) against the oracle
    and against the multi-launch path (PBS_FUSED=0), whole and split into pieces."""
    data = mk()
    n = data.size
    ref = oracle.chunk_feed(avg, data)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    bounds = np.linspace(0, n, pieces + 1).astype(np.int64)
    bounds[1:-1] += 4093  # unaligned piece starts
    for fused in ("1", "0"):
        monkeypatch.setenv("PBS_FUSED", fused)
        monkeypatch.setenv("PBS_FUSED_MIN_AVG", "65536")
        got = []
        with gpu.Chunker(avg) as c:
            for a, b in zip(bounds[:-1], bounds[1:]):
                got.append(c.find_cuts(data[a:b], is_final=b == n))
        got = np.concatenate(got)
        assert np.array_equal(got, ref), (name, fused, got.size, ref.size)


@pytest.mark.parametrize("kind,avg", [(1, 64 * KiB), (2, 64 * KiB), (2, 128 * KiB), (1, 4 * MiB)],
                         ids=["random-64K", "vm-64K", "vm-128K", "random-4M"])
def test_fused_pass_pinned_out(gpu, oracle, monkeypatch, kind, avg):
    """A pass from HBM into the caller's pinned cut array (as bench.py hands it), 640 MiB + 5
    split in two calls, the one-launch pass forced from 64 KiB: the oracle's cuts (random
    bytes at 64 KiB stand down to the multi-launch path)."""
    import torch
    monkeypatch.setenv("PBS_FUSED", "1")
    monkeypatch.setenv("PBS_FUSED_MIN_AVG", "65536")
    n = 640 * MiB + 5
    seed = 0x5EED0002 if kind == 1 else 0x5EED0003
    n8 = (n + 7) // 8 * 8
    dev = torch.empty(n8, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n8, kind, seed, 0)
    host = dev[:n].cpu().numpy()
    got = []
    with gpu.Chunker(avg) as c:
        half = 300 * MiB + 3
        for a, b in ((0, half), (half, n)):
            out = torch.empty(c.cuts_bound(b - a), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
            got.append(c.find_cuts_device(dev.data_ptr() + a, b - a, is_final=b == n, out=out).copy())
            if avg >= 128 * KiB:
                assert c.last_timing()["fused"] == b - a
    del dev
    got = np.concatenate(got)
    ref = oracle.chunk_feed(avg, host)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert np.array_equal(got, ref)


def test_fused_pass_stands_down_on_dense_input(gpu, oracle, monkeypatch):
    """Every 7th byte a candidate at a 256 KiB average: a tile holds far more than 64
    flagged blocks, the fused kernel stands down and the multi-launch path chunks the
    batch -- same cuts as the oracle.  (PBS_FUSED=1: a 24 MiB batch would otherwise take
    the multi-launch path directly.)"""
    monkeypatch.setenv("PBS_FUSED", "1")
    pat = _passing_pattern(oracle, 7, 256 * KiB)
    n = 24 * MiB + 3
    rnd = gen_np.gen_random(n, 44)
    host = rnd.copy()
    host[8 * MiB:16 * MiB] = np.tile(pat, (8 * MiB) // 7 + 1)[:8 * MiB]
    with gpu.Chunker(256 * KiB) as c:
        got = c.find_cuts(host, is_final=True)
    ref = oracle.chunk_feed(256 * KiB, host)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert np.array_equal(got, ref)


@pytest.mark.slow
@pytest.mark.parametrize("gib,kind,avg,div,rnd", [(1, 1, 1 * MiB, 2, 8), (2, 2, 4 * MiB, 4, 8)],
                         ids=["1GiB+ragged-random-1M-pool2", "2GiB+ragged-vm-4M-pool4"])
def test_fused_pass_pool(gpu, oracle, monkeypatch, gib, kind, avg, div, rnd):
    """The static order's pool (pbs_chunker_capi.cpp fused_static_plan: the last, short
    round drawn from a counter as small tiles; by default only from 8 rounds on, i.e. the
    64 GiB headline stream) forced on smaller streams: full cut lists against the oracle."""
    import torch
    monkeypatch.setenv("PBS_FUSED", "1")
    monkeypatch.setenv("PBS_POOL_DIV", str(div))
    monkeypatch.setenv("PBS_POOL_ROUND", str(rnd))
    n = int(gib * GiB) + 12345
    seed = 0x5EED0002 if kind == 1 else 0x5EED0003
    n8 = (n + 7) // 8 * 8
    dev = torch.empty(n8, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n8, kind, seed, 0)
    with gpu.Chunker(avg) as c:
        got = c.find_cuts_device(dev.data_ptr(), n, is_final=False)
        t = c.last_timing()
    host = dev[:n].cpu().numpy()
    del dev
    cand, ref = _oracle_two_phase_parallel(oracle, host, avg)
    assert t["fused"] == n and t["scan_pass"] == 0 and t["candidates"] == cand.size
    assert np.array_equal(got, ref)
