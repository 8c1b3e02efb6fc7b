"""C++ ports of the reference's chunker examples (examples/test_chunk_speed.rs,
test_chunk_speed2.rs, test_chunk_size.rs) over the drop-in host mirror: they build on
CPU, fail loudly without a device, and on the GPU print what the oracle predicts for the
same input (chunk counts, every chunk size, the Welford mean/deviation lines)."""
import math
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")
SEED = 0x5EED0001


@pytest.fixture(scope="module")
def examples(pbschunk):
    subprocess.run(["make", "-s", "-C", EX], check=True)
    return {n: os.path.join(EX, n) for n in ("test_chunk_speed", "test_chunk_speed2", "test_chunk_size")}


def test_examples_fail_loudly_without_device(examples, pbschunk):
    if pbschunk.device_count() > 0:
        pytest.skip("device visible: covered by the gpu tests")
    for exe, args in ((examples["test_chunk_speed"], ["1000", "1"]),
                      (examples["test_chunk_speed2"], ["-", "100000"]),
                      (examples["test_chunk_size"], ["100000"])):
        r = subprocess.run([exe, *args], capture_output=True, text=True)
        assert r.returncode == 1 and "no HIP device" in r.stdout, (exe, r.stdout)


@pytest.mark.gpu
@pytest.mark.parametrize("words,passes", [(1 << 20, 5), (777777, 3)])
def test_chunk_speed_example(examples, gpu, oracle, words, passes):
    # test_chunk_speed.rs:21-36: the chunker state carries across passes, so the count
    # is the oracle's over the buffer repeated `passes` times
    r = subprocess.run([examples["test_chunk_speed"], str(words), str(passes)], capture_output=True,
                       text=True, check=True, timeout=120)
    buf = np.arange(words, dtype="<u4").view(np.uint8)
    ref = oracle.chunk_feed(64 * 1024, np.tile(buf, passes))
    out = dict(ln.split(" ", 1) for ln in r.stdout.strip().splitlines())
    assert int(out["CHUNKS"]) == len(ref)
    assert out["SPEED"].startswith("= ") and "avg chunk size" in out["SPEED"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,piece,avg", [(3 << 20, 8192, 65536), (1 << 20, 1000, 4096), (5 << 20, 65536, 4 << 20)])
def test_chunk_speed2_example(examples, gpu, oracle, n, piece, avg):
    r = subprocess.run([examples["test_chunk_speed2"], "-", str(n), str(piece), str(avg)], capture_output=True,
                       text=True, check=True, timeout=120)
    sizes = [int(ln.split()[2]) for ln in r.stdout.splitlines() if ln.startswith("Got chunk ")]
    ends = oracle.chunk_feed(avg, oracle.gen_random(n, SEED)).tolist()
    bounds = [0] + ends + ([n] if not ends or ends[-1] != n else [])
    assert sizes == [b - a for a, b in zip(bounds, bounds[1:])]
    assert f"Uploaded {len(sizes)} chunks" in r.stdout
    assert f"Average chunk size was {n // len(sizes)} bytes." in r.stdout
    # the default is the unchanged caller (one scan() per read); the gathering mode's
    # rate is printed beside it, over the same chunks
    assert f"beside: min_scan 4194304 (4 MiB gathered per scan): {len(sizes)} chunks" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("limit,avg", [(8 << 20, 65536), (3 << 20, 4096)])
def test_chunk_size_example(examples, gpu, oracle, limit, avg):
    # test_chunk_size.rs:98-113: 64 KiB writes until more than `limit` bytes
    r = subprocess.run([examples["test_chunk_size"], str(limit), str(avg)], capture_output=True, text=True,
                       check=True, timeout=120)
    total = (limit // 65536 + 1) * 65536
    ends = oracle.chunk_feed(avg, oracle.gen_random(total, SEED)).tolist()
    sizes = np.diff([0] + ends).astype(float)
    lines = r.stdout.strip().splitlines()
    assert len(lines) == len(sizes)
    # Welford as in test_chunk_size.rs:38-64
    m_old = s_old = 0.0
    for i, (ln, x) in enumerate(zip(lines, sizes), 1):
        if i == 1:
            m_new, s_new = x, 0.0
        else:
            m_new = m_old + (x - m_old) / i
            s_new = s_old + (x - m_old) * (x - m_new)
        m_old, s_old = m_new, s_new
        dev = math.sqrt(s_new / (i - 1) if i > 1 else 0.0) * 100.0 / m_new
        f = ln.split()
        assert (int(f[1]), int(f[3]), int(f[5]), int(f[7].rstrip("%"))) == (i, int(x), int(m_new), int(dev)), ln
