"""CPU checks of the 8(f) host pieces: the library's host SHA-256 (index checksum)
against FIPS 180-4 known answers and hashlib, and the .didx image against the oracle's
restatement of dynamic_index.rs (header layout, entries, index_csum)."""
import hashlib
import os

import numpy as np
import pytest

# FIPS 180-4 / NIST CAVS known answers
KAT = [
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


@pytest.mark.parametrize("msg,hexd", KAT, ids=["empty", "abc", "448bit", "million_a"])
def test_host_sha256_known_answers(pbschunk, msg, hexd):
    assert pbschunk.sha256(msg).hex() == hexd
    assert hashlib.sha256(msg).hexdigest() == hexd  # the oracle's hash agrees too


def test_host_sha256_lengths(pbschunk):
    rng = np.random.default_rng(7)
    for n in list(range(0, 200)) + [4095, 4096, 4097, 65536 + 13]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert pbschunk.sha256(d) == hashlib.sha256(d).digest(), n


@pytest.mark.parametrize("n", [0, 1, 3, 1000])
def test_didx_image_matches_oracle(pbschunk, oracle, n):
    rng = np.random.default_rng(n)
    ends = np.cumsum(rng.integers(65, 1 << 24, n)).astype(np.uint64)
    dig = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    uuid = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    img, csum = pbschunk.didx_build(ends, dig, uuid, 1700000000 + n)
    ref_img, ref_csum = oracle.didx_image(ends, dig, uuid, 1700000000 + n)
    assert img == ref_img and csum == ref_csum
    assert len(img) == 4096 + 40 * n
    u, ct, c, e, d = pbschunk.read_didx(img)
    assert u == uuid and ct == 1700000000 + n and c == csum
    assert np.array_equal(e, ends) and np.array_equal(d, dig)


def test_didx_negative_ctime_and_capacity(pbschunk, oracle):
    img, _ = pbschunk.didx_build([5], [bytes(32)], bytes(16), -1)
    assert img[24:32] == b"\xff" * 8
    assert img == oracle.didx_image([5], [bytes(32)], bytes(16), -1)[0]


def test_dynamic_index_writer_file(pbschunk, oracle, tmp_path):
    path = str(tmp_path / "test.didx")
    w = pbschunk.DynamicIndexWriter(path, uuid=bytes(range(16)), ctime=42)
    ends, digs = [], []
    for k in range(1, 6):
        d = hashlib.sha256(str(k).encode()).digest()
        w.add_chunk(k * 4096, d)
        ends.append(k * 4096)
        digs.append(np.frombuffer(d, np.uint8))
    csum = w.close()
    data = open(path, "rb").read()
    ref, ref_csum = oracle.didx_image(ends, digs, bytes(range(16)), 42)
    assert data == ref and csum == ref_csum
    assert not os.path.exists(str(tmp_path / "test.tmp_didx"))
    with pytest.raises(RuntimeError):
        w.add_chunk(1, bytes(32))
    with pytest.raises(RuntimeError):
        w.close()


def _blob_writer_vectors():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "blob_writer_digests.json")) as f:
        return json.load(f)


def test_reference_digest_vectors_pin_the_oracle(pbschunk):
    """The reference's own golden digests (tests/blob_writer.rs:11-32): hashlib (the
    oracle's SHA-256) and the library's host SHA-256 both reproduce TEST_DIGEST_PLAIN and
    TEST_DIGEST_ENC (keyed with the PBKDF2-derived id_key, crypt_config.rs:42-51)."""
    v = _blob_writer_vectors()
    data = bytes(i % 255 for i in range(100_000))
    key = hashlib.pbkdf2_hmac("sha256", bytes([1] * 32), b"_id_key", 10, 32)
    assert key.hex() == v["id_key"]
    assert hashlib.sha256(data).hexdigest() == v["digest_plain"]
    assert hashlib.sha256(data + key).hexdigest() == v["digest_enc"]
    assert pbschunk.sha256(data).hex() == v["digest_plain"]
    assert pbschunk.sha256(data + key).hex() == v["digest_enc"]


def _host_digest_cases():
    """Chunk lengths around the padding boundaries, beside a few long ones, in one buffer."""
    rng = np.random.default_rng(11)
    lens = list(range(0, 130)) + [191, 192, 193, 4095, 4096, 4097, (4 << 20) + 17, (1 << 20) * 9 - 3]
    rng.shuffle(lens)
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(bounds[-1]), dtype=np.uint8)
    return data, bounds


@pytest.mark.parametrize("klen", [0, 1, 32, 55, 56, 64])
def test_host_chunk_digests(pbschunk, oracle, klen):
    """pbs_digest_chunks_host (the hybrid digest's host share) against the oracle:
    every padding boundary, keys that push the padding into a third block, 4 threads."""
    data, bounds = _host_digest_cases()
    key = bytes((200 + j) % 256 for j in range(klen)) if klen else None
    got = pbschunk.digest_chunks_host(data, bounds, key=key, threads=4)
    assert np.array_equal(got, oracle.chunk_digests(data, bounds, key or b""))


@pytest.mark.parametrize("lanes", ["1", "2", "3", "4"])
@pytest.mark.parametrize("threads", [1, 3])
def test_host_chunk_digests_lanes(pbschunk, oracle, threads, lanes, monkeypatch):
    """The host threads hash up to four chunks in step (sha256_host_lanes; PBS_SHA_HOST_LANES
    caps it, read per call): lanes that end at different blocks, refill from the list and
    run alone in 128 KiB steps; short and long chunks interleaved, one and three threads."""
    monkeypatch.setenv("PBS_SHA_HOST_LANES", lanes)
    rng = np.random.default_rng(12)
    lens = [int(v) for v in rng.integers(0, 300_000, 40)] + [0, 1, 63, 64, 65, 2 << 20, (3 << 20) + 5]
    rng.shuffle(lens)
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = rng.integers(0, 256, int(bounds[-1]), dtype=np.uint8)
    got = pbschunk.digest_chunks_host(data, bounds, key=b"lane-key", threads=threads)
    assert np.array_equal(got, oracle.chunk_digests(data, bounds, b"lane-key"))


def test_host_chunk_digests_base_and_range(pbschunk, oracle):
    data, bounds = _host_digest_cases()
    base = 1000
    sub = data[base:]
    b = bounds[bounds >= base]
    got = pbschunk.digest_chunks_host(sub, b, base=base, threads=2)
    assert np.array_equal(got, oracle.chunk_digests(data, b))
    with pytest.raises(pbschunk.ChunkerError):
        pbschunk.digest_chunks_host(sub, np.array([base - 1, base + 5], dtype=np.uint64), base=base)


def test_host_sha_portable_block_function(tmp_path):
    """The portable FIPS 180-4 block function (used when the CPU lacks the SHA
    extensions) gives the same digests; run in a child with PBS_SHA_HOST_PORTABLE=1."""
    import subprocess
    import sys

    code = (
        "import sys, hashlib, numpy as np; sys.path[:0] = ['proxmox-backup_amd', 'tests'];"
        "import pbschunk; assert not pbschunk.sha256_host_uses_ni();"
        "rng = np.random.default_rng(3); lens = list(range(0, 140)) + [100000];"
        "b = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64);"
        "d = rng.integers(0, 256, int(b[-1]), dtype=np.uint8);"
        "g = pbschunk.digest_chunks_host(d, b, key=b'k' * 40, threads=3);"
        "mv = memoryview(d);"
        "assert all(g[i].tobytes() == hashlib.sha256(mv[int(b[i]):int(b[i+1])].tobytes() + b'k' * 40).digest()"
        " for i in range(len(lens)))"
    )
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PBS_SHA_HOST_PORTABLE="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
