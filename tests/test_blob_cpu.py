"""Blob CRC stage on CPU: the oracle pinned by the CRC-32
check value, the library's host CRC and the uncompressed DataBlob layout against it,
and the C ABI exports (compute calls need a GPU: tests/test_gpu_blob.py)."""
import zlib

import numpy as np
import pytest

import gen_np


def test_oracle_crc_check_value(oracle):
    # CRC-32/ISO-HDLC check value (the catalogue entry crc32fast implements)
    assert oracle.chunk_crcs(np.frombuffer(b"123456789", dtype=np.uint8), [0, 9]).tolist() == [0xCBF43926]
    assert oracle.chunk_crcs(np.zeros(0, dtype=np.uint8), [0, 0]).tolist() == [0]


def test_host_crc_matches_oracle(pbschunk, oracle):
    data = gen_np.gen_random(100_003, 9)
    assert pbschunk.crc32(b"123456789") == 0xCBF43926
    bounds = [0, 0, 1, 3, 4, 5, 64, 4096, 4100, 50_000, 100_003]
    ref = oracle.chunk_crcs(data, bounds)
    got = [pbschunk.crc32(data[a:b]) for a, b in zip(bounds, bounds[1:])]
    assert got == ref.tolist()
    # Hasher::update continuation
    assert pbschunk.crc32(data[777:], pbschunk.crc32(data[:777])) == zlib.crc32(data.tobytes())


@pytest.mark.parametrize("n", [0, 1, 4095, 65536])
def test_blob_encode_uncompressed_layout(pbschunk, oracle, n):
    data = gen_np.gen_random(n, 3).tobytes()
    blob = pbschunk.blob_encode_uncompressed(data, zlib.crc32(data))
    assert blob == oracle.blob_uncompressed(data)
    assert blob[:8] == pbschunk.UNCOMPRESSED_BLOB_MAGIC_1_0


def test_blob_too_large(pbschunk):
    with pytest.raises(ValueError, match="too large"):
        pbschunk.blob_encode_uncompressed(np.zeros(128 * 1024 * 1024 + 1, dtype=np.uint8), 0)


def test_crc_device_entry_rejects_bad_bounds(pbschunk):
    if pbschunk.device_count() > 0:
        pytest.skip("device visible")
    with pytest.raises(pbschunk.ChunkerError):
        pbschunk.crc32_chunks_device(0x1000, 100, np.array([50, 10], dtype=np.uint64))


def _crc_row_model(buf: bytes, s: int, e: int, lanes: int = 8) -> int:
    """Pure-Python model of crc32_chunks_kernel's decomposition (csrc/pbs_blob.hip) at a
    small scale: rows of lanes*16 bytes at absolute offsets, lane t owns the 16-byte word
    at 16 t of each row, word-to-word step F(r ^ w) = absorb 16 bytes then row-16 zero
    bytes, last word bytewise, then x^(8 (end - c)) and the XOR over lanes; the init
    value as 0xFF XOR-ed into the first four bytes."""
    poly = 0xEDB88320
    T = []
    for v in range(256):
        c = v
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        T.append(c)

    def raw(r, data):
        for b in data:
            r = (r >> 8) ^ T[(r ^ b) & 0xFF]
        return r

    def multmodp(a, b):
        p = 0
        for k in range(31, -1, -1):
            if (a >> k) & 1:
                p ^= b
            b = (b >> 1) ^ poly if b & 1 else b >> 1
        return p

    def x8(d):
        p = 1 << 31
        for _ in range(8 * d):
            p = (p >> 1) ^ poly if p & 1 else p >> 1
        return p

    row = lanes * 16
    xs = [x8(row - 1 - i) for i in range(16)]
    tf = [[multmodp(xs[i], T[v]) for v in range(256)] for i in range(16)]
    if e - s < 4:
        return raw(0xFFFFFFFF, buf[s:e]) ^ 0xFFFFFFFF
    mb = bytearray(buf)
    for k in range(4):
        mb[s + k] ^= 0xFF
    r0 = (s // row) * row
    tot = 0
    for t in range(lanes):
        words = []
        w = r0 + 16 * t
        while w < e:
            if w + 16 > s:
                words.append(w)
            w += row
        r, c = 0, None
        for j, w in enumerate(words):
            wd = bytes(mb[p] if s <= p < e else 0 for p in range(w, w + 16))
            if j + 1 < len(words):
                x = bytearray(wd)
                for k in range(4):
                    x[k] ^= (r >> (8 * k)) & 0xFF
                r = 0
                for i in range(16):
                    r ^= tf[i][x[i]]
            else:
                c = min(w + 16, e)
                r = raw(r, wd[:c - w])
        if c is not None and r:
            tot ^= multmodp(x8(e - c), r)
    return tot ^ 0xFFFFFFFF


def test_crc_row_decomposition_model():
    """The linear algebra the GPU kernel relies on, checked against zlib's CRC-32 on
    starts/ends at every alignment of the lane word and the row."""
    import random

    rng = random.Random(7)
    buf = bytes(rng.getrandbits(8) for _ in range(700))
    cases = [(0, 700), (5, 6), (5, 9), (0, 4), (17, 160), (100, 699), (128, 256), (127, 257), (33, 49)]
    cases += [tuple(sorted(rng.sample(range(701), 2))) for _ in range(40)]
    for s, e in cases:
        assert _crc_row_model(buf, s, e) == zlib.crc32(buf[s:e]), (s, e)
