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
