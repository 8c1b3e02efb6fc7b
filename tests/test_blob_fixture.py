"""The reference's own pin for compressed blobs, on the GPU path.

The reference never compares compressed bytes.  tests/blob_writer.rs:35-87 writes
TEST_DATA (100 000 bytes, byte i = i % 255) into a blob -- compressed and uncompressed --
and `verify_test_blob` checks that the blob loads (magic, DataBlob::verify_crc), reads back
through DataBlobReader with 1-, 3- and 64 KiB buffers, and decodes
(DataBlob::decode -> zstd::stream::decode_all, data_blob.rs:196-216) to TEST_DATA with
SHA-256 TEST_DIGEST_PLAIN (tests/golden/blob_writer_digests.json).  Here the same check
(oracle.blob_load_decode, a restatement of those functions) runs on blobs the GPU wrote:
pbs_blob_encode_chunks_device / _spans_device with compress = 1 and 0, TEST_DATA alone and
as one chunk among others at several start alignments, and pbs_upload_stream_host.

Byte equality with libzstd 1.5 level 1 is NOT a reference contract (the reference only
decodes its frames) and is not asserted here.

CPU tests pin the verifier itself (libzstd's own blob passes, corrupted blobs fail);
`-m gpu` tests run it on the GPU encoder's output.
"""
import hashlib
import json
import os
import struct
import zlib

import numpy as np
import pytest

import gen_np

KiB, MiB = 1024, 1024 * 1024
TEST_DATA = (np.arange(100_000) % 255).astype(np.uint8)  # tests/blob_writer.rs:11-19


def _digest_plain() -> bytes:
    with open(os.path.join(os.path.dirname(__file__), "golden", "blob_writer_digests.json")) as f:
        return bytes.fromhex(json.load(f)["digest_plain"])


# ---- CPU: the verifier against blobs of known provenance ---------------------------

def _libzstd_blob(oracle, data: bytes) -> bytes:
    L = oracle.libzstd()
    src = np.frombuffer(data, np.uint8)
    dst = np.empty(L.ZSTD_compressBound(src.size), np.uint8)
    n = L.ZSTD_compress(dst.ctypes.data, dst.size, src.ctypes.data, src.size, 1)
    frame = dst[:n].tobytes()
    return oracle.COMPRESSED_BLOB_MAGIC + struct.pack("<I", zlib.crc32(frame)) + frame


def test_verifier_accepts_reference_shaped_blobs(oracle):
    """What DataBlobWriter::new_compressed / new_uncompressed write for TEST_DATA (a
    libzstd level-1 frame behind the header; the raw bytes) passes, and the digest is the
    reference's TEST_DIGEST_PLAIN."""
    td = TEST_DATA.tobytes()
    dig = _digest_plain()
    assert hashlib.sha256(td).digest() == dig
    assert oracle.blob_load_decode(_libzstd_blob(oracle, td), dig) == td
    assert oracle.blob_load_decode(oracle.blob_uncompressed(td), dig) == td
    assert oracle.blob_load_decode(oracle.blob_compressed(td), dig) == td  # the twin's frame


@pytest.mark.parametrize("fault", ["crc", "payload", "magic", "short", "truncated", "digest"])
def test_verifier_rejects(oracle, fault):
    td = TEST_DATA.tobytes()
    blob = bytearray(_libzstd_blob(oracle, td))
    dig = _digest_plain()
    if fault == "crc":
        blob[9] ^= 1
    elif fault == "payload":
        blob[40] ^= 0x10
    elif fault == "magic":
        blob[0] ^= 1
    elif fault == "short":
        blob = blob[:11]
    elif fault == "truncated":  # CRC recomputed so only the frame is at fault
        blob = blob[:-5]
        blob[8:12] = struct.pack("<I", zlib.crc32(bytes(blob[12:])))
    elif fault == "digest":
        dig = bytes(32)
    with pytest.raises(ValueError):
        oracle.blob_load_decode(bytes(blob), dig)


# ---- GPU: the encoder's blobs through the same check ------------------------------

@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch

    torch.cuda.set_device(0)
    return torch


def _to_dev(torch, host: np.ndarray, pad: int):
    t = torch.empty(host.size + pad, dtype=torch.uint8, device="cuda")
    t[pad:] = torch.from_numpy(host).to("cuda")
    return t, t.data_ptr() + pad


def _blobs(torch, out, offs):
    torch.cuda.synchronize()
    raw = out[: int(offs[-1])].cpu().numpy().tobytes()
    return [raw[int(offs[i]):int(offs[i + 1])] for i in range(offs.size - 1)]


def _check_blob(oracle, blob: bytes, chunk: bytes, crc: int, comp: int, compress: bool, digest: bytes):
    assert oracle.blob_load_decode(blob, digest) == chunk
    assert struct.unpack("<I", blob[8:12])[0] == int(crc)
    assert bool(comp) == (blob[:8] == oracle.COMPRESSED_BLOB_MAGIC)
    if not compress:
        assert blob[:8] == oracle.UNCOMPRESSED_BLOB_MAGIC


@pytest.mark.gpu
@pytest.mark.parametrize("compress", [True, False])
@pytest.mark.parametrize("pad", [0, 1, 3, 8, 15, 4093])
def test_gpu_blob_of_test_data(gpu, oracle, torch_dev, compress, pad):
    """test_compressed_blob_writer / test_uncompressed_blob_writer on the GPU encoder:
    TEST_DATA as one chunk at device start alignment `pad`."""
    torch = torch_dev
    t, ptr = _to_dev(torch, TEST_DATA, pad)
    bounds = np.array([0, TEST_DATA.size], np.uint64)
    cap = gpu.blob_stream_bound(bounds)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs, crcs, comp, _ = gpu.blob_encode_chunks_device(ptr, TEST_DATA.size, bounds, out.data_ptr(), cap,
                                                         compress=compress)
    blob = _blobs(torch, out, offs)[0]
    _check_blob(oracle, blob, TEST_DATA.tobytes(), crcs[0], comp[0], compress, _digest_plain())
    if compress:  # period-255 data: the frame is far shorter than the chunk
        assert comp[0] == 1 and len(blob) < 2000


def _stream():
    """TEST_DATA twice among other chunks: random, zeros, text, and the copies at start
    offsets 777 and 777 + 100000 + 4105 + 65536 + 3 (odd, not 16-aligned)."""
    import corpus_gen
    parts = [gen_np.gen_random(777, 5), TEST_DATA, gen_np.gen_random(4096 + 9, 6), np.zeros(64 * KiB, np.uint8),
             corpus_gen.text(3, 2), TEST_DATA, corpus_gen.text(200 * KiB + 1, 4), np.zeros(0, np.uint8)]
    data = np.concatenate(parts)
    bounds = np.concatenate([[0], np.cumsum([p.size for p in parts])]).astype(np.uint64)
    return data, bounds, (1, 5)


@pytest.mark.gpu
@pytest.mark.parametrize("compress", [True, False])
@pytest.mark.parametrize("pad", [0, 2, 7])
def test_gpu_blob_of_test_data_in_stream(gpu, oracle, torch_dev, compress, pad):
    """TEST_DATA as chunks 1 and 5 of a stream at absolute offsets above 2^33 (base):
    each of its blobs passes verify_test_blob with TEST_DIGEST_PLAIN; every other blob
    loads and decodes to its chunk, whose digest it is checked against."""
    torch = torch_dev
    data, bounds, fixture_idx = _stream()
    base = (1 << 33) + 5
    t, ptr = _to_dev(torch, data, pad)
    b = bounds + np.uint64(base)
    cap = gpu.blob_stream_bound(b)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs, crcs, comp, _ = gpu.blob_encode_chunks_device(ptr, data.size, b, out.data_ptr(), cap, base=base,
                                                         compress=compress)
    blobs = _blobs(torch, out, offs)
    for i, blob in enumerate(blobs):
        chunk = data[int(bounds[i]):int(bounds[i + 1])].tobytes()
        want = _digest_plain() if i in fixture_idx else hashlib.sha256(chunk).digest()
        _check_blob(oracle, blob, chunk, crcs[i], comp[i], compress, want)
    assert all(comp[i] == int(compress) for i in fixture_idx)


@pytest.mark.gpu
def test_gpu_blob_spans_of_test_data(gpu, oracle, torch_dev):
    """pbs_blob_encode_spans_device (the upload's new-chunk form): the stream's chunks as
    spans in reverse order with gaps; blob k is span k's."""
    torch = torch_dev
    data, bounds, fixture_idx = _stream()
    t, ptr = _to_dev(torch, data, 1)
    pick = [5, 3, 1, 0]
    spans = np.array([[bounds[i], bounds[i + 1]] for i in pick], np.uint64)
    cap = 12 * len(pick) + int(sum(int(e - s) for s, e in spans))
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs, crcs, comp, _ = gpu.blob_encode_spans_device(ptr, data.size, spans, out.data_ptr(), cap)
    blobs = _blobs(torch, out, offs)
    for k, i in enumerate(pick):
        chunk = data[int(bounds[i]):int(bounds[i + 1])].tobytes()
        want = _digest_plain() if i in fixture_idx else hashlib.sha256(chunk).digest()
        _check_blob(oracle, blobs[k], chunk, crcs[k], comp[k], True, want)


@pytest.mark.gpu
@pytest.mark.parametrize("compress", [True, False])
def test_gpu_upload_of_test_data(gpu, oracle, compress):
    """pbs_upload_stream_host over TEST_DATA as a whole stream (at the 4 MiB average it is
    one final chunk): the upload's digest is TEST_DIGEST_PLAIN and its blob passes
    verify_test_blob."""
    out = gpu.upload_stream_host(TEST_DATA, 4 * MiB, compress=compress)
    assert out["ends"].tolist() == [TEST_DATA.size]
    assert bytes(out["digests"][0]) == _digest_plain()
    assert out["new_chunks"] == [(0, TEST_DATA.size)]
    blob = out["blobs"][int(out["blob_offsets"][0]):int(out["blob_offsets"][1])].tobytes()
    assert oracle.blob_load_decode(blob, _digest_plain()) == TEST_DATA.tobytes()
    assert bool(out["compressed"][0]) == compress
    assert out["stats"]["size_compressed"] == len(blob)


@pytest.mark.gpu
@pytest.mark.parametrize("avg", [64 * KiB, 256 * KiB])
def test_gpu_upload_of_repeated_test_data(gpu, oracle, avg):
    """An upload stream of TEST_DATA repeated 40 times behind a random head: whatever the
    chunker cuts, every new chunk's blob loads, decodes to its bytes and matches the
    upload's own digest for it (verify_digest); repeats are known chunks with no blob."""
    head = gen_np.gen_random(12345, 9)
    data = np.concatenate([head] + [TEST_DATA] * 40)
    out = gpu.upload_stream_host(data, avg, piece=1 * MiB + 7)
    ref_ends = oracle.chunk_feed(avg, data)
    if ref_ends.size == 0 or int(ref_ends[-1]) != data.size:
        ref_ends = np.append(ref_ends, np.uint64(data.size))
    assert np.array_equal(out["ends"], ref_ends)
    bounds = np.concatenate([[0], ref_ends]).astype(np.uint64)
    offs = out["blob_offsets"]
    for i in range(ref_ends.size):
        chunk = data[int(bounds[i]):int(bounds[i + 1])].tobytes()
        assert bytes(out["digests"][i]) == hashlib.sha256(chunk).digest()
        blob = out["blobs"][int(offs[i]):int(offs[i + 1])].tobytes()
        if out["known"][i]:
            assert blob == b""
        else:
            assert oracle.blob_load_decode(blob, bytes(out["digests"][i]), read_sizes=(64 * KiB,)) == chunk
