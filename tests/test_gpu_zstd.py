"""GPU parity of the zstd-1 blob stage (pbs_blob_encode_chunks_device, csrc/pbs_zstd.hip):
every blob image equals the one built on the host from the twin's frame
(oracle.blob_compressed: the GPU parse step for step, oracle/zstd_twin.cpp), its CRC
equals zlib's, and every compressed payload decodes with libzstd back to the chunk.
The bytes are not libzstd level 1's (parity unpinned: DESIGN.md section 10).

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import struct
import zlib

import numpy as np
import pytest

import gen_np

pytestmark = pytest.mark.gpu
KiB, MiB = 1024, 1024 * 1024


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch

    torch.cuda.set_device(0)
    return torch


def _mixed():
    """Chunks of every block kind: empty, tiny, RLE (zero / 0xFF), compressible text,
    incompressible random, periodic runs across the 64 KiB blocks, VM-image pages,
    lengths at 64 KiB +- 1 and 3 x 64 KiB (the last block full), English-like text and
    pxar-like archives (Huffman literals; tests/corpus_gen.py), bytes above 128 (FSE-coded
    Huffman weights), two-symbol literals, and a 16 MiB chunk."""
    import corpus_gen
    rng = np.random.default_rng(17)
    text = np.frombuffer(b"proxmox backup chunk store " * 8000, dtype=np.uint8)
    parts = [np.zeros(0, np.uint8), rng.integers(0, 256, 3, dtype=np.uint8), np.zeros(64 * KiB, np.uint8),
             np.full(64 * KiB + 1, 0xFF, np.uint8), np.resize(text, 64 * KiB - 1), gen_np.gen_random(300 * KiB, 4),
             np.resize(np.arange(7, dtype=np.uint8), 400 * KiB), gen_np.gen_vmimage(4 * MiB, 0x5EED0003, 0),
             gen_np.gen_counter(MiB), np.zeros(0, np.uint8), rng.integers(0, 256, 100, dtype=np.uint8),
             corpus_gen.text(3 * 64 * KiB, 5), corpus_gen.pxar(2 * MiB + 17, 6),
             (255 - np.minimum(rng.geometric(0.08, 200 * KiB), 200)).astype(np.uint8),
             rng.choice(np.array([7, 200], np.uint8), 100 * KiB), corpus_gen.text(64 * KiB + 1, 7),
             gen_np.gen_vmimage(16 * MiB, 0x5EED0003, 1 << 30)]
    data = np.concatenate(parts)
    bounds = np.concatenate([[0], np.cumsum([p.size for p in parts])]).astype(np.uint64)
    return data, bounds


def _encode(gpu, torch, data, bounds, base=0, compress=True, pad=0):
    t = torch.empty(data.size + pad, dtype=torch.uint8, device="cuda")
    if data.size:
        t[pad:] = torch.from_numpy(data).to("cuda")
    cap = gpu.blob_stream_bound(bounds)
    out = torch.empty(max(cap, 1), dtype=torch.uint8, device="cuda")
    offs, crcs, comp, tm = gpu.blob_encode_chunks_device(t.data_ptr() + pad, data.size, bounds, out.data_ptr(), cap,
                                                         base=base, compress=compress)
    torch.cuda.synchronize()
    return out[: int(offs[-1])].cpu().numpy().tobytes(), offs, crcs, comp, tm


def _check(oracle, data, bounds, blob, offs, crcs, comp, base=0, compress=True):
    for i in range(bounds.size - 1):
        chunk = data[int(bounds[i]) - base:int(bounds[i + 1]) - base].tobytes()
        b = blob[int(offs[i]):int(offs[i + 1])]
        exp = oracle.blob_compressed(chunk) if compress else oracle.blob_uncompressed(chunk)
        assert b == exp, f"chunk {i} ({len(chunk)} bytes)"
        assert struct.unpack("<I", b[8:12])[0] == int(crcs[i]) == zlib.crc32(b[12:])
        assert bool(comp[i]) == (b[:8] == oracle.COMPRESSED_BLOB_MAGIC)
        if comp[i]:
            assert oracle.zstd_decompress(b[12:], len(chunk)) == chunk


@pytest.mark.parametrize("pad", [0, 3])
def test_blob_encode_mixed_chunks(gpu, oracle, torch_dev, pad):
    data, bounds = _mixed()
    blob, offs, crcs, comp, tm = _encode(gpu, torch_dev, data, bounds, pad=pad)
    _check(oracle, data, bounds, blob, offs, crcs, comp)
    assert comp.sum() >= 6 and tm["compressed_chunks"] == comp.sum()


@pytest.mark.parametrize("batch,deal", [("7", "1"), ("7", "0"), ("64", "1")])
def test_blob_encode_batches(gpu, oracle, torch_dev, monkeypatch, batch, deal):
    """Many parse / entropy launch pairs in one call (PBS_ZSTD_BATCH items each: the
    default 32 768 makes every other test here one batch), the items dealt by each batch's
    counters or statically, the entropy kernel over each batch's list: the twin's blobs."""
    monkeypatch.setenv("PBS_ZSTD_BATCH", batch)
    monkeypatch.setenv("PBS_ZSTD_DEAL", deal)
    data, bounds = _mixed()
    blob, offs, crcs, comp, tm = _encode(gpu, torch_dev, data, bounds, pad=1)
    _check(oracle, data, bounds, blob, offs, crcs, comp)


def test_blob_encode_uncompressed(gpu, oracle, torch_dev):
    """compress = false (DataBlob::encode(.., false), :162-173): every blob raw."""
    data, bounds = _mixed()
    blob, offs, crcs, comp, _ = _encode(gpu, torch_dev, data, bounds, compress=False)
    _check(oracle, data, bounds, blob, offs, crcs, comp, compress=False)
    assert comp.sum() == 0


def test_blob_encode_base_and_errors(gpu, oracle, torch_dev):
    data, bounds = _mixed()
    base = int(bounds[3])
    sub = data[base:]
    b = bounds[3:]
    blob, offs, crcs, comp, _ = _encode(gpu, torch_dev, sub, b, base=base)
    _check(oracle, data, b, blob, offs, crcs, comp)
    t = torch_dev.empty(sub.size, dtype=torch_dev.uint8, device="cuda")
    out = torch_dev.empty(16, dtype=torch_dev.uint8, device="cuda")
    with pytest.raises(gpu.ChunkerError):  # capacity
        gpu.blob_encode_chunks_device(t.data_ptr(), sub.size, b, out.data_ptr(), 16, base=base)
    with pytest.raises(gpu.ChunkerError):  # a chunk outside the device range
        gpu.blob_encode_chunks_device(t.data_ptr(), sub.size, np.array([base - 1, base + 9], np.uint64),
                                      out.data_ptr(), 16, base=base)


@pytest.mark.parametrize("avg", [256 * KiB, 4 * MiB])
def test_chunker_to_blobs_vm_stream(gpu, oracle, torch_dev, avg):
    """Chunker -> compressed blobs on a 192 MiB VM-image stream (zero pages as RLE blocks,
    forced 4*avg chunks of zero extents, random pages raw)."""
    n = 192 * MiB + 11
    data = gen_np.gen_vmimage(n, 0x5EED0007, 0)
    t = torch_dev.from_numpy(data).to("cuda")
    with gpu.Chunker(avg) as c:
        ends = c.find_cuts_device(t.data_ptr(), n, is_final=True)
    if ends.size == 0 or int(ends[-1]) != n:
        ends = np.append(ends, np.uint64(n))
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    blob, offs, crcs, comp, tm = _encode(gpu, torch_dev, data, bounds)
    _check(oracle, data, bounds, blob, offs, crcs, comp)
    assert tm["bytes_out"] < n  # the zero pages compress


@pytest.mark.parametrize("corpus", ["text", "pxar"])
def test_chunker_to_blobs_corpus(gpu, oracle, torch_dev, corpus):
    """Chunker -> compressed blobs on 24 MiB of English-like text / a pxar-like archive
    (tests/corpus_gen.py) at 1 MiB: Huffman literals, FSE sequence tables and repeat codes
    in every block, bit-exact with the twin, and the payloads within 10 % of libzstd
    level 1 (the reference's compressor, data_blob.rs:151)."""
    import corpus_gen
    n = 24 * MiB
    data = corpus_gen.text(n, 11) if corpus == "text" else corpus_gen.pxar(n, 12)
    n = data.size
    t = torch_dev.from_numpy(data).to("cuda")
    with gpu.Chunker(MiB) as c:
        ends = c.find_cuts_device(t.data_ptr(), n, is_final=True)
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    blob, offs, crcs, comp, tm = _encode(gpu, torch_dev, data, bounds)
    _check(oracle, data, bounds, blob, offs, crcs, comp)
    L = oracle.libzstd()
    ref = 0
    for i in range(bounds.size - 1):
        ch = np.ascontiguousarray(data[int(bounds[i]):int(bounds[i + 1])])
        dst = np.empty(L.ZSTD_compressBound(ch.size), np.uint8)
        ref += L.ZSTD_compress(dst.ctypes.data, dst.size, ch.ctypes.data, ch.size, 1)
    ours = int(offs[-1]) - 12 * (bounds.size - 1)
    assert ours <= ref * 1.10, (ours, ref)


def test_blob_encode_after_release(gpu, oracle, torch_dev):
    """pbs_blob_encode_release frees the cached scratch; the next call allocates it anew
    and writes the same blobs."""
    data, bounds = _mixed()
    a = _encode(gpu, torch_dev, data, bounds)[0]
    gpu.blob_encode_release()
    b = _encode(gpu, torch_dev, data, bounds)[0]
    assert a == b
