"""GPU parity of the blob CRC: DataBlob::compute_crc
(data_blob.rs:70-75, crc32fast = CRC-32/ISO-HDLC) of every chunk on the device against
the oracle (zlib.crc32), bit-exact: lengths around the 4-byte init register, the 16-byte
lane word and the 4096-byte row; every start alignment mod 16 and several mod 4096;
chunks of 16 MiB + odd; the chunker's own cut lists end to end; the blob image.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import numpy as np
import pytest

import gen_np

pytestmark = pytest.mark.gpu
KiB, MiB = 1024, 1024 * 1024


def _dev(torch, host: np.ndarray, pad_front: int = 0):
    t = torch.empty(host.size + pad_front, dtype=torch.uint8, device="cuda")
    if host.size:
        t[pad_front:] = torch.from_numpy(host).to("cuda")
    return t, t.data_ptr() + pad_front


@pytest.fixture(scope="module")
def torch_dev(gpu):
    import torch

    torch.cuda.set_device(0)
    return torch


def test_edge_lengths_and_alignment(gpu, oracle, torch_dev):
    lens = [0, 1, 2, 3, 4, 5, 6, 7, 8, 15, 16, 17, 19, 20, 31, 32, 33, 63, 64, 255, 256, 1000,
            4079, 4080, 4081, 4095, 4096, 4097, 4111, 4112, 4113, 8191, 8192, 8193, 12288 + 5,
            65536 + 7]
    rng = np.random.default_rng(3)
    for pad in (0, 1, 2, 3, 4, 5, 7, 8, 13, 15, 16, 4095 - 16, 4093, 2048 + 9):
        order = rng.permutation(len(lens))
        bounds = np.concatenate([[0], np.cumsum([lens[i] for i in order])]).astype(np.uint64)
        data = gen_np.gen_random(int(bounds[-1]), 0xC2C + pad)
        t, ptr = _dev(torch_dev, data, pad)
        got = gpu.crc32_chunks_device(ptr, data.size, bounds)
        assert np.array_equal(got, oracle.chunk_crcs(data, bounds)), f"pad {pad}"
        del t


def test_every_length_small(gpu, oracle, torch_dev):
    """Every length 0..600 back to back (every start mod 16 and lane position)."""
    lens = np.arange(601)
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = gen_np.gen_random(int(bounds[-1]), 41)
    t, ptr = _dev(torch_dev, data, 3)
    assert np.array_equal(gpu.crc32_chunks_device(ptr, data.size, bounds), oracle.chunk_crcs(data, bounds))


@pytest.mark.parametrize("kind", ["random", "zeros", "ones"])
def test_large_chunks(gpu, oracle, torch_dev, kind):
    """Max-size chunks (16 MiB at the 4 MiB average) and odd large sizes; constant data
    (all 0x00 / 0xFF) is where a wrong init or zero-row handling would show."""
    lens = [16 * MiB, 16 * MiB + 1, 5 * MiB + 4093, 1 * MiB - 3, 3]
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(7)
    n = int(bounds[-1]) + 9
    data = {"random": lambda: gen_np.gen_random(n, 5),
            "zeros": lambda: np.zeros(n, dtype=np.uint8),
            "ones": lambda: np.full(n, 0xFF, dtype=np.uint8)}[kind]()
    t, ptr = _dev(torch_dev, data, 1)
    assert np.array_equal(gpu.crc32_chunks_device(ptr, data.size, bounds), oracle.chunk_crcs(data, bounds))


def test_base_offset_and_bad_range(gpu, oracle, torch_dev):
    data = gen_np.gen_random(2 * MiB + 11, 6)
    base = 7 * MiB + 5
    t, ptr = _dev(torch_dev, data)
    rel = np.array([3, 100, 5000, 1 * MiB + 1, 2 * MiB + 11], dtype=np.uint64)
    got = gpu.crc32_chunks_device(ptr, data.size, rel + np.uint64(base), base=base)
    assert np.array_equal(got, oracle.chunk_crcs(data, rel))
    with pytest.raises(gpu.ChunkerError):
        gpu.crc32_chunks_device(ptr, data.size, rel + np.uint64(base + 1), base=base)


@pytest.mark.parametrize("kind,avg", [("vmimage", 64 * KiB), ("random", 4 * MiB), ("vmimage", 4 * MiB)])
def test_chunker_to_blob_end_to_end(gpu, oracle, torch_dev, kind, avg):
    """GPU cut list -> GPU CRC per chunk -> uncompressed blobs, against the oracle
    chunker + zlib + the blob layout."""
    n = 40 * MiB + 123
    data = gen_np.gen_vmimage(n, 11, 0) if kind == "vmimage" else gen_np.gen_random(n, 12)
    t, ptr = _dev(torch_dev, data)
    c = gpu.Chunker(avg)
    ends = c.find_cuts_device(ptr, n, is_final=True)
    ref_ends = oracle.chunk_feed(avg, data)
    assert np.array_equal(ends[:-1], ref_ends) and int(ends[-1]) == n
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    crcs = gpu.crc32_chunks_device(ptr, n, bounds)
    assert np.array_equal(crcs, oracle.chunk_crcs(data, bounds))
    for i in (0, len(ends) // 2, len(ends) - 1):
        chunk = data[int(bounds[i]):int(bounds[i + 1])].tobytes()
        assert gpu.blob_encode_uncompressed(chunk, int(crcs[i])) == oracle.blob_uncompressed(chunk)


def test_async_form_and_order(gpu, oracle, torch_dev):
    """Device-only form with an explicit (reversed) order and many tiny chunks."""
    torch = torch_dev
    rng = np.random.default_rng(8)
    lens = rng.integers(0, 3000, size=5000)
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = gen_np.gen_random(int(bounds[-1]), 13)
    t, ptr = _dev(torch, data, 2)
    b_dev = torch.from_numpy(bounds.view(np.int64)).to("cuda")
    o_dev = torch.from_numpy(np.arange(lens.size, dtype=np.int32)[::-1].copy()).to("cuda")
    out = torch.zeros(lens.size, dtype=torch.int32, device="cuda")
    gpu.crc32_chunks_async(ptr, data.size, b_dev.data_ptr(), o_dev.data_ptr(), lens.size, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, oracle.chunk_crcs(data, bounds))


def test_back_to_back_launches_one_stream(gpu, oracle, torch_dev):
    """The dynamic chunk order's counters reset themselves at the end of each launch:
    three launches of different sizes queued back to back on one stream (and one on a
    second stream), one sync, all results exact."""
    torch = torch_dev
    rng = np.random.default_rng(9)
    data = gen_np.gen_random(96 * MiB, 17)
    t, ptr = _dev(torch, data)
    s2 = torch.cuda.Stream()
    runs = []
    for k, (nchunks, stream) in enumerate([(5000, 0), (20000, 0), (300, 0), (7000, s2.cuda_stream)]):
        lens = rng.integers(1, 4000, size=nchunks)
        bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64) + np.uint64(k * 1000)
        assert int(bounds[-1]) <= data.size
        b_dev = torch.from_numpy(bounds.view(np.int64)).to("cuda")
        out = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
        runs.append((bounds, b_dev, out, stream, nchunks))
    torch.cuda.synchronize()  # inputs in place; then the four launches without a sync between
    for bounds, b_dev, out, stream, nchunks in runs:
        gpu.crc32_chunks_async(ptr, data.size, b_dev.data_ptr(), 0, nchunks, out.data_ptr(), hip_stream=stream)
    torch.cuda.synchronize()
    for bounds, _, out, _, _ in runs:
        assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle.chunk_crcs(data, bounds))
