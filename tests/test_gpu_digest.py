"""GPU parity of the 8(f) stages: per-chunk SHA-256 on the device (one lane per chunk)
against the oracle (hashlib, the FIPS 180-4 function the reference calls through
openssl, data_blob.rs:516-536; keyed form crypt_config.rs:79-84), and the end-to-end
device path chunk -> digest -> .didx against the oracle chunker + hashlib + the
oracle's dynamic_index.rs restatement.  Bit-exact.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import numpy as np
import pytest

import gen_np

pytestmark = pytest.mark.gpu
KiB, MiB = 1024, 1024 * 1024


def _dev(torch, host: np.ndarray, pad_front: int = 0):
    """Device copy of `host` starting `pad_front` bytes into a fresh allocation (so the
    stream start can be misaligned); returns (tensor, device pointer of byte 0)."""
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
    """Chunk lengths around every padding boundary (55/56/63/64/119/120/...), each
    start alignment 0..3, the last chunk ending exactly at the buffer end."""
    lens = [0, 1, 2, 3, 4, 5, 31, 32, 54, 55, 56, 57, 63, 64, 65, 118, 119, 120, 121, 127,
            128, 129, 191, 192, 193, 1000, 4095, 4096, 4097, 65536 + 7]
    rng = np.random.default_rng(1)
    for pad in range(4):
        order = rng.permutation(len(lens))
        bounds = np.concatenate([[0], np.cumsum([lens[i] for i in order])]).astype(np.uint64)
        data = gen_np.gen_random(int(bounds[-1]), 0xD16E57 + pad)
        t, ptr = _dev(torch_dev, data, pad)
        got = gpu.digest_chunks_device(ptr, data.size, bounds)
        ref = oracle.chunk_digests(data, bounds)
        assert np.array_equal(got, ref), f"pad {pad}"
        del t


@pytest.mark.parametrize("klen", [1, 5, 32, 55, 56, 64])
def test_keyed_digest(gpu, oracle, torch_dev, klen):
    """SHA-256(chunk || id_key) (crypt_config.rs:79-84) for key lengths that move the
    padding across block boundaries."""
    key = bytes(range(100, 100 + klen))
    lens = [0, 1, 7, 8, 9, 55, 56, 63, 64, 100, 4096 + 3]
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = gen_np.gen_random(int(bounds[-1]), 77 + klen)
    t, ptr = _dev(torch_dev, data, 1)
    got = gpu.digest_chunks_device(ptr, data.size, bounds, key=key)
    assert np.array_equal(got, oracle.chunk_digests(data, bounds, key))


def test_base_offset_and_subrange(gpu, oracle, torch_dev):
    """Device buffer holding stream bytes [base, base + len): chunks addressed by
    absolute offsets; only a sub-range of the buffer is chunked."""
    data = gen_np.gen_random(3 * MiB + 11, 5)
    base = 10 * MiB + 3
    t, ptr = _dev(torch_dev, data)
    rel = np.array([17, 100, 5000, 1 * MiB + 1, 2 * MiB + 999, 3 * MiB + 11], dtype=np.uint64)
    got = gpu.digest_chunks_device(ptr, data.size, rel + np.uint64(base), base=base)
    assert np.array_equal(got, oracle.chunk_digests(data, rel))
    with pytest.raises(gpu.ChunkerError):  # a chunk outside the device range
        gpu.digest_chunks_device(ptr, data.size, rel + np.uint64(base - 1000), base=base)


@pytest.mark.parametrize("kind,avg", [("vmimage", 64 * KiB), ("random", 4 * MiB), ("zeros", 256 * KiB)])
def test_chunker_to_didx_end_to_end(gpu, oracle, torch_dev, kind, avg):
    """The client path on a device-resident stream: GPU cut list, GPU digests, .didx
    image and index_csum -- all equal to the oracle chunker + hashlib + the oracle's
    restatement of DynamicIndexWriter (incl. the forced 4*avg cuts of zero runs)."""
    n = 24 * MiB + 333
    if kind == "vmimage":
        data = gen_np.gen_vmimage(n, 0x5EED0003, 0)
    elif kind == "random":
        data = gen_np.gen_random(n, 0x5EED0002)
    else:
        data = np.zeros(n, dtype=np.uint8)
    t, ptr = _dev(torch_dev, data)
    uuid = bytes(range(16))
    with gpu.Chunker(avg) as c:
        ends, dig, csum, image = gpu.index_stream_device(c, ptr, n, uuid=uuid, ctime=123)
    ref_ends = oracle.chunk_feed(avg, data)
    if ref_ends.size == 0 or int(ref_ends[-1]) != n:
        ref_ends = np.append(ref_ends, np.uint64(n))
    assert np.array_equal(ends, ref_ends)
    bounds = np.concatenate([[0], ref_ends]).astype(np.uint64)
    ref_dig = oracle.chunk_digests(data, bounds)
    assert np.array_equal(dig, ref_dig)
    ref_img, ref_csum = oracle.didx_image(ref_ends, ref_dig, uuid, 123)
    assert csum == ref_csum and image == ref_img


def test_large_chunks_sorted_lanes(gpu, oracle, torch_dev):
    """Max-size (16 MiB) chunks beside tiny ones in one launch (the host orders lanes by
    length), 64+ chunks so several waves run."""
    rng = np.random.default_rng(3)
    lens = [16 * MiB, 16 * MiB - 1, 1, 64, 9 * MiB + 5] + [int(x) for x in rng.integers(1, 300 * KiB, 90)]
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = gen_np.gen_vmimage(int(bounds[-1]), 11, 0)
    t, ptr = _dev(torch_dev, data, 2)
    got = gpu.digest_chunks_device(ptr, data.size, bounds)
    assert np.array_equal(got, oracle.chunk_digests(data, bounds))


def test_async_device_form(gpu, oracle, torch_dev):
    """pbs_digest_chunks_async with device bounds/order/digests (the bench's form)."""
    torch = torch_dev
    lens = np.random.default_rng(9).integers(1, 100 * KiB, 40)
    bounds = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = gen_np.gen_random(int(bounds[-1]), 9)
    t, ptr = _dev(torch, data, 3)
    n = bounds.size - 1
    bd = torch.from_numpy(bounds.view(np.int64)).to("cuda")
    order = torch.from_numpy(np.argsort(-(np.diff(bounds.astype(np.int64))), kind="stable").astype(np.int32)).to("cuda")
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    gpu.digest_chunks_async(ptr, data.size, bd.data_ptr(), order.data_ptr(), n, out.data_ptr(), hip_stream=s)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(n, 32)
    assert np.array_equal(got, oracle.chunk_digests(data, bounds))


def _known_case(rng, n, k, prefix_clash=False):
    dig = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    # repeats inside the stream (runs and scattered), like the zero chunks of an image
    for _ in range(n // 5):
        a, b = rng.integers(0, n, 2)
        dig[max(a, b)] = dig[min(a, b)]
    dig[n // 2: n // 2 + 40] = dig[n // 2]
    if prefix_clash:  # same first 8 bytes, different digests (forces the slow path)
        dig[10:30, :8] = dig[3, :8]
        dig[25] = dig[12]
    prev = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    if k:
        prev[: k // 3] = dig[rng.integers(0, n, k // 3)]
    known = np.unique(prev.view("S32").reshape(-1)).view(np.uint8).reshape(-1, 32) if k else prev
    return dig, known


@pytest.mark.parametrize("n,k,clash", [(1, 0, False), (500, 0, False), (5000, 300, False),
                                       (3000, 1000, True), (20000, 5000, True)])
def test_known_chunks(gpu, oracle, torch_dev, n, k, clash):
    """Known-chunk flags (previous index + repeats within the stream) equal the
    reference's HashSet walk."""
    torch = torch_dev
    rng = np.random.default_rng(n + k)
    dig, known = _known_case(rng, n, k, clash)
    d = torch.from_numpy(dig.reshape(-1)).to("cuda")
    kn = torch.from_numpy(known.reshape(-1).copy()).to("cuda") if k else None
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    cnt = gpu.known_chunks_device(d.data_ptr(), n, kn.data_ptr() if k else 0, known.shape[0] if k else 0,
                                  out.data_ptr(), hip_stream=torch.cuda.current_stream().cuda_stream)
    ref = oracle.known_chunks(dig, known if k else [])
    got = out.cpu().numpy()
    assert np.array_equal(got, ref) and cnt == int(ref.sum())


@pytest.mark.parametrize("kind,avg,piece,key,host_min", [
    ("vmimage", 1 << 20, 8 << 20, None, None),          # chunks shorter than a piece (deadline routing)
    ("vmimage", 1 << 20, 8 << 20, None, "slack"),       # deadline far away: every digest on the GPU queue
    ("vmimage", 4 << 20, 5 << 20 | 3, b"k" * 32, None),  # 16 MiB chunks spanning pieces, keyed
    ("random", 64 << 10, 1 << 20, None, None),           # many chunks per piece
    ("vmimage", 4 << 20, 8 << 20, b"k" * 32, "0"),       # GPU digests only
    ("vmimage", 1 << 20, 4 << 20, None, "1"),            # host digests only (GPU: the CRCs)
    ("vmimage", 256 << 10, 3 << 20, b"k" * 5, "262144"),  # split at the average
])
def test_pipeline_host(gpu, oracle, monkeypatch, kind, avg, piece, key, host_min):
    """Overlapped copy -> chunk -> digest over a pageable host buffer (pbs_pipeline_host)
    equals the oracle chunker + hashlib, with chunks straddling the copy pieces, and the
    digests split between the GPU's digest queue and the host threads (by the copy-end
    deadline, or PBS_PIPE_HOST_MIN) or all on one side; all-zero chunks hashed once per
    length on the host."""
    if host_min == "slack":
        monkeypatch.setenv("PBS_PIPE_SLACK_MS", "100000")
    elif host_min is not None:
        monkeypatch.setenv("PBS_PIPE_HOST_MIN", host_min)
    n = 100 * MiB + 77
    data = gen_np.gen_vmimage(n, 0x5EED0003, 0) if kind == "vmimage" else gen_np.gen_random(n, 21)
    ends, dig, crcs, t = gpu.pipeline_host(data, avg, piece=piece, key=key, digest_cus=32, crc=True)
    ref = oracle.chunk_feed(avg, data)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert np.array_equal(ends, ref)
    bounds = np.concatenate([[0], ref]).astype(np.uint64)
    assert np.array_equal(dig, oracle.chunk_digests(data, bounds, key or b""))
    assert np.array_equal(crcs, oracle.chunk_crcs(data, bounds))  # the blob CRCs
    assert t["chunks"] == ref.size and t["bytes"] == n
    if host_min in ("0", "slack"):
        assert t["host_chunks"] == 0
    elif host_min == "1":
        assert t["host_chunks"] == ref.size
    # without the CRC output: same cut list and digests, from the same device work area
    a0 = gpu.debug_arena_allocs()
    ends2, dig2, _ = gpu.pipeline_host(data, avg, piece=piece, key=key, digest_cus=32)
    assert np.array_equal(ends2, ends) and np.array_equal(dig2, dig)
    assert gpu.debug_arena_allocs() == a0


def test_pipeline_release(gpu, oracle):
    """pbs_pipeline_release frees the idle work area; the next call allocates a new one
    and gives the same result."""
    n = 20 * MiB + 3
    data = gen_np.gen_vmimage(n, 0x5EED0003, 0)
    ends, dig, _ = gpu.pipeline_host(data, 1 << 20, piece=4 << 20)
    gpu.pipeline_release()
    a0 = gpu.debug_arena_allocs()
    ends2, dig2, _ = gpu.pipeline_host(data, 1 << 20, piece=4 << 20)
    assert gpu.debug_arena_allocs() > a0
    assert np.array_equal(ends2, ends) and np.array_equal(dig2, dig)
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    assert np.array_equal(dig, oracle.chunk_digests(data, bounds))


def test_pipeline_area_changes(gpu, oracle):
    """The kept work area across calls that change what it holds: another average (a new
    chunker handle), another CU split (new streams), a longer stream (larger buffers), a
    failed call (invalid average: the call raises, the next one is unaffected)."""
    n = 24 * MiB + 11
    data = gen_np.gen_vmimage(2 * n, 0x5EED0003, 0)
    for avg, cus, ln in [(1 << 20, 32, n), (256 << 10, 32, n), (256 << 10, 16, n), (1 << 20, 16, 2 * n)]:
        ends, dig, t = gpu.pipeline_host(data[:ln], avg, piece=5 << 20, digest_cus=cus)
        ref = oracle.chunk_feed(avg, data[:ln])
        if ref.size == 0 or int(ref[-1]) != ln:
            ref = np.append(ref, np.uint64(ln))
        assert np.array_equal(ends, ref), (avg, cus, ln)
        assert np.array_equal(dig, oracle.chunk_digests(data[:ln], np.concatenate([[0], ref]).astype(np.uint64)))
        if avg == 1 << 20 and cus == 32:
            with pytest.raises(gpu.ChunkerError):
                gpu.pipeline_host(data[:ln], 3 << 19, piece=5 << 20)


def test_pipeline_queue_idle_exit(gpu, oracle, monkeypatch):
    """The digest queue grid's idle exit (PBS_PIPE_IDLE_MS=0: a workgroup leaves as soon as
    one poll finds no new job), its relaunch when the next piece publishes jobs, and the
    end-of-call host hashing of jobs no grid claimed: digests and blob CRCs still equal the
    oracle, and the run did relaunch the grid or leave jobs to the host (the paths round 4
    left untested)."""
    monkeypatch.setenv("PBS_PIPE_IDLE_MS", "0")
    monkeypatch.setenv("PBS_PIPE_HOST_MIN", "0")  # every digest on the GPU queue
    n = 48 * MiB + 5
    data = gen_np.gen_vmimage(n, 0x5EED0003, 0)
    ends, dig, crcs, t = gpu.pipeline_host(data, 256 << 10, piece=1 << 20, digest_cus=32, crc=True)
    ref = oracle.chunk_feed(256 << 10, data)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert np.array_equal(ends, ref)
    bounds = np.concatenate([[0], ref]).astype(np.uint64)
    assert np.array_equal(dig, oracle.chunk_digests(data, bounds))
    assert np.array_equal(crcs, oracle.chunk_crcs(data, bounds))
    assert t["gpu_jobs"] == ref.size and t["host_chunks"] == 0
    assert t["queue_launches"] > 1 or t["gpu_claimed"] < t["gpu_jobs"], t


def test_pipeline_beside_null_stream_work(gpu, oracle, torch_dev):
    """pbs_pipeline_host while another thread keeps issuing null-stream work (torch's
    default stream, and new Chunker handles, whose table upload once went through the null
    stream): the pipeline's resident queue grid sits on a blocking stream, so each such
    operation waits for the grid, the grid for the main thread's next publish, and that
    for a scan queued behind the null-stream work.  The idle exit (50 ms) breaks the cycle;
    the call finishes in bounded time and the results equal the oracle."""
    import threading
    import time

    torch = torch_dev
    n = 96 * MiB + 3
    data = gen_np.gen_vmimage(n, 0x5EED0003, 0)
    gpu.pipeline_host(data[: 8 * MiB], 1 << 20, piece=2 << 20)  # warm-up (work area, code objects)
    stop = threading.Event()
    ops = [0]

    def other():
        x = torch.zeros(1 << 20, device="cuda")
        while not stop.is_set():
            with gpu.Chunker(64 << 10):
                pass
            x.add_(1)  # the default (null) stream
            torch.cuda.current_stream().synchronize()
            ops[0] += 1

    th = threading.Thread(target=other)
    th.start()
    try:
        t0 = time.perf_counter()
        ends, dig, t = gpu.pipeline_host(data, 1 << 20, piece=2 << 20, digest_cus=32)
        wall = time.perf_counter() - t0
    finally:
        stop.set()
        th.join()
    ref = oracle.chunk_feed(1 << 20, data)
    if ref.size == 0 or int(ref[-1]) != n:
        ref = np.append(ref, np.uint64(n))
    assert np.array_equal(ends, ref)
    assert np.array_equal(dig, oracle.chunk_digests(data, np.concatenate([[0], ref]).astype(np.uint64)))
    assert ops[0] > 0
    # 48 pieces: with round 4's 10 s idle exit one such cycle alone took 10 s
    assert wall < 8.0, (wall, ops[0], t)


@pytest.mark.parametrize("spec", ["1", "0"])
@pytest.mark.parametrize("prev,compress", [(0, True), (5, True), (40, True), (5, False)])
def test_upload_stream_host(gpu, oracle, monkeypatch, prev, compress, spec):
    """backup_writer.rs:631-706 end to end from a host buffer: cut list, digests, the
    known-chunk mask against a previous index holding some of this stream's digests (plus
    unrelated ones) and repeats inside the stream, the .didx image, and every new chunk's
    blob as DataChunkBuilder::new(data).compress(compress).build() writes it (oracle: the
    twin's frame behind the blob header where shorter, data_blob.rs:139-176; the
    uncompressed blob otherwise), plus UploadStats.  spec 1 (default): the known test,
    the encoding and the blobs' copy per piece beside the copies; 0: after the pipeline."""
    monkeypatch.setenv("PBS_UPLOAD_SPEC", spec)
    n = 48 * MiB + 5
    data = gen_np.gen_vmimage(n, 0x5EED0003, 0)
    ref_ends = oracle.chunk_feed(1 * MiB, data)
    if ref_ends.size == 0 or int(ref_ends[-1]) != n:
        ref_ends = np.append(ref_ends, np.uint64(n))
    bounds = np.concatenate([[0], ref_ends]).astype(np.uint64)
    ref_dig = oracle.chunk_digests(data, bounds)
    rng = np.random.default_rng(prev)
    pick = rng.choice(ref_dig.shape[0], size=min(prev, ref_dig.shape[0]), replace=False)
    known = [bytes(ref_dig[i]) for i in pick] + [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(prev)]
    out = gpu.upload_stream_host(data, 1 * MiB, known=known, piece=16 * MiB, uuid=bytes(range(16)), ctime=77,
                                 compress=compress)
    assert np.array_equal(out["ends"], ref_ends)
    assert np.array_equal(out["digests"], ref_dig)
    ref_known = oracle.known_chunks(ref_dig, known)
    assert np.array_equal(out["known"], ref_known)
    img, csum = oracle.didx_image(ref_ends, ref_dig, bytes(range(16)), 77)
    assert out["didx"] == img and out["csum"] == csum
    _check_blobs(oracle, data, bounds, ref_known, out, compress)


def _check_blobs(oracle, data, bounds, ref_known, out, compress):
    new = [i for i in range(ref_known.size) if not ref_known[i]]
    assert out["new_chunks"] == [(int(bounds[i]), int(bounds[i + 1] - bounds[i])) for i in new]
    size_compressed = 0
    offs = out["blob_offsets"]
    for (s, ln), i in zip(out["new_chunks"], new):
        chunk = data[s:s + ln].tobytes()
        blob = out["blobs"][int(offs[i]):int(offs[i + 1])].tobytes()
        exp = oracle.blob_compressed(chunk) if compress else oracle.blob_uncompressed(chunk)
        assert blob == exp, f"chunk {i} ({ln} bytes)"
        assert bool(out["compressed"][i]) == (blob[:8] == oracle.COMPRESSED_BLOB_MAGIC)
        if out["compressed"][i]:
            assert oracle.zstd_decompress(blob[12:], ln) == chunk
        size_compressed += len(blob)
    assert all(out["blob_offsets"][i + 1] == out["blob_offsets"][i] for i in range(ref_known.size) if ref_known[i])
    st = out["stats"]
    assert st["chunk_count"] == ref_known.size and st["chunk_reused"] == int(ref_known.sum())
    assert st["size"] == data.size and st["size_compressed"] == size_compressed
    assert st["size_reused"] == sum(int(bounds[i + 1] - bounds[i]) for i in range(ref_known.size) if ref_known[i])


def test_upload_stream_mixed_compressed(gpu, oracle):
    """The compressing upload over a mixed stream -- English-like text, a pxar-like
    archive, VM-image pages, and a second copy of the text (its chunks repeat once the
    chunker resyncs: known within the stream) -- with a previous index holding a few of
    its digests: blobs equal the twin's, every zstd payload decodes with libzstd."""
    import corpus_gen
    text = corpus_gen.text(6 * MiB, 11)
    data = np.concatenate([text, corpus_gen.pxar(6 * MiB, 12), gen_np.gen_vmimage(8 * MiB, 0x5EED0003, 0), text])
    avg = 256 << 10
    ref_ends = oracle.chunk_feed(avg, data)
    if ref_ends.size == 0 or int(ref_ends[-1]) != data.size:
        ref_ends = np.append(ref_ends, np.uint64(data.size))
    bounds = np.concatenate([[0], ref_ends]).astype(np.uint64)
    ref_dig = oracle.chunk_digests(data, bounds)
    known = [bytes(ref_dig[i]) for i in (3, 40, 77)]
    out = gpu.upload_stream_host(data, avg, known=known, piece=5 * MiB + 3)
    assert np.array_equal(out["ends"], ref_ends) and np.array_equal(out["digests"], ref_dig)
    ref_known = oracle.known_chunks(ref_dig, known)
    assert np.array_equal(out["known"], ref_known)
    assert int(ref_known.sum()) > 10  # the repeated text's chunks
    _check_blobs(oracle, data, bounds, ref_known, out, True)


def test_reference_digest_vectors(gpu, torch_dev):
    """The reference-held golden digests (tests/blob_writer.rs:11-32, fixture
    tests/golden/blob_writer_digests.json): TEST_DATA = 100 000 bytes i % 255 digested on
    the GPU gives TEST_DIGEST_PLAIN, and with the id_key of CryptConfig::new([1; 32])
    (PBKDF2-HMAC-SHA256, "_id_key", 10 rounds; crypt_config.rs:42-51, 79-84)
    TEST_DIGEST_ENC -- also as one chunk among others at every start alignment."""
    import hashlib
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "golden", "blob_writer_digests.json")) as f:
        v = json.load(f)
    test_data = (np.arange(100_000) % 255).astype(np.uint8)
    key = hashlib.pbkdf2_hmac("sha256", bytes([1] * 32), b"_id_key", 10, 32)
    for pad in range(4):
        t, ptr = _dev(torch_dev, test_data, pad)
        bounds = np.array([0, test_data.size], dtype=np.uint64)
        assert bytes(gpu.digest_chunks_device(ptr, test_data.size, bounds)[0]).hex() == v["digest_plain"]
        assert bytes(gpu.digest_chunks_device(ptr, test_data.size, bounds, key=key)[0]).hex() == v["digest_enc"]
        del t
    # inside a stream, between other chunks (absolute offsets with a base)
    head = gen_np.gen_random(777, 5)
    tail = gen_np.gen_random(4096 + 9, 6)
    stream = np.concatenate([head, test_data, tail])
    t, ptr = _dev(torch_dev, stream, 3)
    base = 1 << 33
    bounds = np.array([0, head.size, head.size + test_data.size, stream.size], dtype=np.uint64) + np.uint64(base)
    for k, want in ((None, v["digest_plain"]), (key, v["digest_enc"])):
        dig = gpu.digest_chunks_device(ptr, stream.size, bounds, base=base, key=k)
        assert bytes(dig[1]).hex() == want


def _hybrid_case():
    """Chunks of 0..3 MiB random data, a few long ones (9 MiB - 3, 4 MiB + 17 bytes: more
    than one 4 MiB D2H slice, not 64-byte multiples), all-zero chunks of two lengths
    (3 x 2 MiB, 2 x (1 MiB + 5)) beside a non-zero 2 MiB chunk, a zero chunk under the
    1 MiB zero-test floor and empty chunks."""
    rng = np.random.default_rng(21)
    segs = [("r", int(x)) for x in rng.integers(0, 3 * MiB, 24)]
    segs += [("r", 9 * MiB - 3), ("r", 4 * MiB + 17), ("r", 2 * MiB), ("r", 0), ("r", 0)]
    segs += [("z", 2 * MiB)] * 3 + [("z", MiB + 5)] * 2 + [("z", MiB - 1)]
    order = rng.permutation(len(segs))
    parts = []
    for k, i in enumerate(order):
        kind, n = segs[i]
        parts.append(np.zeros(n, np.uint8) if kind == "z" else gen_np.gen_random(n, 1000 + k))
    data = np.concatenate(parts)
    bounds = np.concatenate([[0], np.cumsum([p.size for p in parts])]).astype(np.uint64)
    return data, bounds


@pytest.mark.parametrize("mode", ["auto", "host_from_hbm", "host_from_hbm_slices", "host_from_copy", "gpu_only",
                                  "one_thread", "one_thread_all"])
@pytest.mark.parametrize("key", [None, bytes(range(32))])
def test_hybrid_digest(gpu, oracle, torch_dev, mode, key, monkeypatch):
    """pbs_digest_chunks_hybrid against the oracle: the host share reading from HBM
    (whole chunks through the pinned ring -- with one thread and every chunk on the host
    its 12 slots are reused -- or, PBS_DIGEST_RING=0, 4 MiB slices per thread) or from a
    host copy, the GPU share, and the all-zero long chunks hashed once per length and
    copied to the rest."""
    data, bounds = _hybrid_case()
    t, ptr = _dev(torch_dev, data, 3)
    kw = {"auto": dict(threads=4),
          "host_from_hbm": dict(threads=4, host_min_len=1),
          "host_from_hbm_slices": dict(threads=4, host_min_len=1),
          "host_from_copy": dict(threads=4, host_min_len=1, host=data),
          "gpu_only": dict(threads=-1),
          "one_thread": dict(threads=1, host_min_len=MiB),
          "one_thread_all": dict(threads=1, host_min_len=1)}[mode]
    if mode == "host_from_hbm_slices":
        monkeypatch.setenv("PBS_DIGEST_RING", "0")
    got, tm = gpu.digest_chunks_hybrid(ptr, data.size, bounds, key=key, **kw)
    assert np.array_equal(got, oracle.chunk_digests(data, bounds, key or b""))
    n = bounds.size - 1
    if mode == "gpu_only":
        assert tm["host_chunks"] == 0 and tm["gpu_chunks"] == n and tm["zero_chunks"] == 0
    else:
        assert tm["zero_chunks"] == 5 and tm["zero_lengths"] == 2
        assert tm["host_chunks"] + tm["gpu_chunks"] == n - 3
    if mode.startswith("host_from") or mode == "one_thread_all":
        assert tm["gpu_chunks"] == 2  # the empty chunks (length 0 < host_min_len)


def test_hybrid_digest_vm_stream(gpu, oracle, torch_dev):
    """Chunker -> hybrid digest on a 512 MiB VM-image stream at 4 MiB (forced 16 MiB
    chunks of the zero extents, long data chunks) with the default cost model."""
    n = 512 * MiB + 77
    data = gen_np.gen_vmimage(n, 0x5EED0009, 0)
    t, ptr = _dev(torch_dev, data)
    with gpu.Chunker(4 * MiB) as c:
        ends = c.find_cuts_device(ptr, n, is_final=True)
    if ends.size == 0 or int(ends[-1]) != n:
        ends = np.append(ends, np.uint64(n))
    bounds = np.concatenate([[0], ends]).astype(np.uint64)
    want = oracle.chunk_digests(data, bounds)
    got, tm = gpu.digest_chunks_hybrid(ptr, n, bounds, threads=8)
    assert np.array_equal(got, want)
    # (at this size the model hands the host every chunk: 8 threads clear 512 MiB before
    # one GPU lane finishes a 4 MiB chunk)
    assert tm["host_chunks"] > 0
    # a slow host rate in the model: a real split
    got, tm = gpu.digest_chunks_hybrid(ptr, n, bounds, threads=8, host_mb_s=100)
    assert np.array_equal(got, want)
    assert tm["host_chunks"] > 0 and tm["gpu_chunks"] > 0


def test_hybrid_digest_threads(gpu, oracle, torch_dev):
    """Two threads run the hybrid digest at once on their own streams (the device's host
    stage -- ring, copy streams -- is shared under its lock): every digest equal to the
    oracle's."""
    import threading

    import torch

    cases = []
    for k in range(2):
        data, bounds = _hybrid_case()
        data = data.copy()
        data[::4097] ^= np.uint8(k + 1)  # different bytes per thread
        t, ptr = _dev(torch_dev, data)
        cases.append((data, bounds, t, ptr, torch.cuda.Stream()))
    torch.cuda.synchronize()
    got, errs = [None, None], []

    def run(k):
        data, bounds, t, ptr, s = cases[k]
        try:
            for _ in range(3):
                got[k], _ = gpu.digest_chunks_hybrid(ptr, data.size, bounds, threads=2, host_min_len=1,
                                                     hip_stream=s.cuda_stream)
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    ths = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    [x.start() for x in ths]
    [x.join() for x in ths]
    assert not errs, errs
    for k in range(2):
        data, bounds = cases[k][0], cases[k][1]
        assert np.array_equal(got[k], oracle.chunk_digests(data, bounds))
