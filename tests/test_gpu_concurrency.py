"""Distinct chunker handles used at the same time from different threads, one HIP stream
each -- the concurrency include/pbs_chunker.h promises (SURVEY.md 8(b) "Threading":
separate instances are independent and may run concurrently).  The fused pass waits
across workgroups (its resolver reads other workgroups' tile records) and scan() keeps a
persistent polling kernel per handle, so these runs check that neither starves the
other and that every result still equals the oracle's.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
import threading
import time

import numpy as np
import pytest

import gen_np
from test_gpu_parity import _oracle_two_phase_parallel

pytestmark = pytest.mark.gpu
KiB, MiB, GiB = 1024, 1024 * 1024, 1024 * 1024 * 1024


def _scan_loop(c, data, piece):
    """ChunkStream's loop (chunk_stream.rs:40-77): one scan() per `piece`-byte read."""
    got = []
    for start in range(0, data.size, piece):
        p = data[start:start + piece]
        off = 0
        while off < p.size:
            k = c.scan(p[off:])
            if k == 0:
                break
            off += k
            got.append(start + off)
    return np.array(got, dtype=np.uint64)


def _with_end(cuts, n):
    """The oracle's cut list plus the stream end (find_cuts with is_final reports the tail)."""
    if cuts.size == 0 or int(cuts[-1]) != n:
        cuts = np.append(cuts, np.uint64(n))
    return cuts


def _run_threads(*fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # surfaced in the main thread
            errs.append(e)

    ths = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    [t.start() for t in ths]
    [t.join(timeout=300) for t in ths]
    assert not any(t.is_alive() for t in ths), "a handle did not finish (deadlock?)"
    if errs:
        raise errs[0]


def test_fused_pass_beside_scan_server(gpu, oracle, monkeypatch):
    """Thread A: one handle on its own stream, fused passes (PBS_FUSED=1) over an 8 GiB
    device-resident VM image, as many as fit while thread B runs.  Thread B: another
    handle, scan() per 8 KiB read over 192 MiB of random host bytes (the scan server's
    persistent kernel).  Both diffed against the oracle."""
    import torch

    monkeypatch.setenv("PBS_FUSED", "1")
    torch.cuda.set_device(0)
    n = 8 * GiB
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.generate_device(dev.data_ptr(), n, gpu.GEN_VMIMAGE, 0x5EED0003, 0)
    torch.cuda.synchronize()
    ref_a = _with_end(_oracle_two_phase_parallel(oracle, dev.cpu().numpy(), 4 * MiB)[1], n)
    data_b = gen_np.gen_random(192 * MiB, 0x5EED00B0)
    ref_b = oracle.chunk_feed(4 * MiB, data_b)
    a_out, b_out, b_running = [], [], threading.Event()
    b_running.set()

    def run_a():
        s = torch.cuda.Stream()
        with gpu.Chunker(4 * MiB) as c:
            c.set_stream(s.cuda_stream)
            while b_running.is_set() or len(a_out) < 3:
                a_out.append(c.find_cuts_device(dev.data_ptr(), n, is_final=True))
                assert c.last_timing()["fused"] == n  # the one-launch pass served it

    def run_b():
        try:
            with gpu.Chunker(4 * MiB) as c:
                b_out.append(_scan_loop(c, data_b, 8 * KiB))
        finally:
            b_running.clear()

    _run_threads(run_a, run_b)
    assert len(a_out) >= 3
    for i, got in enumerate(a_out):
        assert np.array_equal(got, ref_a), f"pass {i}"
    assert np.array_equal(b_out[0], ref_b)


def test_two_fused_passes_at_once(gpu, oracle, monkeypatch):
    """Two handles, two streams, two threads, each running fused passes over its own
    4 GiB stream at the same time (the two persistent grids compete for the CUs; each
    resolver waits only for its own pass's tile records)."""
    import torch

    monkeypatch.setenv("PBS_FUSED", "1")
    torch.cuda.set_device(0)
    n = 4 * GiB
    bufs, refs = [], []
    for kind, seed in ((gpu.GEN_VMIMAGE, 0x5EED0003), (gpu.GEN_RANDOM, 0x5EED0002)):
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        gpu.generate_device(d.data_ptr(), n, kind, seed, 0)
        torch.cuda.synchronize()
        bufs.append(d)
        refs.append(_with_end(_oracle_two_phase_parallel(oracle, d.cpu().numpy(), 1 * MiB)[1], n))
    outs = [[], []]
    t_end = time.monotonic() + 3.0

    def run(k):
        s = torch.cuda.Stream()
        with gpu.Chunker(1 * MiB) as c:
            c.set_stream(s.cuda_stream)
            while time.monotonic() < t_end or len(outs[k]) < 3:
                outs[k].append(c.find_cuts_device(bufs[k].data_ptr(), n, is_final=True))

    _run_threads(lambda: run(0), lambda: run(1))
    for k in range(2):
        assert len(outs[k]) >= 3
        for i, got in enumerate(outs[k]):
            assert np.array_equal(got, refs[k]), f"handle {k} pass {i}"


def test_blob_and_digest_threads_reuse_work_areas(gpu, oracle):
    """Two threads, two streams: blob encoding (zstd frames + CRC) of one stream and
    SHA-256 + CRC-32 of another's chunks at the same time, three rounds each.  Every
    result equals the twin's / hashlib's / zlib's, and after one warm-up call of each the
    repeated calls allocate no device memory (per-device work areas, csrc/dev_arena.h:
    no hipMalloc / hipFree on the hot call)."""
    import zlib

    import torch

    import corpus_gen
    torch.cuda.set_device(0)
    ta = np.concatenate([corpus_gen.text(6 * MiB, 31), corpus_gen.pxar(6 * MiB, 32),
                         gen_np.gen_vmimage(4 * MiB, 0x5EED0003, 0)])
    tb = gen_np.gen_vmimage(96 * MiB, 0x5EED0004, 5 * GiB)
    bounds = []
    for d in (ta, tb):
        c = oracle.chunk_feed(256 * KiB, d)
        bounds.append(np.concatenate([[0], _with_end(c, d.size)]).astype(np.uint64))
    da, db = (torch.from_numpy(x).to("cuda") for x in (ta, tb))
    torch.cuda.synchronize()
    cap = gpu.blob_stream_bound(bounds[0])
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    exp_blobs = [oracle.blob_compressed(ta[int(a):int(b)].tobytes()) for a, b in zip(bounds[0][:-1], bounds[0][1:])]
    exp_dig = oracle.chunk_digests(tb, bounds[1])
    exp_crc = oracle.chunk_crcs(tb, bounds[1])
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def blobs():
        offs, crcs, comp, tm = gpu.blob_encode_chunks_device(da.data_ptr(), ta.size, bounds[0], out.data_ptr(), cap,
                                                             hip_stream=sa.cuda_stream)
        img = out[: int(offs[-1])].cpu().numpy().tobytes()
        for i, e in enumerate(exp_blobs):
            b = img[int(offs[i]):int(offs[i + 1])]
            assert b == e, f"blob {i}"
            assert int(crcs[i]) == zlib.crc32(b[12:])

    def digests():
        dg = gpu.digest_chunks_device(db.data_ptr(), tb.size, bounds[1], hip_stream=sb.cuda_stream)
        assert np.array_equal(dg, exp_dig)
        cr = gpu.crc32_chunks_device(db.data_ptr(), tb.size, bounds[1], hip_stream=sb.cuda_stream)
        assert np.array_equal(cr, exp_crc)

    blobs()
    digests()
    a0 = gpu.debug_arena_allocs()

    def loop(f):
        return lambda: [f() for _ in range(3)]

    _run_threads(loop(blobs), loop(digests))
    assert gpu.debug_arena_allocs() == a0, "a repeated call allocated device memory"
