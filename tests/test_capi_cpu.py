"""CPU-only checks of the C-ABI library (no compute calls): it loads, exports every
symbol include/*.h declares, carries the right table, and fails loudly
without a device.  Plus the Python host mirror's caller logic (ChunkStream,
DynamicChunkWriter) driven by the oracle chunker as a stand-in."""
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include"))
                 if h.endswith(".h"))
KiB, MiB = 1024, 1024 * 1024


def declared_functions():
    src = "".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pbs_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_api():
    names = declared_functions()
    for n in ("pbs_chunker_new", "pbs_chunker_scan", "pbs_chunker_free", "pbs_chunker_find_cuts",
              "pbs_chunker_find_cuts_device", "pbs_chunker_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol(pbschunk):
    lib = pbschunk.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) == set(pbschunk.EXPORTED_SYMBOLS)
    nm = subprocess.run(["nm", "-D", "--defined-only", pbschunk.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (pbs_[a-z0-9_]+)\b", nm))
    assert set(declared_functions()) <= exported


def test_library_has_gfx950_code_object(pbschunk):
    # the fat binary embeds the offload bundle id "hipv4-amdgcn-amd-amdhsa--gfx950"
    assert b"amdgcn-amd-amdhsa--gfx950" in open(pbschunk.LIB_PATH, "rb").read()


def test_table_digest_of_library(pbschunk, oracle):
    t = pbschunk.table()
    assert hashlib.sha256(t.astype("<u4").tobytes()).hexdigest() == oracle.TABLE_SHA256


def test_strerror_and_max_cuts(pbschunk):
    assert "power of two" in pbschunk.strerror(pbschunk.PBS_ERR_NOT_POW2)
    assert pbschunk.max_cuts(0) >= 1
    assert pbschunk.max_cuts(65 * 1000) >= 1000
    # without a handle the bound falls back to the any-average one
    assert pbschunk.lib().pbs_chunker_cuts_bound(None, 65 * 1000) == pbschunk.max_cuts(65 * 1000)


@pytest.mark.parametrize("avg", [64, 1024, 64 * KiB, 4 * MiB])
def test_cuts_bound_holds_on_oracle_cuts(oracle, avg):
    """pbs_chunker_cuts_bound(len) = len // max(avg/4, 65) + 3 covers the cuts any call
    over a byte range can return (checked on the oracle's cut lists, any split)."""
    import gen_np
    n = 24 * MiB if avg >= 64 * KiB else 2 * MiB
    data = gen_np.gen_vmimage(n, 0x5EED0003, 700 * MiB)
    cuts = oracle.chunk_feed(avg, data).astype(np.int64)
    ends = np.append(cuts, n) if cuts.size == 0 or cuts[-1] != n else cuts
    min_eff = max(avg // 4, 65)
    rng = np.random.default_rng(avg)
    for _ in range(200):
        a, b = sorted(rng.integers(0, n + 1, 2))
        inside = int(((ends > a) & (ends <= b)).sum())
        assert inside <= (b - a) // min_eff + 3, (a, b, inside)


def test_non_power_of_two_rejected_like_reference(pbschunk):
    for avg in (0, 3, 3 * MiB):
        with pytest.raises(ValueError, match="not a power of two"):
            pbschunk.Chunker(avg)


def test_no_device_fails_loudly(pbschunk):
    if pbschunk.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(pbschunk.ChunkerError) as ei:
        pbschunk.Chunker(4 * MiB)
    assert ei.value.code == pbschunk.PBS_ERR_NO_DEVICE


# ---- host caller logic, with the oracle Chunker standing in for the GPU one --------

def _patch_chunker(monkeypatch, pbschunk, oracle):
    monkeypatch.setattr(pbschunk, "Chunker", lambda avg: oracle.Chunker(avg))


def test_chunk_stream_logic(monkeypatch, pbschunk, oracle):
    _patch_chunker(monkeypatch, pbschunk, oracle)
    data = oracle.gen_random(3 * MiB + 17, 21)
    ref = oracle.chunk_feed(64 * KiB, data)
    for piece, min_scan in ((1000, 0), (1000, 300 * KiB), (64 * KiB, 4 * MiB), (256 * KiB, 0), (256 * KiB, 1)):
        pieces = [data[i:i + piece].tobytes() for i in range(0, data.size, piece)]
        cs = pbschunk.ChunkStream(pieces, 64 * KiB)
        cs.min_scan = min_scan  # coalescing pieces per scan must not move a cut
        chunks = list(cs)
        ends = np.cumsum([len(c) for c in chunks])
        assert b"".join(chunks) == data.tobytes()
        assert np.array_equal(ends[:-1], ref) or np.array_equal(ends, ref)


def test_dynamic_chunk_writer_logic(monkeypatch, pbschunk, oracle):
    _patch_chunker(monkeypatch, pbschunk, oracle)
    data = oracle.gen_vmimage(2 * MiB, 5, 0)
    got = []
    w = pbschunk.DynamicChunkWriter(lambda end, b: got.append((end, len(b))), 16 * KiB)
    for i in range(0, data.size, 65536):
        w.write_all(data[i:i + 65536].tobytes())
    w.close()
    ref = oracle.chunk_feed(16 * KiB, data).tolist()
    ends = [e for e, _ in got]
    assert ends[:len(ref)] == ref and ends[-1] == data.size
    assert sum(n for _, n in got) == data.size


@pytest.mark.parametrize("nw", [2045, 1021, 13])
def test_fused_static_plan_covers_the_batch(pbschunk, nw):
    """The static tile plan of the fused pass (pbs_chunker_capi.cpp fused_static_plan):
    the tiles cover the batch up to less than one row of 64 blocks (8 KiB; batches under 32
    rows are tail items only), no segment
    exceeds the kernel's bitmap (40 KiB), every wave gets the same number of full-round
    tiles, and the short last round (if any) is one tile per wave or, from 8 rounds on, a
    pool of 8 small tiles per wave."""
    import ctypes
    lib = pbschunk.lib()
    f = lib.pbs_test_fused_static_plan
    f.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
    out = (ctypes.c_uint64 * 8)()
    rng = np.random.default_rng(7)
    sizes = [0, 1, 8191, 8192, 32 * 8192 - 1, 32 * 8192, 1 << 20, (1 << 20) + 77, 64 * MiB + 12345,
             1 << 30, (1 << 30) + 12345, 8 << 30, int(5.5 * (1 << 30)) + 12345, 64 << 30,
             (64 << 30) + 4099, 200 << 30] + [int(x) for x in rng.integers(1, 70 << 30, 40)]
    for n in sizes:
        assert f(n, nw, out) == 0
        nt, q, tl, ts, qs, tsl, cov, pool = (int(x) for x in out)
        if nt == 0:  # under 32 rows: tail items only (the fused pass serves > 1 MiB)
            assert cov == 0 and n < 32 * 64 * 128
            continue
        assert cov <= n and n - cov < 64 * 128, (n, list(out))
        assert 0 < ts <= nt and tl < max(ts, 1) and tsl <= nt - ts
        assert (q + (tl > 0)) * 128 <= 40960 and (qs + (tsl > 0)) * 128 <= 40960
        assert q >= 32 or ts == nt
        if nt > ts:  # rounds of full tiles plus one short round, or a pool drawn dynamically
            assert ts % nw == 0 and (nt - ts) % nw == 0 and 0 < qs <= q
            assert (nt - ts == nw) == (pool == 0)
        elif nt >= nw:
            assert nt % nw == 0
