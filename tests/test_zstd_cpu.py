"""CPU checks of the zstd-1 blob stage's format writer (csrc/zstd_enc.h) through its host
twin (oracle/zstd_twin.cpp, the GPU parse written as loops): every frame decodes with the
image's libzstd (1.4.8) back to the input, across block boundaries, RLE, raw and
compressed blocks, and the blob rules of data_blob.rs:139-176.

Parity of the compressed BYTES with the reference is unpinned: the reference writes
libzstd 1.5.x level-1 frames (data_blob.rs:151), which no encoder here reproduces; the
reference only ever decodes them with `zstd::stream::decode_all` (:214), so a frame that
decodes to the chunk is a valid drop-in."""
import struct
import zlib

import numpy as np
import pytest

import gen_np

KiB, MiB = 1024, 1024 * 1024


def _inputs():
    rng = np.random.default_rng(5)
    text = np.frombuffer(b"proxmox backup chunk store " * 5000, dtype=np.uint8)
    yield "empty", np.zeros(0, np.uint8)
    for n in (1, 2, 3, 4, 5, 31, 32, 33, 63, 64, 255, 256, 257, 4095, 4096, 65791, 65792):
        yield f"random_{n}", rng.integers(0, 256, n, dtype=np.uint8)
    yield "text", text
    yield "zeros_128K", np.zeros(128 * KiB, np.uint8)
    yield "zeros_128K+1", np.zeros(128 * KiB + 1, np.uint8)
    yield "ff_300K", np.full(300 * KiB, 0xFF, np.uint8)
    yield "text_256K+5", np.resize(text, 256 * KiB + 5)
    yield "random_300K", gen_np.gen_random(300 * KiB, 9)
    yield "counter_1M", gen_np.gen_counter(MiB)
    yield "vm_4M", gen_np.gen_vmimage(4 * MiB, 0x5EED0003, 0)
    # periodic data whose matches run across block boundaries and to the block end
    yield "period7_400K", np.resize(np.arange(7, dtype=np.uint8), 400 * KiB)
    # random pages with short repeats (many sequences per block)
    base = rng.integers(0, 256, 64, dtype=np.uint8)
    import corpus_gen
    yield "text_1M", corpus_gen.text(MiB, 3)
    yield "pxar_1M", corpus_gen.pxar(MiB, 4)
    # binary literals (symbols above 128: FSE-coded Huffman weights) and skewed bytes
    yield "skewed_300K", np.minimum(rng.geometric(0.05, 300 * KiB), 255).astype(np.uint8)
    yield "high_bytes_200K", (255 - np.minimum(rng.geometric(0.08, 200 * KiB), 200)).astype(np.uint8)
    yield "two_symbols_100K", rng.choice(np.array([7, 200], np.uint8), 100 * KiB)
    yield "short_repeats_512K", np.concatenate([np.concatenate([base[:rng.integers(4, 60)],
                                                                rng.integers(0, 256, 9, dtype=np.uint8)])
                                                for _ in range(12000)])[: 512 * KiB]


@pytest.mark.parametrize("name,data", list(_inputs()), ids=[n for n, _ in _inputs()])
def test_twin_frames_decode_with_libzstd(oracle, name, data):
    f = oracle.zstd_twin_frame(data.tobytes())
    assert f[:4] == b"\x28\xb5\x2f\xfd"
    assert oracle.zstd_decompress(f, data.size) == data.tobytes()
    assert len(f) <= 13 + data.size + 3 * max(1, -(-data.size // (64 * KiB)))  # frame bound


def test_blob_rules(oracle):
    """data_blob.rs:139-176: compressed blob only if the frame is shorter; CRC over the
    payload (compute_crc :70-75); header magic per file_formats.rs:9/:12."""
    zeros = bytes(200 * KiB)
    b = oracle.blob_compressed(zeros)
    assert b[:8] == oracle.COMPRESSED_BLOB_MAGIC
    assert struct.unpack("<I", b[8:12])[0] == zlib.crc32(b[12:])
    assert oracle.zstd_decompress(b[12:], len(zeros)) == zeros
    rnd = gen_np.gen_random(100 * KiB, 3).tobytes()  # incompressible: stays uncompressed
    b = oracle.blob_compressed(rnd)
    assert b == oracle.blob_uncompressed(rnd)


@pytest.mark.parametrize("corpus", ["text", "pxar", "vmimage"])
def test_ratio_near_libzstd_level1(oracle, corpus):
    """Not parity, the ratio bar: over 4 MiB chunks of text-like, pxar-like and VM-image
    data (tests/corpus_gen.py, seeded generators) the frames are within 10 % of libzstd
    level 1's size -- the reference's compressor (data_blob.rs:151) -- and decode."""
    import corpus_gen
    n = 8 * MiB
    data = {"text": lambda: corpus_gen.text(n), "pxar": lambda: corpus_gen.pxar(n),
            "vmimage": lambda: gen_np.gen_vmimage(n, 0x5EED0003, 0)}[corpus]()
    L = oracle.libzstd()
    ours = ref = 0
    for i in range(0, data.size, 4 * MiB):
        c = np.ascontiguousarray(data[i:i + 4 * MiB])
        dst = np.empty(L.ZSTD_compressBound(c.size), np.uint8)
        ref += L.ZSTD_compress(dst.ctypes.data, dst.size, c.ctypes.data, c.size, 1)
        f = oracle.zstd_twin_frame(c.tobytes())
        assert oracle.zstd_decompress(f, c.size) == c.tobytes()
        ours += len(f)
    assert ours <= ref * 1.10, (corpus, ours, ref, ours / ref)


def test_code_functions_match_tables(tmp_path):
    """The encoder's arithmetic code functions (zstd_enc.h: ll_code / ml_code and the
    baseline / extra-bit functions the GPU kernels use instead of table loads) equal the RFC
    8878 tables and their searches for every length a block can produce."""
    import shutil
    import subprocess
    from pathlib import Path

    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    root = Path(__file__).resolve().parent.parent
    exe = tmp_path / "zstd_codes_check"
    subprocess.run([cxx, "-std=c++17", "-O1", "-I", str(root / "proxmox-backup_amd" / "csrc"),
                    str(root / "tests" / "cpp" / "zstd_codes_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and "bad 0" in r.stdout, r.stdout
