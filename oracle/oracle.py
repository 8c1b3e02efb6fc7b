"""ctypes wrapper of the CPU oracle (oracle/chunker_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` as the checker.  The product (the HIP path in
``proxmox-backup_amd/``) never imports this module.

Reference: pbs-datastore/src/chunker.rs:75-186 (see chunker_oracle.c header).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

WINDOW = 64
TABLE_SHA256 = "5b52080d38287da9d2e278466e3e0db7ec98e5e8b226f50612a56fa012b1f660"


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, p = ctypes.c_uint64, ctypes.c_void_p
        L.ora_sizeof_chunker.restype = u64
        L.ora_new.argtypes = [p, u64]
        L.ora_new.restype = ctypes.c_int
        L.ora_scan.argtypes = [p, p, u64]
        L.ora_scan.restype = u64
        L.ora_chunk_feed.argtypes = [u64, p, u64, u64, p, u64]
        L.ora_chunk_feed.restype = ctypes.c_int64
        L.ora_window_hash.argtypes = [p, u64]
        L.ora_window_hash.restype = ctypes.c_uint32
        L.ora_candidates.argtypes = [u64, p, u64, p, u64]
        L.ora_candidates.restype = ctypes.c_int64
        L.ora_resolve.argtypes = [u64, p, u64, u64, p, u64]
        L.ora_resolve.restype = ctypes.c_int64
        L.ora_splitmix64.argtypes = [u64]
        L.ora_splitmix64.restype = u64
        for name in ("ora_gen_random", "ora_gen_vmimage"):
            getattr(L, name).argtypes = [p, u64, u64, u64]
            getattr(L, name).restype = None
        L.ora_gen_counter.argtypes = [p, u64, u64]
        L.ora_gen_counter.restype = None
        L.ora_gen_block.argtypes = [ctypes.c_int, u64, p, u64, u64]
        L.ora_gen_block.restype = None
        L.ora_chunk_generated.argtypes = [ctypes.c_int, u64, u64, u64, u64, p, u64]
        L.ora_chunk_generated.restype = ctypes.c_int64
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


class Chunker:
    """Streaming oracle with the reference's surface: Chunker::new(avg) / scan(data)."""

    def __init__(self, chunk_size_avg: int):
        L = lib()
        self._buf = ctypes.create_string_buffer(int(L.ora_sizeof_chunker()))
        if L.ora_new(self._buf, int(chunk_size_avg)) != 0:
            raise ValueError("got unexpected chunk size - not a power of two.")

    def scan(self, data) -> int:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        return int(lib().ora_scan(self._buf, _ptr(a), a.size))


def build_info() -> dict:
    """The oracle library's compiler and flags (ora_build_info) and the SHA-256 of the .so."""
    import hashlib
    L = lib()
    L.ora_build_info.restype = ctypes.c_char_p
    with open(_LIB_PATH, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    return {"compiler_flags": L.ora_build_info().decode(), "so_sha256": sha[:16]}


def chunk_feed(avg: int, data: np.ndarray, feed: int = 0) -> np.ndarray:
    """Chunk END offsets (exclusive) of every cut when the stream arrives in pieces of
    ``feed`` bytes (0 = whole buffer).  The tail is not included."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cap = data.size // 65 + 2
    out = np.empty(cap, dtype=np.uint64)
    n = lib().ora_chunk_feed(int(avg), _ptr(data), data.size, int(feed), _ptr(out), cap)
    if n < 0:
        raise ValueError(f"oracle chunk_feed failed ({n})")
    return out[:n].copy()


def window_hash(data: np.ndarray, p: int) -> int:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    assert p >= WINDOW - 1
    return int(lib().ora_window_hash(_ptr(data), int(p)))


def candidates(avg: int, data: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    cap = max(16, data.size)
    out = np.empty(cap, dtype=np.uint64)
    n = lib().ora_candidates(int(avg), _ptr(data), data.size, _ptr(out), cap)
    if n < 0:
        raise ValueError(f"oracle candidates failed ({n})")
    return out[:n].copy()


def resolve(avg: int, cand: np.ndarray, length: int) -> np.ndarray:
    cand = np.ascontiguousarray(cand, dtype=np.uint64)
    cap = length // 65 + 2
    out = np.empty(cap, dtype=np.uint64)
    n = lib().ora_resolve(int(avg), _ptr(cand), cand.size, int(length), _ptr(out), cap)
    if n < 0:
        raise ValueError(f"oracle resolve failed ({n})")
    return out[:n].copy()


def gen_counter(length: int, offset: int = 0) -> np.ndarray:
    a = np.empty(length, dtype=np.uint8)
    lib().ora_gen_counter(_ptr(a), length, offset)
    return a


def gen_random(length: int, seed: int, offset: int = 0) -> np.ndarray:
    a = np.empty(length, dtype=np.uint8)
    lib().ora_gen_random(_ptr(a), length, seed, offset)
    return a


def gen_vmimage(length: int, seed: int, offset: int = 0) -> np.ndarray:
    a = np.empty(length, dtype=np.uint8)
    lib().ora_gen_vmimage(_ptr(a), length, seed, offset)
    return a


GEN_KINDS = {"counter": 0, "random": 1, "vmimage": 2}


def gen_block(kind: str, length: int, seed: int, offset: int = 0) -> np.ndarray:
    """The word-at-a-time generator (same bytes as gen_counter/gen_random/gen_vmimage)."""
    a = np.empty(length, dtype=np.uint8)
    lib().ora_gen_block(GEN_KINDS[kind], seed, _ptr(a), length, offset)
    return a


def chunk_generated(kind: str, seed: int, avg: int, length: int, piece: int = 16 << 20) -> np.ndarray:
    """Cut list (chunk END offsets, the stream end appended when the tail is non-empty:
    find_cuts(..., is_final=True)'s list) of a whole generated stream, generated and
    scanned `piece` bytes at a time by the streaming restatement of Chunker::scan --
    streams of any length in bounded memory.  Releases the GIL (ctypes)."""
    min_eff = max(avg // 4, 65)
    cap = length // min_eff + 2
    out = np.empty(cap, dtype=np.uint64)
    n = lib().ora_chunk_generated(GEN_KINDS[kind], seed, int(avg), int(length), int(piece),
                                  _ptr(out), cap)
    if n < 0:
        raise ValueError(f"oracle chunk_generated failed ({n})")
    return out[:n].copy()


def splitmix64(x: int) -> int:
    return int(lib().ora_splitmix64(x & 0xFFFFFFFFFFFFFFFF))


# ---- chunk digests and the dynamic index (checker only) ---------------
# The digest is openssl::sha::sha256 in the reference (data_blob.rs:516-536); hashlib's
# SHA-256 is the same FIPS 180-4 function.  With a crypt config the message is
# chunk || id_key (pbs-tools/src/crypt_config.rs:79-84).

def chunk_digests(data: np.ndarray, bounds, key: bytes = b"") -> np.ndarray:
    import hashlib

    b = [int(x) for x in bounds]
    mv = memoryview(np.ascontiguousarray(data))
    out = np.empty((max(0, len(b) - 1), 32), dtype=np.uint8)
    for i in range(len(b) - 1):
        h = hashlib.sha256(mv[b[i]:b[i + 1]])
        if key:
            h.update(key)
        out[i] = np.frombuffer(h.digest(), dtype=np.uint8)
    return out


DIDX_MAGIC = bytes([28, 145, 78, 165, 25, 186, 179, 205])  # file_formats.rs:24


def didx_image(ends, digests, uuid: bytes = bytes(16), ctime: int = 0):
    """dynamic_index.rs:28-37 (header: magic, uuid, ctime i64 LE, index_csum, 4032 zero
    bytes), :61-66 (entries {end_le u64, digest}), :373-391 (index_csum = SHA-256 over
    the entries as written).  Returns (image, index_csum)."""
    import hashlib
    import struct

    entries = b"".join(struct.pack("<Q", int(e)) + (d if isinstance(d, bytes) else
                                                    bytes(np.asarray(d, dtype=np.uint8)))
                       for e, d in zip(ends, digests))
    csum = hashlib.sha256(entries).digest()
    header = DIDX_MAGIC + bytes(uuid) + struct.pack("<q", int(ctime)) + csum
    header += bytes(4096 - len(header))
    return header + entries, csum


def known_chunks(digests, known) -> np.ndarray:
    """backup_writer.rs:677-697: a chunk is known iff its digest is in the set (the
    previous index's digests, :524-547); every new digest joins the set (:697)."""
    seen = {bytes(d) for d in known}
    out = np.zeros(len(digests), dtype=np.uint8)
    for i, d in enumerate(digests):
        b = bytes(d)
        if b in seen:
            out[i] = 1
        else:
            seen.add(b)
    return out


# ---- the blob CRC (checker only) --------------------------------
# DataBlob::compute_crc (data_blob.rs:70-75) is crc32fast::Hasher (Cargo.toml:111,
# crc32fast "1"), whose published algorithm is CRC-32/ISO-HDLC: reflected polynomial
# 0xEDB88320, init 0xFFFFFFFF, final XOR 0xFFFFFFFF, check value CRC("123456789") =
# 0xCBF43926 -- the same function as zlib.crc32 (crc32fast's own tests compare against
# it).  An uncompressed blob is UNCOMPRESSED_BLOB_MAGIC_1_0 || crc LE || data
# (file_formats.rs:9, :36-45; data_blob.rs:159-174).

UNCOMPRESSED_BLOB_MAGIC = bytes([66, 171, 56, 7, 190, 131, 112, 161])  # file_formats.rs:9


def chunk_crcs(data: np.ndarray, bounds) -> np.ndarray:
    import zlib

    b = [int(x) for x in bounds]
    mv = memoryview(np.ascontiguousarray(data))
    return np.array([zlib.crc32(mv[b[i]:b[i + 1]]) for i in range(len(b) - 1)], dtype=np.uint32)


def blob_uncompressed(chunk: bytes) -> bytes:
    import struct
    import zlib

    return UNCOMPRESSED_BLOB_MAGIC + struct.pack("<I", zlib.crc32(chunk)) + bytes(chunk)


# ---- zstd-1 blobs (data_blob.rs:139-176): parity of the compressed bytes is UNPINNED ----
# The reference's compressor is libzstd level 1 (zstd crate 0.12 -> libzstd 1.5.x), not in
# this image.  What is checked: (1) the GPU's frames equal the host twin's
# (oracle/zstd_twin.cpp, the same parse written as loops); (2) the image's libzstd.so.1
# (1.4.8, through ctypes) decodes every frame back to the chunk; (3) the blob rules below.
COMPRESSED_BLOB_MAGIC = bytes([49, 185, 88, 66, 111, 182, 163, 127])  # file_formats.rs:12
_twin = None
_zstd = None


def _twin_lib():
    global _twin
    if _twin is None:
        path = os.path.join(_HERE, "build", "libzstd_twin.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.zstd_twin_bound.restype = ctypes.c_uint64
        L.zstd_twin_bound.argtypes = [ctypes.c_uint64]
        L.zstd_twin_frame.restype = ctypes.c_uint64
        L.zstd_twin_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        _twin = L
    return _twin


def zstd_twin_frame(chunk) -> bytes:
    """The frame the GPU encoder must write for `chunk` (host twin)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(chunk), dtype=np.uint8))
    L = _twin_lib()
    out = np.empty(int(L.zstd_twin_bound(a.size)) + 16, dtype=np.uint8)
    n = L.zstd_twin_frame(a.ctypes.data if a.size else None, a.size, out.ctypes.data)
    return out[:n].tobytes()


def libzstd():
    """The image's libzstd.so.1 (decoder of record for the frames; also the CPU
    baseline's level-1 compressor)."""
    global _zstd
    if _zstd is None:
        L = ctypes.CDLL("libzstd.so.1")
        sz, p = ctypes.c_size_t, ctypes.c_void_p
        L.ZSTD_decompress.restype = sz
        L.ZSTD_decompress.argtypes = [p, sz, p, sz]
        L.ZSTD_compress.restype = sz
        L.ZSTD_compress.argtypes = [p, sz, p, sz, ctypes.c_int]
        L.ZSTD_compressBound.restype = sz
        L.ZSTD_compressBound.argtypes = [sz]
        L.ZSTD_isError.restype = ctypes.c_uint
        L.ZSTD_isError.argtypes = [sz]
        L.ZSTD_getErrorName.restype = ctypes.c_char_p
        L.ZSTD_getErrorName.argtypes = [sz]
        L.ZSTD_versionNumber.restype = ctypes.c_uint
        _zstd = L
    return _zstd


def zstd_decompress(frame: bytes, size: int) -> bytes:
    L = libzstd()
    src = np.frombuffer(bytes(frame), dtype=np.uint8)
    dst = np.empty(max(size, 1), dtype=np.uint8)
    r = L.ZSTD_decompress(dst.ctypes.data, dst.size, src.ctypes.data, src.size)
    if L.ZSTD_isError(r):
        raise ValueError(L.ZSTD_getErrorName(r).decode())
    return dst[:r].tobytes()


def blob_compressed(chunk: bytes) -> bytes:
    """DataBlob::encode(chunk, None, true) with the twin's frame in place of libzstd's:
    the compressed blob only if the frame is shorter than the chunk (:153), else the
    uncompressed one; CRC over the payload."""
    import struct
    import zlib

    frame = zstd_twin_frame(chunk)
    if len(frame) < len(chunk):
        return COMPRESSED_BLOB_MAGIC + struct.pack("<I", zlib.crc32(frame)) + frame
    return blob_uncompressed(chunk)


# ---- DataBlob load + decode (the reference's own pin for compressed blobs) ------------
# The reference never compares compressed bytes: tests/blob_writer.rs:35-87
# (verify_test_blob) writes TEST_DATA through DataBlobWriter and checks that the blob
# loads (DataBlob::load_from_reader -> from_raw + verify_crc, data_blob.rs:256-265,
# :268-300, :78-84), reads back through DataBlobReader with 1-, 3- and 64 KiB read buffers
# (a streaming zstd decoder over the payload), and decodes (DataBlob::decode,
# data_blob.rs:196-225: zstd::stream::decode_all of the payload) to TEST_DATA, whose
# SHA-256 is TEST_DIGEST_PLAIN (verify_digest, :335-350).  blob_load_decode restates
# exactly that for the two unencrypted magics; libzstd is the image's (1.4.8).
ENCRYPTED_BLOB_MAGIC = bytes([123, 103, 133, 190, 34, 45, 76, 240])  # file_formats.rs:15
ENCR_COMPR_BLOB_MAGIC = bytes([230, 89, 27, 191, 11, 191, 216, 11])  # file_formats.rs:18


class _ZBuf(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


def zstd_decode_stream(frame: bytes, read_size: int) -> bytes:
    """zstd::stream::read::Decoder as DataBlobReader drives it: the payload decoded into
    an output buffer of `read_size` bytes at a time (ZSTD_decompressStream), until the
    frame ends and the input is consumed."""
    L = libzstd()
    if not hasattr(L, "_dstream_ready"):
        sz, p = ctypes.c_size_t, ctypes.c_void_p
        L.ZSTD_createDCtx.restype = p
        L.ZSTD_createDCtx.argtypes = []
        L.ZSTD_freeDCtx.restype = sz
        L.ZSTD_freeDCtx.argtypes = [p]
        L.ZSTD_decompressStream.restype = sz
        L.ZSTD_decompressStream.argtypes = [p, ctypes.POINTER(_ZBuf), ctypes.POINTER(_ZBuf)]
        L._dstream_ready = True
    src = np.frombuffer(bytes(frame), dtype=np.uint8)
    dst = np.empty(max(read_size, 1), dtype=np.uint8)
    inb = _ZBuf(src.ctypes.data if src.size else None, src.size, 0)
    out = bytearray()
    dctx = L.ZSTD_createDCtx()
    try:
        while True:
            ob = _ZBuf(dst.ctypes.data, read_size, 0)
            r = L.ZSTD_decompressStream(dctx, ctypes.byref(ob), ctypes.byref(inb))
            if L.ZSTD_isError(r):
                raise ValueError(L.ZSTD_getErrorName(r).decode())
            out += dst[:ob.pos].tobytes()
            if r == 0 and inb.pos == inb.size:
                return bytes(out)  # frame complete and flushed, input consumed
            if ob.pos == 0 and inb.pos == inb.size and r != 0:
                raise ValueError("truncated zstd frame")
    finally:
        L.ZSTD_freeDCtx(dctx)


def blob_load_decode(raw: bytes, digest: bytes | None = None, read_sizes=(1, 3, 64 * 1024)) -> bytes:
    """DataBlob::load_from_reader(raw).decode(None, digest) plus DataBlobReader's reads
    (tests/blob_writer.rs:35-68): raises ValueError where the reference bails."""
    import hashlib
    import struct
    import zlib

    raw = bytes(raw)
    if len(raw) < 12:  # from_raw, data_blob.rs:269-271
        raise ValueError(f"blob too small ({len(raw)} bytes).")
    magic = raw[:8]
    if magic in (ENCRYPTED_BLOB_MAGIC, ENCR_COMPR_BLOB_MAGIC):
        raise ValueError("encrypted blob: not produced by this path")
    if magic not in (UNCOMPRESSED_BLOB_MAGIC, COMPRESSED_BLOB_MAGIC):  # from_raw :290-292
        raise ValueError("unable to parse raw blob - wrong magic")
    if struct.unpack("<I", raw[8:12])[0] != zlib.crc32(raw[12:]):  # verify_crc :78-84
        raise ValueError("Data blob has wrong CRC checksum.")
    if magic == UNCOMPRESSED_BLOB_MAGIC:  # decode :201-207
        data = raw[12:]
        reads = [data] * len(read_sizes)
    else:  # decode :208-216 (decode_all) and DataBlobReader's streaming reads
        data = zstd_decode_stream(raw[12:], 1 << 17)
        reads = [zstd_decode_stream(raw[12:], s) for s in read_sizes]
    for s, r in zip(read_sizes, reads):
        if r != data:
            raise ValueError(f"blob data is wrong (read buffer size {s})")
    if digest is not None and hashlib.sha256(data).digest() != bytes(digest):  # verify_digest
        raise ValueError("detected chunk with wrong digest.")
    return data
