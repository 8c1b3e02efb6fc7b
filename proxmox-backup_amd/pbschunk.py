"""Python host mirror of proxmox-backup's chunker interface over the C ABI
(include/pbs_chunker.h, built as proxmox-backup_amd/csrc/libpbschunk.so).

Mirrors, with the same names, argument meaning and error behaviour:
  * ``Chunker(chunk_size_avg)`` / ``Chunker.scan(data) -> int``
      pbs-datastore/src/chunker.rs:75-106 and :112-168.  A non-power-of-two average
      raises (the reference panics: "got unexpected chunk size - not a power of two.").
  * ``ChunkStream(input, chunk_size=None)`` -- iterator of chunks (bytes)
      pbs-client/src/chunk_stream.rs:12-78 (default average 4 MiB, tail emitted at EOF).
  * ``DynamicChunkWriter(sink, chunk_size)`` -- ``write(data) -> consumed`` / ``close()``
      pbs-datastore/src/dynamic_index.rs:397-523, with the digest/compress/index step
      replaced by a callback ``sink(chunk_end_offset, chunk_bytes)``.
  * ``digest_chunks_device(...)`` -- per-chunk SHA-256 on the GPU,
      ``DataChunkBuilder::digest`` (pbs-datastore/src/data_blob.rs:516-536; with a key,
      ``CryptConfig::compute_digest``, pbs-tools/src/crypt_config.rs:79-84).
  * ``DynamicIndexWriter(path)`` -- ``add_chunk(offset, digest)`` / ``close() -> csum``
      pbs-datastore/src/dynamic_index.rs:297-391 (.didx image built by the C library).

The hash scan always runs on the GPU through the HIP library; there is no CPU path.
Loading fails loudly (``ChunkerLibraryError``) when the library is missing and handle
creation fails when no HIP device is visible.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, Iterable, Iterator, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "csrc", "libpbschunk.so")
# (diagnostics only: an A/B against another build of the same library, e.g. a PMC run of
# the previous round's kernels; the product path loads the in-tree build)
if os.environ.get("PBS_LIBPBSCHUNK_AB"):
    LIB_PATH = os.environ["PBS_LIBPBSCHUNK_AB"]

PBS_OK = 0
PBS_ERR_NOT_POW2 = -1
PBS_ERR_NO_DEVICE = -2
PBS_ERR_HIP = -3
PBS_ERR_NOMEM = -4
PBS_ERR_CAPACITY = -5
PBS_ERR_INVALID = -6

GEN_COUNTER, GEN_RANDOM, GEN_VMIMAGE = 0, 1, 2

EXPORTED_SYMBOLS = (
    "pbs_chunker_new", "pbs_chunker_free", "pbs_chunker_scan", "pbs_chunker_find_cuts",
    "pbs_chunker_find_cuts_device", "pbs_chunker_max_cuts", "pbs_chunker_cuts_bound",
    "pbs_chunker_stream_offset",
    "pbs_chunker_chunk_start", "pbs_chunker_reset", "pbs_chunker_set_stream",
    "pbs_chunker_last_error", "pbs_strerror", "pbs_chunker_last_timing",
    "pbs_candidates_host", "pbs_generate_device", "pbs_device_count", "pbs_table_copy", "pbs_build_id",
    "pbs_chunker_candidates_device", "pbs_chunker_resolve_device",
    # include/pbs_digest.h (chunk digests, dynamic index)
    "pbs_digest_chunks_device", "pbs_digest_chunks_async", "pbs_sha256", "pbs_didx_size",
    "pbs_didx_build", "pbs_known_chunks_device", "pbs_pipeline_host", "pbs_chunker_set_cu_count",
    "pbs_digest_chunks_hybrid", "pbs_digest_chunks_host", "pbs_sha256_host_uses_ni",
    # include/pbs_blob.h (blob CRC)
    "pbs_crc32_chunks_device", "pbs_crc32_chunks_async", "pbs_crc32", "pbs_blob_encode_uncompressed",
    "pbs_blob_encode_chunks_device", "pbs_blob_stream_bound", "pbs_zstd_frame_bound",
    "pbs_blob_encode_release", "pbs_digest_hybrid_release", "pbs_debug_arena_allocs",
    "pbs_pipeline_release", "pbs_blob_encode_spans_device", "pbs_upload_stream_host",
)


class ChunkerLibraryError(RuntimeError):
    pass


class ChunkerError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})")


class Timing(ctypes.Structure):
    _fields_ = [
        ("scan_ms", ctypes.c_float), ("exact_ms", ctypes.c_float),
        ("resolve_ms", ctypes.c_float), ("total_ms", ctypes.c_float),
        ("bytes", ctypes.c_uint64), ("suspects", ctypes.c_uint64),
        ("candidates", ctypes.c_uint64), ("cuts", ctypes.c_uint64),
        ("fused", ctypes.c_uint64), ("scan_pass", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class PipelineTiming(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
        ("chunk_ms", ctypes.c_double), ("drain_ms", ctypes.c_double),
        ("bytes", ctypes.c_uint64), ("chunks", ctypes.c_uint64), ("pieces", ctypes.c_uint64),
        ("host_chunks", ctypes.c_uint64), ("host_bytes", ctypes.c_uint64),
        ("host_done_ms", ctypes.c_double), ("host_threads", ctypes.c_int),
        ("gpu_jobs", ctypes.c_uint64), ("gpu_claimed", ctypes.c_uint64), ("queue_launches", ctypes.c_uint64),
        ("gpu_done_ms", ctypes.c_double), ("host_work_ms", ctypes.c_double),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class BlobEncodeTiming(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_double), ("compress_ms", ctypes.c_double),
        ("assemble_ms", ctypes.c_double), ("crc_ms", ctypes.c_double),
        ("bytes_in", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64),
        ("blocks", ctypes.c_uint64), ("compressed_chunks", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class UploadTiming(ctypes.Structure):
    _fields_ = [
        ("pipe", PipelineTiming), ("known_ms", ctypes.c_double), ("encode_ms", ctypes.c_double),
        ("d2h_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
        ("chunk_count", ctypes.c_uint64), ("chunk_reused", ctypes.c_uint64), ("size", ctypes.c_uint64),
        ("size_reused", ctypes.c_uint64), ("size_compressed", ctypes.c_uint64),
        ("compressed_chunks", ctypes.c_uint64), ("blob", BlobEncodeTiming),
    ]

    def as_dict(self) -> dict:
        return {k: (getattr(self, k).as_dict() if k in ("pipe", "blob") else getattr(self, k))
                for k, _ in self._fields_}


class HybridOpts(ctypes.Structure):
    _fields_ = [
        ("host_threads", ctypes.c_int), ("host_min_len", ctypes.c_uint64),
        ("host_mb_s", ctypes.c_double), ("gpu_mb_s", ctypes.c_double),
    ]


class HybridTiming(ctypes.Structure):
    _fields_ = [
        ("total_ms", ctypes.c_double), ("zero_ms", ctypes.c_double),
        ("gpu_ms", ctypes.c_double), ("host_ms", ctypes.c_double),
        ("gpu_chunks", ctypes.c_uint64), ("host_chunks", ctypes.c_uint64),
        ("host_bytes", ctypes.c_uint64), ("zero_chunks", ctypes.c_uint64),
        ("zero_lengths", ctypes.c_uint64), ("threshold", ctypes.c_uint64),
        ("threads", ctypes.c_int),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def lib():
    """Load libpbschunk.so (no fallback: raises if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch wheels bundle their own libamdhip64.so.7; load it first so this library
    # binds to the same HIP runtime instead of a second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ChunkerLibraryError(
            f"{LIB_PATH} not built; run `make -C proxmox-backup_amd/csrc` or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    p, u64, sz, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
    sig = {
        "pbs_chunker_new": ([sz, ctypes.POINTER(i)], p),
        "pbs_chunker_free": ([p], None),
        "pbs_chunker_scan": ([p, p, sz], sz),
        "pbs_chunker_find_cuts": ([p, p, sz, i, p, sz, ctypes.POINTER(sz)], i),
        "pbs_chunker_find_cuts_device": ([p, p, sz, i, p, sz, ctypes.POINTER(sz)], i),
        "pbs_chunker_max_cuts": ([sz], sz),
        "pbs_chunker_cuts_bound": ([p, sz], sz),
        "pbs_chunker_stream_offset": ([p], u64),
        "pbs_chunker_chunk_start": ([p], u64),
        "pbs_chunker_reset": ([p], i),
        "pbs_chunker_set_stream": ([p, p], i),
        "pbs_chunker_last_error": ([p], i),
        "pbs_strerror": ([i], ctypes.c_char_p),
        "pbs_chunker_last_timing": ([p, ctypes.POINTER(Timing)], i),
        "pbs_candidates_host": ([p, sz, sz, p, sz, ctypes.POINTER(sz)], i),
        "pbs_generate_device": ([p, sz, i, u64, u64, p], i),
        "pbs_device_count": ([], i),
        "pbs_table_copy": ([p], i),
        "pbs_build_id": ([], ctypes.c_char_p),
        "pbs_debug_arena_allocs": ([], u64),
        "pbs_chunker_candidates_device": ([p, p, sz, p, sz, u64, p, sz, ctypes.POINTER(sz)], i),
        "pbs_chunker_resolve_device": ([p, p, sz, u64, i, p, sz, ctypes.POINTER(sz)], i),
        "pbs_digest_chunks_device": ([p, sz, u64, p, sz, p, sz, p, p], i),
        "pbs_digest_chunks_async": ([p, sz, u64, p, p, sz, p, sz, p, p], i),
        "pbs_sha256": ([p, sz, p], None),
        "pbs_didx_size": ([sz], sz),
        "pbs_didx_build": ([p, p, sz, p, ctypes.c_int64, p, sz, p], i),
        "pbs_known_chunks_device": ([p, sz, p, sz, p, ctypes.POINTER(sz), p], i),
        "pbs_pipeline_host": ([sz, p, sz, sz, p, sz, i, p, p, p, sz, ctypes.POINTER(sz),
                               ctypes.POINTER(PipelineTiming)], i),
        "pbs_chunker_set_cu_count": ([p, i], i),
        "pbs_digest_chunks_hybrid": ([p, p, sz, u64, p, sz, p, sz, p, ctypes.POINTER(HybridOpts),
                                      ctypes.POINTER(HybridTiming), p], i),
        "pbs_digest_chunks_host": ([p, sz, u64, p, sz, p, sz, p, i], i),
        "pbs_sha256_host_uses_ni": ([], i),
        "pbs_crc32_chunks_device": ([p, sz, u64, p, sz, p, p], i),
        "pbs_crc32_chunks_async": ([p, sz, u64, p, p, sz, p, p], i),
        "pbs_crc32": ([ctypes.c_uint32, p, sz], ctypes.c_uint32),
        "pbs_blob_encode_uncompressed": ([p, sz, ctypes.c_uint32, p, sz], sz),
        "pbs_blob_encode_chunks_device": ([p, sz, u64, p, sz, i, p, sz, p, p, p,
                                           ctypes.POINTER(BlobEncodeTiming), p], i),
        "pbs_blob_encode_spans_device": ([p, sz, u64, p, sz, i, p, sz, p, p, p,
                                          ctypes.POINTER(BlobEncodeTiming), p], i),
        "pbs_upload_stream_host": ([sz, p, sz, sz, p, sz, i, p, sz, i, p, p, p, sz, ctypes.POINTER(sz),
                                    p, sz, p, p, ctypes.POINTER(UploadTiming)], i),
        "pbs_blob_stream_bound": ([p, sz], sz),
        "pbs_zstd_frame_bound": ([sz], sz),
        "pbs_blob_encode_release": ([], None),
        "pbs_digest_hybrid_release": ([], None),
        "pbs_pipeline_release": ([], None),
    }
    for name, (args, res) in sig.items():
        if os.environ.get("PBS_LIBPBSCHUNK_AB") and not hasattr(L, name):
            continue  # (an older build in an A/B run: the symbols it has)
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def strerror(code: int) -> str:
    return lib().pbs_strerror(code).decode()


def device_count() -> int:
    return int(lib().pbs_device_count())


def table() -> np.ndarray:
    t = np.empty(256, dtype=np.uint32)
    lib().pbs_table_copy(t.ctypes.data)
    return t


def build_id() -> str:
    """Digest of the sources the loaded library was built from (pbs_build_id)."""
    return lib().pbs_build_id().decode()


def max_cuts(length: int) -> int:
    return int(lib().pbs_chunker_max_cuts(length))


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def _ptr(a: np.ndarray) -> Optional[int]:
    return a.ctypes.data if a.size else None


class Chunker:
    """`pbs_datastore::Chunker` (chunker.rs:18) backed by the gfx950 kernels."""

    def __init__(self, chunk_size_avg: int):
        L = lib()
        err = ctypes.c_int(0)
        h = L.pbs_chunker_new(int(chunk_size_avg), ctypes.byref(err))
        if not h:
            if err.value == PBS_ERR_NOT_POW2:
                # the reference panics here (chunker.rs:87-89)
                raise ValueError("got unexpected chunk size - not a power of two.")
            raise ChunkerError(err.value, "pbs_chunker_new")
        self._h = ctypes.c_void_p(h)
        self.chunk_size_avg = int(chunk_size_avg)

    def close(self):
        if getattr(self, "_h", None):
            lib().pbs_chunker_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != PBS_OK:
            raise ChunkerError(rc, what)

    def scan(self, data) -> int:
        """chunker.rs:112 -- 0 (no boundary, slice consumed) or the position after the cut."""
        a = _as_u8(data)
        r = lib().pbs_chunker_scan(self._h, _ptr(a), a.size)
        if r == ctypes.c_size_t(-1).value:
            raise ChunkerError(lib().pbs_chunker_last_error(self._h), "pbs_chunker_scan")
        return int(r)

    def cuts_bound(self, length: int) -> int:
        """Output capacity find_cuts needs for ``length`` bytes at this average."""
        return int(lib().pbs_chunker_cuts_bound(self._h, length))

    def _out(self, cap: int) -> np.ndarray:
        # one output array per handle, grown as needed: a fresh multi-MiB array per call
        # would page-fault on every first touch
        buf = getattr(self, "_outbuf", None)
        if buf is None or buf.size < cap:
            buf = self._outbuf = np.empty(cap, dtype=np.uint64)
        return buf

    def find_cuts(self, data, is_final: bool = False) -> np.ndarray:
        """Chunk END offsets (absolute) of every cut decided inside ``data``."""
        a = _as_u8(data)
        cap = self.cuts_bound(a.size)
        out = self._out(cap)
        n = ctypes.c_size_t(0)
        rc = lib().pbs_chunker_find_cuts(self._h, _ptr(a), a.size, int(bool(is_final)),
                                        out.ctypes.data, cap, ctypes.byref(n))
        self._check(rc, "pbs_chunker_find_cuts")
        return out[: n.value].copy()

    def find_cuts_device(self, dev_ptr: int, length: int, is_final: bool = False,
                         out: Optional[np.ndarray] = None) -> np.ndarray:
        """Same over a device (HBM) buffer, e.g. ``tensor.data_ptr()``.  With ``out`` (a
        writeable contiguous uint64 array of at least ``cuts_bound(length)`` entries, ideally
        pinned host memory so the cut list is DMA'd straight into it) the cuts are written
        there and a view of it is returned -- the next call with the same array overwrites
        that view; otherwise a fresh array."""
        cap = self.cuts_bound(length)
        if out is None:
            buf = self._out(cap)
        else:
            if (out.dtype != np.uint64 or not out.flags.c_contiguous or not out.flags.writeable
                    or out.size < cap):
                raise ValueError(f"out must be a writeable contiguous uint64 array of >= {cap} entries")
            buf = out
        n = ctypes.c_size_t(0)
        rc = lib().pbs_chunker_find_cuts_device(self._h, ctypes.c_void_p(dev_ptr), length,
                                               int(bool(is_final)), buf.ctypes.data, cap,
                                               ctypes.byref(n))
        self._check(rc, "pbs_chunker_find_cuts_device")
        return buf[: n.value] if out is not None else buf[: n.value].copy()

    def candidates_device(self, dev_ptr: int, length: int, pre: bytes, base: int,
                          out_dev_ptr: int, cap: int) -> int:
        """Phase A over device bytes [base, base+length) of a stream, given the
        min(base, 63) stream bytes before them (``pre``): sorted absolute candidate
        positions into the device array at ``out_dev_ptr`` (``cap`` u64 entries).
        Returns their number; raises ChunkerError(PBS_ERR_CAPACITY) with
        ``.needed`` set when cap is too small."""
        pre = bytes(pre)
        n = ctypes.c_size_t(0)
        rc = lib().pbs_chunker_candidates_device(
            self._h, ctypes.c_void_p(dev_ptr), length, pre if pre else None, len(pre), base,
            ctypes.c_void_p(out_dev_ptr) if cap else None, cap, ctypes.byref(n))
        if rc == PBS_ERR_CAPACITY:
            e = ChunkerError(rc, "pbs_chunker_candidates_device")
            e.needed = int(n.value)
            raise e
        self._check(rc, "pbs_chunker_candidates_device")
        return int(n.value)

    def resolve_device(self, cand_dev_ptr: int, n: int, end: int, is_final: bool = True) -> np.ndarray:
        """Phase B: cut list of a stream of ``end`` bytes from its complete sorted
        candidate list (device u64 array of ``n`` entries)."""
        cap = self.cuts_bound(end)
        out = np.empty(cap, dtype=np.uint64)
        k = ctypes.c_size_t(0)
        rc = lib().pbs_chunker_resolve_device(self._h, ctypes.c_void_p(cand_dev_ptr), n, end,
                                              int(bool(is_final)), out.ctypes.data, cap,
                                              ctypes.byref(k))
        self._check(rc, "pbs_chunker_resolve_device")
        return out[: k.value].copy()

    def set_stream(self, hip_stream: int):
        self._check(lib().pbs_chunker_set_stream(self._h, ctypes.c_void_p(hip_stream)),
                    "pbs_chunker_set_stream")

    def set_cu_count(self, cus: int):
        self._check(lib().pbs_chunker_set_cu_count(self._h, cus), "pbs_chunker_set_cu_count")

    def reset(self):
        self._check(lib().pbs_chunker_reset(self._h), "pbs_chunker_reset")

    @property
    def stream_offset(self) -> int:
        return int(lib().pbs_chunker_stream_offset(self._h))

    @property
    def chunk_start(self) -> int:
        return int(lib().pbs_chunker_chunk_start(self._h))

    def last_timing(self) -> dict:
        t = Timing()
        self._check(lib().pbs_chunker_last_timing(self._h, ctypes.byref(t)), "last_timing")
        return t.as_dict()


class ChunkStream:
    """pbs-client/src/chunk_stream.rs:12-78: split an iterable of byte pieces into
    dynamic-size chunks (yields ``bytes``); the remainder is emitted at EOF."""

    def __init__(self, input: Iterable, chunk_size: Optional[int] = None):
        self.input = iter(input)
        self.chunker = Chunker(chunk_size if chunk_size is not None else 4 * 1024 * 1024)
        self.buffer = bytearray()
        self.scan_pos = 0
        self.eof = False
        # bytes gathered per device scan: each scan is a host->device round trip, so
        # scanning every small read piece would be latency-bound; the cuts are those of
        # the whole stream either way, only latency changes (0 = scan every piece)
        self.min_scan = 4 * 1024 * 1024

    def __iter__(self) -> Iterator[bytes]:
        return self

    def _pull(self) -> None:
        try:
            self.buffer += bytes(next(self.input))
        except StopIteration:
            self.eof = True

    def __next__(self) -> bytes:
        while True:
            while not self.eof and len(self.buffer) - self.scan_pos < max(self.min_scan, 1):
                self._pull()
            if self.scan_pos < len(self.buffer):
                boundary = self.chunker.scan(memoryview(self.buffer)[self.scan_pos:])
                chunk_size = self.scan_pos + boundary
                if boundary == 0:
                    self.scan_pos = len(self.buffer)
                elif chunk_size <= len(self.buffer):
                    result = bytes(self.buffer[:chunk_size])
                    del self.buffer[:chunk_size]
                    self.scan_pos = 0
                    return result
                else:
                    raise RuntimeError("got unexpected chunk boundary from chunker")
                continue
            self.scan_pos = 0
            if self.buffer:
                result = bytes(self.buffer)
                self.buffer = bytearray()
                return result
            raise StopIteration


class DynamicChunkWriter:
    """dynamic_index.rs:397-523 Write adapter: ``write`` returns the bytes consumed
    (re-submit the rest, as ``write_all`` does); ``close`` flushes the tail.  Each
    finished chunk goes to ``sink(chunk_end_offset, chunk_bytes)``."""

    def __init__(self, sink: Callable[[int, bytes], None], chunk_size: int):
        self.sink = sink
        self.chunker = Chunker(chunk_size)
        self.chunk_offset = 0
        self.last_chunk = 0
        self.chunk_buffer = bytearray()
        self.closed = False
        self.chunk_count = 0

    def _write_chunk_buffer(self):
        if not self.chunk_buffer:
            return
        expected = self.chunk_offset - self.last_chunk
        if expected != len(self.chunk_buffer):
            raise RuntimeError(f"wrong chunk size {expected} != {len(self.chunk_buffer)}")
        self.chunk_count += 1
        self.last_chunk = self.chunk_offset
        self.sink(self.chunk_offset, bytes(self.chunk_buffer))
        self.chunk_buffer = bytearray()

    def write(self, data) -> int:
        mv = memoryview(data).cast("B")
        pos = self.chunker.scan(mv)
        if pos > 0:
            self.chunk_buffer += mv[:pos]
            self.chunk_offset += pos
            self._write_chunk_buffer()
            return pos
        self.chunk_offset += len(mv)
        self.chunk_buffer += mv
        return len(mv)

    def write_all(self, data):
        mv = memoryview(data).cast("B")
        while len(mv):
            k = self.write(mv)
            mv = mv[k:]

    def close(self):
        if self.closed:
            return
        self.closed = True
        self._write_chunk_buffer()


def candidates_host(data, avg: int) -> np.ndarray:
    """Phase-A hook: positions p >= 63 whose window hash passes the cut test (GPU)."""
    a = _as_u8(data)
    cap = max(16, a.size)
    out = np.empty(cap, dtype=np.uint64)
    n = ctypes.c_size_t(0)
    rc = lib().pbs_candidates_host(_ptr(a), a.size, int(avg), out.ctypes.data, cap, ctypes.byref(n))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_candidates_host")
    return out[: n.value].copy()


def generate_device(dev_ptr: int, length: int, kind: int, seed: int, offset: int = 0,
                    hip_stream: int = 0):
    rc = lib().pbs_generate_device(ctypes.c_void_p(dev_ptr), length, kind, seed & (2**64 - 1),
                                   offset, ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_generate_device")


# ---- chunk digests and the dynamic index (include/pbs_digest.h) --------

DIDX_MAGIC = bytes([28, 145, 78, 165, 25, 186, 179, 205])  # file_formats.rs:24
DIDX_HEADER = 4096
DIDX_ENTRY = 40


def sha256(data) -> bytes:
    """Host SHA-256 of the C library (the index checksum's hash)."""
    a = _as_u8(data)
    out = (ctypes.c_uint8 * 32)()
    lib().pbs_sha256(_ptr(a), a.size, out)
    return bytes(out)


def _key_arg(key):
    if key is None:
        return None, 0
    k = bytes(key)
    if len(k) > 64:
        raise ValueError("key longer than PBS_DIGEST_MAX_KEY (64)")
    return ctypes.create_string_buffer(k, len(k) or 1), len(k)


def digest_chunks_device(dev_ptr: int, data_len: int, bounds, base: int = 0, key=None,
                         hip_stream: int = 0) -> np.ndarray:
    """SHA-256 (on the GPU) of every chunk [bounds[i], bounds[i+1]) of the stream whose
    bytes [base, base + data_len) are at device address dev_ptr; (n, 32) uint8 digests.
    ``key``: the crypt config's id_key, appended to every chunk's message."""
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    n = max(0, b.size - 1)
    out = np.empty((n, 32), dtype=np.uint8)
    if n == 0:
        return out
    kb, kl = _key_arg(key)
    rc = lib().pbs_digest_chunks_device(ctypes.c_void_p(dev_ptr), data_len, base, b.ctypes.data, n,
                                        kb, kl, out.ctypes.data, ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_digest_chunks_device")
    return out


def digest_chunks_hybrid(dev_ptr: int, data_len: int, bounds, base: int = 0, key=None,
                         host=None, threads: int = 0, host_min_len: int = 0,
                         host_mb_s: float = 0.0, gpu_mb_s: float = 0.0, hip_stream: int = 0):
    """pbs_digest_chunks_hybrid: the digests of digest_chunks_device with the longest
    chunks hashed on ``threads`` host threads (SHA extensions) and all-zero long chunks
    once per length; ``host`` (optional numpy uint8 array, the same bytes as the device
    range) lets the host threads read them without a copy from HBM.  Returns ((n, 32)
    digests, timing dict)."""
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    n = max(0, b.size - 1)
    out = np.empty((n, 32), dtype=np.uint8)
    t = HybridTiming()
    if n == 0:
        return out, t.as_dict()
    kb, kl = _key_arg(key)
    hp = None
    if host is not None:
        h = _as_u8(host)
        if h.size < data_len:
            raise ValueError("host copy shorter than data_len")
        hp = _ptr(h)
    o = HybridOpts(threads, host_min_len, host_mb_s, gpu_mb_s)
    rc = lib().pbs_digest_chunks_hybrid(ctypes.c_void_p(dev_ptr), hp, data_len, base, b.ctypes.data, n,
                                        kb, kl, out.ctypes.data, ctypes.byref(o), ctypes.byref(t),
                                        ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_digest_chunks_hybrid")
    return out, t.as_dict()


def digest_chunks_host(data, bounds, base: int = 0, key=None, threads: int = 0) -> np.ndarray:
    """SHA-256(chunk || key) of every chunk of a host buffer on host threads (the C
    library's SHA-extension code); (n, 32) uint8 digests."""
    a = _as_u8(data)
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    n = max(0, b.size - 1)
    out = np.empty((n, 32), dtype=np.uint8)
    if n == 0:
        return out
    kb, kl = _key_arg(key)
    rc = lib().pbs_digest_chunks_host(_ptr(a), a.size, base, b.ctypes.data, n, kb, kl, out.ctypes.data,
                                      threads)
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_digest_chunks_host")
    return out


def sha256_host_uses_ni() -> bool:
    return bool(lib().pbs_sha256_host_uses_ni())


def digest_chunks_async(dev_ptr: int, data_len: int, bounds_dev: int, order_dev: int, n: int,
                        digests_dev: int, base: int = 0, key=None, hip_stream: int = 0):
    """Device-only form (all pointers device memory; order_dev may be 0)."""
    kb, kl = _key_arg(key)
    rc = lib().pbs_digest_chunks_async(ctypes.c_void_p(dev_ptr), data_len, base,
                                       ctypes.c_void_p(bounds_dev), ctypes.c_void_p(order_dev or None),
                                       n, kb, kl, ctypes.c_void_p(digests_dev),
                                       ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_digest_chunks_async")


def crc32(data, crc: int = 0) -> int:
    """Host CRC-32 of the C library (crc32fast::Hasher: continue ``crc`` over data)."""
    a = _as_u8(data)
    return int(lib().pbs_crc32(crc, _ptr(a), a.size))


def crc32_chunks_device(dev_ptr: int, data_len: int, bounds, base: int = 0, hip_stream: int = 0) -> np.ndarray:
    """DataBlob::compute_crc (data_blob.rs:70-75) on the GPU for every chunk
    [bounds[i], bounds[i+1]) of the stream whose bytes [base, base + data_len) are at
    device address dev_ptr; uint32 CRCs in chunk order."""
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    n = max(0, b.size - 1)
    out = np.empty(n, dtype=np.uint32)
    if n == 0:
        return out
    rc = lib().pbs_crc32_chunks_device(ctypes.c_void_p(dev_ptr), data_len, base, b.ctypes.data, n,
                                       out.ctypes.data, ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_crc32_chunks_device")
    return out


def blob_encode_chunks_device(dev_ptr: int, data_len: int, bounds, blobs_dev: int, blobs_cap: int,
                              base: int = 0, compress: bool = True, hip_stream: int = 0):
    """pbs_blob_encode_chunks_device: the DataBlob image of every chunk written back to
    back at device address blobs_dev (data_blob.rs:87-176; zstd frames where shorter).
    Returns (offsets (n + 1), crcs (n), compressed flags (n), timing dict)."""
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    n = max(0, b.size - 1)
    offs = np.zeros(n + 1, dtype=np.uint64)
    crcs = np.empty(n, dtype=np.uint32)
    comp = np.empty(n, dtype=np.uint8)
    t = BlobEncodeTiming()
    rc = lib().pbs_blob_encode_chunks_device(ctypes.c_void_p(dev_ptr), data_len, base, b.ctypes.data, n,
                                             1 if compress else 0, ctypes.c_void_p(blobs_dev), blobs_cap,
                                             offs.ctypes.data, crcs.ctypes.data, comp.ctypes.data,
                                             ctypes.byref(t), ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_blob_encode_chunks_device")
    return offs, crcs, comp, t.as_dict()


def blob_encode_spans_device(dev_ptr: int, data_len: int, spans, blobs_dev: int, blobs_cap: int,
                             base: int = 0, compress: bool = True, hip_stream: int = 0):
    """pbs_blob_encode_spans_device: as blob_encode_chunks_device for chunks given as
    (start, end) absolute spans in any order (e.g. an upload's new chunks); blob i is
    written for span i.  Returns (offsets (n + 1), crcs (n), compressed flags (n), timing)."""
    sp = np.ascontiguousarray(np.asarray(spans, dtype=np.uint64).reshape(-1, 2))
    n = sp.shape[0]
    offs = np.zeros(n + 1, dtype=np.uint64)
    crcs = np.empty(n, dtype=np.uint32)
    comp = np.empty(n, dtype=np.uint8)
    t = BlobEncodeTiming()
    rc = lib().pbs_blob_encode_spans_device(ctypes.c_void_p(dev_ptr), data_len, base, sp.ctypes.data, n,
                                            1 if compress else 0, ctypes.c_void_p(blobs_dev), blobs_cap,
                                            offs.ctypes.data, crcs.ctypes.data, comp.ctypes.data,
                                            ctypes.byref(t), ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_blob_encode_spans_device")
    return offs, crcs, comp, t.as_dict()


def debug_arena_allocs() -> int:
    """Device buffers the per-device work areas have allocated so far (tests)."""
    return int(lib().pbs_debug_arena_allocs())


def blob_encode_release() -> None:
    """Free the blob encoder's cached device scratch."""
    lib().pbs_blob_encode_release()


def digest_hybrid_release() -> None:
    """Free the hybrid digest's cached pinned host slices."""
    lib().pbs_digest_hybrid_release()


def pipeline_release() -> None:
    """Free the idle pipeline work areas (pipeline_host keeps the stream-sized device
    buffer between calls)."""
    lib().pbs_pipeline_release()


def blob_stream_bound(bounds) -> int:
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    return int(lib().pbs_blob_stream_bound(b.ctypes.data, max(0, b.size - 1)))


def crc32_chunks_async(dev_ptr: int, data_len: int, bounds_dev: int, order_dev: int, n: int, crcs_dev: int,
                       base: int = 0, hip_stream: int = 0):
    """Device-only form (all pointers device memory; order_dev may be 0)."""
    rc = lib().pbs_crc32_chunks_async(ctypes.c_void_p(dev_ptr), data_len, base, ctypes.c_void_p(bounds_dev),
                                      ctypes.c_void_p(order_dev or None), n, ctypes.c_void_p(crcs_dev),
                                      ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_crc32_chunks_async")


UNCOMPRESSED_BLOB_MAGIC_1_0 = bytes([66, 171, 56, 7, 190, 131, 112, 161])  # file_formats.rs:9


def blob_encode_uncompressed(data, crc: int) -> bytes:
    """DataBlob::encode(data, None, compress=false) (data_blob.rs:159-174) with the CRC
    from crc32_chunks_device: magic || crc LE || data."""
    a = _as_u8(data)
    out = np.empty(a.size + 12, dtype=np.uint8)
    n = lib().pbs_blob_encode_uncompressed(_ptr(a), a.size, crc, out.ctypes.data, out.size)
    if n != a.size + 12:
        raise ValueError(f"data blob too large ({a.size} bytes).")
    return out.tobytes()


def known_chunks_device(digests_dev: int, n: int, known_dev: int, k: int, is_known_dev: int,
                        hip_stream: int = 0) -> int:
    """backup_writer.rs:677-697 on the GPU: is_known[i] = digest i is in the previous
    index (known_dev: k sorted 32-byte digests) or repeats an earlier chunk's digest.
    All pointers device memory; returns the number of known chunks."""
    cnt = ctypes.c_size_t(0)
    rc = lib().pbs_known_chunks_device(ctypes.c_void_p(digests_dev), n, ctypes.c_void_p(known_dev or None),
                                       k, ctypes.c_void_p(is_known_dev), ctypes.byref(cnt),
                                       ctypes.c_void_p(hip_stream))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_known_chunks_device")
    return int(cnt.value)


def didx_build(ends, digests, uuid: bytes = bytes(16), ctime: int = 0):
    """.didx image (bytes) and index_csum of chunks with END offsets ``ends`` and
    32-byte ``digests`` (dynamic_index.rs:28-68 header/entries, :373-391 csum)."""
    e = np.ascontiguousarray(np.asarray(ends, dtype=np.uint64))
    if isinstance(digests, (list, tuple)):
        digests = np.frombuffer(b"".join(bytes(x) for x in digests), dtype=np.uint8)
    d = np.ascontiguousarray(np.asarray(digests, dtype=np.uint8).reshape(-1, 32))
    if d.shape[0] != e.size:
        raise ValueError("ends and digests differ in length")
    if len(uuid) != 16:
        raise ValueError("uuid must be 16 bytes")
    n = e.size
    cap = int(lib().pbs_didx_size(n))
    out = np.empty(cap, dtype=np.uint8)
    csum = (ctypes.c_uint8 * 32)()
    ub = ctypes.create_string_buffer(bytes(uuid), 16)
    rc = lib().pbs_didx_build(e.ctypes.data if n else None, d.ctypes.data if n else None, n, ub,
                              int(ctime), out.ctypes.data, cap, csum)
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_didx_build")
    return out.tobytes(), bytes(csum)


class DynamicIndexWriter:
    """dynamic_index.rs:297-391: ``add_chunk(offset, digest)`` per chunk (offset = the
    chunk's END offset, as DynamicChunkWriter passes it), ``close()`` writes the .didx
    file (tmp file + rename) and returns index_csum.  uuid/ctime default to a random
    uuid and the current time (Uuid::generate / epoch_i64 in the reference)."""

    def __init__(self, path: str, uuid: Optional[bytes] = None, ctime: Optional[int] = None):
        import time

        self.path = path
        self.uuid = bytes(uuid) if uuid is not None else os.urandom(16)
        self.ctime = int(time.time()) if ctime is None else int(ctime)
        self.ends = []
        self.digests = []
        self.closed = False

    def add_chunk(self, offset: int, digest: bytes):
        if self.closed:
            raise RuntimeError(f"cannot write to closed dynamic index file {self.path!r}")
        if len(digest) != 32:
            raise ValueError("digest must be 32 bytes")
        self.ends.append(int(offset))
        self.digests.append(bytes(digest))

    def close(self) -> bytes:
        if self.closed:
            raise RuntimeError(f"cannot close already closed archive index file {self.path!r}")
        self.closed = True
        image, csum = didx_build(self.ends, self.digests, self.uuid, self.ctime)
        tmp = os.path.splitext(self.path)[0] + ".tmp_didx"
        with open(tmp, "wb") as f:
            f.write(image)
        os.replace(tmp, self.path)
        return csum


def read_didx(image: bytes):
    """Parse a .didx image: (uuid, ctime, index_csum, ends (u64), digests (n, 32))."""
    if len(image) < DIDX_HEADER or image[:8] != DIDX_MAGIC:
        raise ValueError("not a dynamic index image")
    body = np.frombuffer(image, dtype=np.uint8, offset=DIDX_HEADER)
    if body.size % DIDX_ENTRY:
        raise ValueError("truncated entry")
    ent = body.reshape(-1, DIDX_ENTRY)
    ends = ent[:, :8].copy().view("<u8").reshape(-1)
    ctime = int.from_bytes(image[24:32], "little", signed=True)
    return image[8:24], ctime, image[32:64], ends, ent[:, 8:].copy()


def index_stream_device(chunker: "Chunker", dev_ptr: int, length: int, key=None,
                        hip_stream: int = 0, uuid: bytes = bytes(16), ctime: int = 0):
    """The client's per-stream path on a device-resident stream: chunk boundaries
    (GPU chunker), chunk digests (the hybrid SHA-256: GPU lanes, the longest chunks on
    host cores), then the .didx image and index_csum (host).  Returns (ends, digests,
    csum, didx_bytes)."""
    start = chunker.stream_offset
    ends = chunker.find_cuts_device(dev_ptr, length, is_final=True)
    bounds = np.concatenate([np.array([start], dtype=np.uint64), ends.astype(np.uint64)])
    dig, _ = digest_chunks_hybrid(dev_ptr, length, bounds, base=start, key=key, hip_stream=hip_stream)
    image, csum = didx_build(ends, dig, uuid, ctime)
    return ends, dig, csum, image


def upload_stream_host(data, avg: int, known=None, key=None, piece: int = 1 << 30,
                       uuid: bytes = bytes(16), ctime: int = 0, compress: bool = True,
                       digest_cus: int = 64, blobs_out=None) -> dict:
    """The client's upload of one dynamic-index stream from a host buffer, up to the
    network (pbs-client/src/backup_writer.rs:631-706 upload_chunk_info_stream; the client
    backs up with compress = true, proxmox-backup-client/src/main.rs:1011-1016): chunk
    (ChunkStream), digest every chunk, mark it known when its digest is in ``known`` (the
    previous index's digests, :524-547) or repeats an earlier chunk of this stream (:697),
    build each new chunk's blob -- DataChunkBuilder::new(data).compress(compress).build()
    (:671, :698; zstd frames where shorter, data_blob.rs:139-176) -- and the .didx image.
    Everything up to the blobs runs on the GPU from one HBM copy of the stream
    (pbs_upload_stream_host).  Returns a dict: ends, digests, known (uint8 mask), csum,
    didx (bytes), blobs (uint8 array: the new chunks' blobs back to back; chunk i's is
    blobs[blob_offsets[i]:blob_offsets[i + 1]], empty for a known chunk), blob_offsets
    (n + 1), compressed (n flags), new_chunks = [(start, length), ...], stats (UploadStats,
    backup_writer.rs:56-64) and timing.
    ``blobs_out``: an optional preallocated uint8 array (e.g. pinned) for the blobs."""
    a = _as_u8(data)
    cap = a.size // max(int(avg) >> 2, 65) + 4
    ends = np.empty(cap, dtype=np.uint64)
    dig = np.empty((cap, 32), dtype=np.uint8)
    is_known = np.empty(cap, dtype=np.uint8)
    offs = np.zeros(cap + 1, dtype=np.uint64)
    comp = np.empty(cap, dtype=np.uint8)
    bcap = 12 * cap + a.size
    blobs = blobs_out if blobs_out is not None else np.empty(max(bcap, 1), dtype=np.uint8)
    if blobs.size < bcap:
        raise ValueError(f"blobs_out holds {blobs.size} bytes, the stream needs up to {bcap}")
    kd = np.zeros((0, 32), dtype=np.uint8)
    if known is not None and len(known):
        kd = np.frombuffer(b"".join(sorted(bytes(x) for x in known)), dtype=np.uint8).reshape(-1, 32)
    kb, kl = _key_arg(key)
    n = ctypes.c_size_t(0)
    t = UploadTiming()
    rc = lib().pbs_upload_stream_host(avg, _ptr(a), a.size, piece, kb, kl, digest_cus,
                                      kd.ctypes.data if kd.size else None, kd.shape[0], 1 if compress else 0,
                                      ends.ctypes.data, dig.ctypes.data, is_known.ctypes.data, cap,
                                      ctypes.byref(n), blobs.ctypes.data, blobs.size, offs.ctypes.data,
                                      comp.ctypes.data, ctypes.byref(t))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_upload_stream_host")
    m = n.value
    ends, dig, is_known, offs, comp = ends[:m].copy(), dig[:m].copy(), is_known[:m].copy(), offs[:m + 1].copy(), comp[:m].copy()
    image, csum = didx_build(ends, dig, uuid, ctime)
    starts = np.concatenate([[0], ends[:-1]]).astype(np.uint64) if m else np.zeros(0, np.uint64)
    new = [(int(starts[i]), int(ends[i] - starts[i])) for i in np.flatnonzero(is_known == 0)]
    td = t.as_dict()
    stats = {k: td[k] for k in ("chunk_count", "chunk_reused", "size", "size_reused", "size_compressed")}
    return {"ends": ends, "digests": dig, "known": is_known, "csum": csum, "didx": image,
            "blobs": blobs[:int(offs[-1])] if m else blobs[:0], "blob_offsets": offs, "compressed": comp,
            "new_chunks": new, "stats": stats, "timing": td}


def pipeline_host(data, avg: int, piece: int = 1 << 30, key=None, digest_cus: int = 64, crc: bool = False):
    """pbs_pipeline_host: chunk END offsets, (n, 32) digests and the timing dict of the
    overlapped copy -> chunk -> digest path over a host buffer; with crc=True also the
    per-chunk blob CRC-32s: (ends, digests, crcs, timing)."""
    a = _as_u8(data)
    # pbs_chunker_cuts_bound without a handle (min_eff = max(avg / 4, 65)); an average
    # that is not a power of two fails in the call below
    cap = a.size // max(int(avg) >> 2, 65) + 4
    ends = np.empty(cap, dtype=np.uint64)
    dig = np.empty((cap, 32), dtype=np.uint8)
    crcs = np.empty(cap, dtype=np.uint32) if crc else None
    n = ctypes.c_size_t(0)
    t = PipelineTiming()
    kb, kl = _key_arg(key)
    rc = lib().pbs_pipeline_host(avg, _ptr(a), a.size, piece, kb, kl, digest_cus, ends.ctypes.data,
                                 dig.ctypes.data, crcs.ctypes.data if crc else None, cap, ctypes.byref(n),
                                 ctypes.byref(t))
    if rc != PBS_OK:
        raise ChunkerError(rc, "pbs_pipeline_host")
    if crc:
        return ends[: n.value].copy(), dig[: n.value].copy(), crcs[: n.value].copy(), t.as_dict()
    return ends[: n.value].copy(), dig[: n.value].copy(), t.as_dict()
