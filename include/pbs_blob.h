/*
 * pbs_blob.h -- C ABI of the per-chunk blob CRC stage (SURVEY.md section 8(f) rank 4:
 * the client-side per-chunk work after the digest).
 *
 * Reference interfaces replaced:
 *  - `DataBlob::compute_crc` (pbs-datastore/src/data_blob.rs:70-75):
 *    crc32fast::Hasher over the blob payload -- the chunk bytes for an uncompressed blob,
 *    set by `DataBlob::encode` (data_blob.rs:87-179; set_crc :64-67) and checked by
 *    `DataBlob::verify_crc` (:78-84) on every load/verify.  crc32fast (Cargo.toml:111,
 *    "1") computes CRC-32/ISO-HDLC: reflected polynomial 0xEDB88320, init and final
 *    XOR 0xFFFFFFFF -- the same function as zlib's crc32.
 *  - the uncompressed blob layout (pbs-datastore/src/file_formats.rs:9 and :36-45):
 *    magic UNCOMPRESSED_BLOB_MAGIC_1_0 (8 bytes) || crc (u32 LE) || data.
 *
 * Chunk i of a stream is [bounds[i], bounds[i+1]) in absolute stream offsets, as in
 * pbs_digest.h.
 */
#ifndef PBS_BLOB_H
#define PBS_BLOB_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBS_BLOB_HEADER_SIZE 12 /* DataBlobHeader: magic[8] + crc[4] */

/* CRC-32 of every chunk on the GPU.  `dev_data` (device) holds stream bytes
 * [base, base + data_len); `bounds` (host, n + 1 ascending absolute offsets); writes n
 * CRCs to host `crcs` (chunk order).  Synchronous.  Returns PBS_OK or PBS_ERR_*. */
int pbs_crc32_chunks_device(const uint8_t *dev_data, size_t data_len, uint64_t base,
                            const uint64_t *bounds, size_t n, uint32_t *crcs, void *hip_stream);

/* Device-only, asynchronous form: `bounds_dev` (n + 1 offsets), `order_dev` (NULL or a
 * permutation of 0..n-1; workgroup k takes chunk order_dev[k] -- longest first balances
 * the tail), `crcs_dev` (n u32) are device memory. */
int pbs_crc32_chunks_async(const uint8_t *dev_data, size_t data_len, uint64_t base,
                           const uint64_t *bounds_dev, const uint32_t *order_dev, size_t n,
                           uint32_t *crcs_dev, void *hip_stream);

/* Host CRC-32 (crc32fast::Hasher::update/finalize): continue `crc` (0 to start) over
 * `data`. */
uint32_t pbs_crc32(uint32_t crc, const uint8_t *data, size_t len);

/* Uncompressed DataBlob image of `data` with its precomputed CRC (from
 * pbs_crc32_chunks_*): magic || crc LE || data into `out` (cap >= len + 12).  Returns
 * the bytes written (len + 12) or 0 if `cap` is too small or len exceeds MAX_BLOB_SIZE
 * (128 MiB, data_blob.rs:13 / :92). */
size_t pbs_blob_encode_uncompressed(const uint8_t *data, size_t len, uint32_t crc, uint8_t *out,
                                    size_t cap);

/* DataBlob images of every chunk on the GPU (`DataBlob::encode(data, None, compress)`,
 * data_blob.rs:87-176, unencrypted path).  compress != 0: each chunk is compressed into a
 * zstd frame (64 KiB blocks: RLE, compressed -- Huffman, raw or RLE literals; sequences
 * with repeat offsets and predefined, RLE or own FSE tables -- or raw; the match window
 * reaches 16 KiB before each 8 KiB sub-block; decodable by any zstd decoder, the reference's
 * `zstd::stream::decode_all` :214 included -- but not byte-identical to libzstd level 1,
 * which is what the reference writes: "parity unpinned"); the blob
 * is {COMPRESSED_BLOB_MAGIC_1_0, CRC, frame} when the frame is shorter than the chunk
 * (:153), else {UNCOMPRESSED_BLOB_MAGIC_1_0, CRC, chunk}.  compress == 0: every blob
 * uncompressed.  CRC = crc32fast over the payload (compute_crc, :70-75).
 * `dev_data` (device) holds stream bytes [base, base + data_len); `bounds` (host, n + 1
 * ascending absolute offsets; every chunk <= 128 MiB, MAX_BLOB_SIZE :13/:92).  The blobs
 * are written back to back into `blobs_dev` (device, blobs_cap >= pbs_blob_stream_bound);
 * blob i is [blob_offsets[i], blob_offsets[i+1]) (host, n + 1); `crcs` (host, n) and
 * `compressed` (host, n: 1 = zstd) may be NULL.  Needs ~ (bytes of the chunks) of device
 * scratch, kept between calls until pbs_blob_encode_release.  Synchronous.  C ABI of include/pbs_chunker.h's codes. */
typedef struct {
    double total_ms;    /* call entry .. outputs on the host */
    double compress_ms; /* block compression + frame sizes + offset scans (HIP events) */
    double assemble_ms; /* blocks / chunk bytes into the blob images */
    double crc_ms;      /* payload CRCs + headers */
    uint64_t bytes_in, bytes_out, blocks, compressed_chunks;
} pbs_blob_encode_timing;
int pbs_blob_encode_chunks_device(const uint8_t *dev_data, size_t data_len, uint64_t base,
                                  const uint64_t *bounds, size_t n, int compress, uint8_t *blobs_dev,
                                  size_t blobs_cap, uint64_t *blob_offsets, uint32_t *crcs,
                                  uint8_t *compressed, pbs_blob_encode_timing *timing,
                                  void *hip_stream);
/* The same for chunks given as spans: chunk i = [spans[2i], spans[2i+1]) (host, absolute
 * offsets in any order, gaps allowed -- e.g. the new chunks of an upload stream). */
int pbs_blob_encode_spans_device(const uint8_t *dev_data, size_t data_len, uint64_t base,
                                 const uint64_t *spans, size_t n, int compress, uint8_t *blobs_dev,
                                 size_t blobs_cap, uint64_t *blob_offsets, uint32_t *crcs,
                                 uint8_t *compressed, pbs_blob_encode_timing *timing,
                                 void *hip_stream);
/* Frees the device scratch pbs_blob_encode_chunks_device keeps between calls. */
void pbs_blob_encode_release(void);
/* 12 n + (bounds[n] - bounds[0]): the largest blob stream of n chunks. */
size_t pbs_blob_stream_bound(const uint64_t *bounds, size_t n);
/* Largest zstd frame this encoder writes for `len` bytes (header + raw blocks). */
size_t pbs_zstd_frame_bound(size_t len);

#ifdef __cplusplus
}
#endif

#endif /* PBS_BLOB_H */
