/*
 * pbs_digest.h -- C ABI of the per-chunk SHA-256 stage and the dynamic index image
 * (the consumers right after the chunker).
 *
 * Reference interfaces replaced:
 *  - chunk digest: `DataChunkBuilder::digest` / `compute_digest`
 *    (pbs-datastore/src/data_blob.rs:516-536): `openssl::sha::sha256(data)`, or with a
 *    crypt config `CryptConfig::compute_digest` (pbs-tools/src/crypt_config.rs:79-84):
 *    SHA-256(data || id_key).  Called per chunk by the client upload stream
 *    (pbs-client/src/backup_writer.rs:671-678) and by `DynamicChunkWriter`
 *    (pbs-datastore/src/dynamic_index.rs:463-466).
 *  - index: `DynamicIndexWriter::create` / `add_chunk` / `close`
 *    (pbs-datastore/src/dynamic_index.rs:297-391): a 4096-byte header (magic
 *    DYNAMIC_SIZED_CHUNK_INDEX_1_0, pbs-datastore/src/file_formats.rs:24, uuid, ctime,
 *    index_csum) followed by 40-byte entries {end_le: u64, digest: [u8; 32]}
 *    (dynamic_index.rs:28-68); index_csum = SHA-256(end1_le || digest1 || ...)
 *    (dynamic_index.rs:373-391, and the client's own csum, backup_writer.rs:683-688).
 *
 * Chunk i of a stream is [bounds[i], bounds[i+1]) in absolute stream offsets; with the
 * chunker's cut list `ends` (pbs_chunker_find_cuts*), bounds = {start, ends...}.
 */
#ifndef PBS_DIGEST_H
#define PBS_DIGEST_H

#include <stddef.h>
#include <stdint.h>

#include "pbs_blob.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PBS_DIGEST_MAX_KEY 64 /* id_key is 32 bytes in the reference */

/* SHA-256 of every chunk on the GPU.  `dev_data` (device) holds stream bytes
 * [base, base + data_len); every chunk must lie inside it.  `bounds` (host, n + 1
 * ascending absolute offsets), `key` (host, key_len <= PBS_DIGEST_MAX_KEY bytes
 * appended to every chunk's message; NULL/0 for the plain digest).  Writes 32 * n
 * digest bytes to host `digests` (chunk order).  Synchronous.  Returns PBS_OK or a
 * PBS_ERR_* code (pbs_chunker.h). */
int pbs_digest_chunks_device(const uint8_t *dev_data, size_t data_len, uint64_t base,
                             const uint64_t *bounds, size_t n, const uint8_t *key,
                             size_t key_len, uint8_t *digests, void *hip_stream);

/* Device-only, asynchronous form for pipelines and the benchmark: `bounds_dev`
 * (n + 1 offsets), `order_dev` (NULL or a permutation of 0..n-1: lane k hashes chunk
 * order_dev[k]; pass the chunks sorted by length, longest first, so that the 64 lanes
 * of a wave finish together), `digests_dev` (32 * n bytes) are device memory; `key`
 * is host memory (copied into the launch). */
int pbs_digest_chunks_async(const uint8_t *dev_data, size_t data_len, uint64_t base,
                            const uint64_t *bounds_dev, const uint32_t *order_dev, size_t n,
                            const uint8_t *key, size_t key_len, uint8_t *digests_dev,
                            void *hip_stream);

/* Hybrid per-chunk SHA-256: same digests as pbs_digest_chunks_device, with the work
 * split between the GPU and host threads.  A GPU lane walks one chunk's serial chain
 * (~35 MB/s), so the longest chunks set the GPU's makespan; a host core with the SHA
 * extensions walks one ~70x faster (~120x with four chunks in step per thread).  The
 * longest chunks go to host threads until the host's estimated time (their bytes /
 * (threads x host_mb_s), at most 50 GB/s when they are copied from HBM: whole chunks, back
 * to back on two streams, into a pinned ring kept between calls) meets the GPU's (the
 * longest remaining chunk / gpu_mb_s);
 * long chunks (>= 1 MiB) that are all zero bytes are hashed once per distinct length.
 * `dev_data` (device) holds stream bytes [base, base + data_len); `host_data` (NULL or a
 * host copy of the same bytes) lets the host threads read the bytes directly instead of
 * copying their chunks from HBM.  `bounds` (host, n + 1), `digests` (host, 32 n) as in
 * pbs_digest_chunks_device.  `opts` may be NULL (defaults).  Synchronous. */
typedef struct {
    int host_threads;      /* 0: min(hardware threads, 16); < 0: GPU only */
    uint64_t host_min_len; /* 0: cost model; else chunks at least this long go to the host */
    double host_mb_s;      /* per-thread host SHA-256 rate for the model (0: 4000 with the SHA
                            * extensions, 250 without) */
    double gpu_mb_s;       /* one GPU lane's chain rate for the model (0: 35) */
} pbs_digest_hybrid_opts;
typedef struct {
    double total_ms; /* call entry .. digests in `digests` */
    double zero_ms;  /* plan: sort + zero test of the long chunks (one sync) */
    double gpu_ms;   /* the GPU share's kernel, HIP events */
    double host_ms;  /* the host share, all threads joined */
    uint64_t gpu_chunks, host_chunks, host_bytes, zero_chunks, zero_lengths;
    uint64_t threshold; /* shortest chunk given to the host (0: none) */
    int threads;
} pbs_digest_hybrid_timing;
int pbs_digest_chunks_hybrid(const uint8_t *dev_data, const uint8_t *host_data, size_t data_len,
                             uint64_t base, const uint64_t *bounds, size_t n, const uint8_t *key,
                             size_t key_len, uint8_t *digests, const pbs_digest_hybrid_opts *opts,
                             pbs_digest_hybrid_timing *timing, void *hip_stream);

/* Frees the pinned host memory (ring, slices) the hybrid digest keeps between calls. */
void pbs_digest_hybrid_release(void);

/* SHA-256(chunk || key) of every chunk of a host buffer on `threads` host threads (0:
 * hardware threads), SHA extensions when the CPU has them (pbs_sha256_host_uses_ni).
 * Same arguments as pbs_digest_chunks_device with host memory. */
int pbs_digest_chunks_host(const uint8_t *host_data, size_t data_len, uint64_t base,
                           const uint64_t *bounds, size_t n, const uint8_t *key, size_t key_len,
                           uint8_t *digests, int threads);
int pbs_sha256_host_uses_ni(void);

/* Known-chunk test of the upload stream (pbs-client/src/backup_writer.rs:677-697):
 * chunk i is "known" -- uploaded as a reference, not as data -- iff its digest is in the
 * previous backup's index (`known_chunks`, filled from the downloaded index,
 * backup_writer.rs:524-547) or equals the digest of an earlier chunk of this stream
 * (the reference inserts every new digest into the same set, :697).  `digests_dev` (32 n
 * bytes) and `known_dev` (32 k bytes, sorted ascending as byte strings, duplicates
 * allowed) are device memory; writes is_known_dev[i] = 0/1 (device, n bytes).
 * Synchronous on `hip_stream`; *n_known (host, may be NULL) receives the count. */
int pbs_known_chunks_device(const uint8_t *digests_dev, size_t n, const uint8_t *known_dev,
                            size_t k, uint8_t *is_known_dev, size_t *n_known, void *hip_stream);

/* Client upload path on a host-resident stream (ChunkStream
 * pbs-client/src/chunk_stream.rs:40-77 + the per-chunk digest of the upload stream,
 * backup_writer.rs:671-678): a copy thread moves `host` (pageable, `len` bytes) to HBM
 * in `piece`-byte pieces; the chunker cuts every resident piece on CUs
 * [digest_cus, n) and the chunks each piece completes are digested on CU-masked
 * streams over CUs [0, digest_cus) while the next pieces copy.  Writes the chunk END
 * offsets (`ends`, the tail included) and their 32-byte digests (SHA-256(chunk || key))
 * in chunk order, and with `crcs` != NULL each chunk's CRC-32 (the uncompressed blob's
 * DataBlob::compute_crc, include/pbs_blob.h; computed right after each digest launch on
 * the same stream); cap >= pbs_chunker_cuts_bound for the average.  Needs `len` bytes of
 * device memory, kept in the device's pipeline work area between calls (freed by
 * pbs_pipeline_release).  Each chunk is routed when the chunker completes it: to a
 * persistent GPU digest grid when its serial hash (len / PBS_PIPE_GPU_MBS, default 15 MB/s)
 * ends before the copy's projected end + PBS_PIPE_SLACK_MS (default 10), else to
 * PBS_PIPE_HOST_THREADS host threads (default min(hardware threads, 16) - 2, up to four
 * chunks in step each) straight from `host`; PBS_PIPE_HOST_MIN=<bytes> instead sends chunks of at least that length to the
 * host and the rest to the GPU.  Synchronous. */
typedef struct {
    double total_ms; /* first copy issued .. digests on the host */
    double h2d_ms;   /* copy thread: all pieces issued and landed */
    double chunk_ms; /* main thread inside the chunker calls */
    double drain_ms; /* last piece chunked .. digests on the host */
    uint64_t bytes, chunks, pieces;
    uint64_t host_chunks, host_bytes; /* digests computed on the host threads */
    double host_done_ms;              /* host threads joined (ms after the first copy) */
    int host_threads;
    uint64_t gpu_jobs;                /* chunks routed to the GPU's digest queue */
    uint64_t gpu_claimed;             /* of those, taken by the queue's workgroups (the rest:
                                       * hashed on the host at the end) */
    uint64_t queue_launches;          /* launches of the queue grid (it exits when idle) */
    double gpu_done_ms;               /* the digest queue and the CRC launches finished */
    double host_work_ms;              /* the host threads' last digest finished */
} pbs_pipeline_timing;
int pbs_pipeline_host(size_t avg, const uint8_t *host, size_t len, size_t piece,
                      const uint8_t *key, size_t key_len, int digest_cus, uint64_t *ends,
                      uint8_t *digests, uint32_t *crcs, size_t cap, size_t *n_out,
                      pbs_pipeline_timing *timing);

/* The client's upload of one dynamic-index stream up to the network
 * (pbs-client/src/backup_writer.rs:631-706, upload_chunk_info_stream, with
 * proxmox-backup-client's `compress: true`, main.rs:1011-1016): pbs_pipeline_host's chunks
 * and digests, then on the GPU from the same HBM copy the known-chunk test
 * (pbs_known_chunks_device: `known`, 32 n_known bytes sorted ascending = the previous
 * index's digests, :524-547; and repeats of earlier chunks of this stream, :697) and the
 * blob of every new chunk, `DataChunkBuilder::new(data).compress(compress).build()`
 * (:671, :698; DataBlob::encode, pbs-datastore/src/data_blob.rs:139-176 -- the zstd frame
 * of include/pbs_blob.h, parity of its bytes unpinned).  Writes `ends`, `digests`,
 * `is_known` (n bytes), the blobs back to back into `blobs` (host, blobs_cap >= 12 n +
 * len suffices) with chunk i's blob at [blob_offsets[i], blob_offsets[i+1]) (n + 1
 * entries; a known chunk's blob is empty -- it is uploaded as a reference) and
 * `compressed` (n bytes, may be NULL).  Timing: the pipeline's, the stages after it, and
 * the reference's UploadStats (backup_writer.rs:56-64; size_compressed = the new blobs'
 * raw sizes, :699).  Synchronous. */
typedef struct {
    pbs_pipeline_timing pipe; /* chunks + digests */
    double known_ms;          /* digests H2D + known-chunk test + flags D2H */
    double encode_ms;         /* blob encoding of the new chunks (GPU, HBM -> HBM) */
    double d2h_ms;            /* blobs to the host buffer */
    double total_ms;          /* call entry .. everything on the host */
    uint64_t chunk_count, chunk_reused, size, size_reused, size_compressed;
    uint64_t compressed_chunks; /* new chunks stored as zstd blobs */
    pbs_blob_encode_timing blob;
} pbs_upload_timing;
int pbs_upload_stream_host(size_t avg, const uint8_t *host, size_t len, size_t piece,
                           const uint8_t *key, size_t key_len, int digest_cus, const uint8_t *known,
                           size_t n_known, int compress, uint64_t *ends, uint8_t *digests,
                           uint8_t *is_known, size_t cap, size_t *n_out, uint8_t *blobs,
                           size_t blobs_cap, uint64_t *blob_offsets, uint8_t *compressed,
                           pbs_upload_timing *timing);

/* Frees the idle pipeline work areas (device memory of the last stream lengths). */
void pbs_pipeline_release(void);

/* Host SHA-256 (FIPS 180-4), used for the index checksum (the reference's
 * openssl::sha::Sha256 over 40-byte entries; a few hundred KiB per index). */
void pbs_sha256(const uint8_t *data, size_t len, uint8_t out[32]);

/* Size in bytes of a dynamic index image with n entries: 4096 + 40 n. */
size_t pbs_didx_size(size_t n);

/* Build the .didx image of n chunks (`ends`: chunk end offsets, `digests`: 32 n bytes)
 * into `out` (cap >= pbs_didx_size(n)): header {magic, uuid[16], ctime (LE i64),
 * index_csum, zeros}, then the entries.  `csum_out` (may be NULL) receives index_csum,
 * what `DynamicIndexWriter::close` returns. */
int pbs_didx_build(const uint64_t *ends, const uint8_t *digests, size_t n, const uint8_t uuid[16],
                   int64_t ctime, uint8_t *out, size_t cap, uint8_t csum_out[32]);

#ifdef __cplusplus
}
#endif

#endif /* PBS_DIGEST_H */
