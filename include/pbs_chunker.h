/*
 * pbs_chunker.h -- C ABI of the MI355X (gfx950) content-defined chunker.
 *
 * Drop-in boundary for proxmox-backup's `pbs_datastore::Chunker`
 * (pbs-datastore/src/chunker.rs, re-exported at pbs-datastore/src/lib.rs:177,199).
 * Every entry point names the reference interface it replaces.  The Rust binding a
 * maintainer would add (extern "C" block + a `Chunker` newtype keeping the
 * reference's `new`/`scan` signatures) is in INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Offsets are absolute stream offsets (u64).
 *  - A handle is single-owner, not thread-safe (the reference's `&mut self`,
 *    chunker.rs:112); distinct handles may be used concurrently, one HIP stream each.
 *  - The hash scan runs on the GPU; a handle cannot be created without a HIP device
 *    (pbs_chunker_new fails with PBS_ERR_NO_DEVICE).  There is no CPU fallback.
 *  - Cut offsets are chunk END offsets (exclusive), i.e. the cut byte + 1, the same
 *    quantity as `chunk_offset` after `DynamicChunkWriter::write`
 *    (pbs-datastore/src/dynamic_index.rs:497-500).
 */
#ifndef PBS_CHUNKER_H
#define PBS_CHUNKER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (negative) */
#define PBS_OK 0
#define PBS_ERR_NOT_POW2 (-1)   /* chunker.rs:87-89 panics: "not a power of two" */
#define PBS_ERR_NO_DEVICE (-2)  /* no HIP device visible */
#define PBS_ERR_HIP (-3)        /* a HIP runtime call or kernel launch failed */
#define PBS_ERR_NOMEM (-4)      /* host or device allocation failed */
#define PBS_ERR_CAPACITY (-5)   /* output array too small; nothing was consumed */
#define PBS_ERR_INVALID (-6)    /* bad argument (NULL handle, NULL data with len > 0) */

typedef struct pbs_chunker pbs_chunker;

/* Replaces `Chunker::new(chunk_size_avg: usize) -> Chunker` (chunker.rs:75-106).
 * Thresholds: min = avg >> 2, max = avg << 2, mask = (2*avg - 1) as u32,
 * minimum = mask - 2 (chunker.rs:91-105).  Returns NULL and *err = PBS_ERR_NOT_POW2
 * where the reference panics (avg not a power of two), PBS_ERR_NO_DEVICE without a
 * GPU.  `err` may be NULL. */
pbs_chunker *pbs_chunker_new(size_t chunk_size_avg, int *err);

/* Drop for `Chunker` (no explicit destructor in the reference). */
void pbs_chunker_free(pbs_chunker *c);

/* Replaces `Chunker::scan(&mut self, data: &[u8]) -> usize` (chunker.rs:112-168).
 * Same contract: returns 0 if `data` holds no chunk boundary (the whole slice is
 * consumed into the state), else the position just after the cut byte, relative to
 * `data`.  The caller re-submits the unconsumed remainder starting at that position
 * (pbs-client/src/chunk_stream.rs:44-54); bytes already scanned are not rescanned
 * (their candidates are cached by absolute offset).  The reference's `scan` is
 * infallible; on a device error this returns SIZE_MAX and pbs_chunker_last_error()
 * tells why (the Rust shim turns that into a panic). */
size_t pbs_chunker_scan(pbs_chunker *c, const uint8_t *data, size_t len);

/* Batch form of repeated `scan` calls over a host buffer (the loop of
 * examples/test_chunk_speed.rs:25-36 and of ChunkStream::poll_next).  `data` starts at
 * the first unconsumed stream byte.  Writes the END offsets of every cut decided
 * inside `data` to `out` (ascending) and their number to *n_out.  With is_final != 0
 * the tail chunk's end (the stream length) is appended if the tail is non-empty, as
 * ChunkStream does at EOF (chunk_stream.rs:64-68), and the handle starts a new
 * stream.  `cap` must be >= pbs_chunker_cuts_bound(c, len) (else PBS_ERR_CAPACITY and
 * no state change).  Returns PBS_OK or an error code. */
int pbs_chunker_find_cuts(pbs_chunker *c, const uint8_t *data, size_t len, int is_final,
                          uint64_t *out, size_t cap, size_t *n_out);

/* Same as pbs_chunker_find_cuts with `dev_data` a device pointer (HBM-resident
 * input, e.g. a torch tensor's data_ptr()); `out` is a host array.  When `out` is pinned
 * or registered host memory the GPU writes long cut lists into it directly (no staging
 * copy, one sync per call); any host array works.  Entries past *n_out are unspecified. */
int pbs_chunker_find_cuts_device(pbs_chunker *c, const uint8_t *dev_data, size_t len,
                                 int is_final, uint64_t *out, size_t cap, size_t *n_out);

/* Upper bound of the cuts one find_cuts call over `len` bytes can return, for any
 * average (every chunk but the tail is >= 65 bytes long). */
size_t pbs_chunker_max_cuts(size_t len);

/* The same bound for this handle's average: every chunk that starts and ends inside
 * the call is >= max(avg/4, 65) bytes long (chunker.rs:172-183), so len/that + 3. */
size_t pbs_chunker_cuts_bound(const pbs_chunker *c, size_t len);

/* Absolute offset of the next unconsumed byte and of the open chunk's start. */
uint64_t pbs_chunker_stream_offset(const pbs_chunker *c);
uint64_t pbs_chunker_chunk_start(const pbs_chunker *c);

/* Start a new stream with the same average (what `Chunker::new` would give). */
int pbs_chunker_reset(pbs_chunker *c);

/* Run the handle's kernels on this hipStream_t (NULL = the handle's own stream).  The
 * handle's own stream is non-blocking: it does not wait for work on the null stream or
 * any other stream, so device input written there (find_cuts_device, the sharded entry
 * points) must be complete before the call -- synchronize, or set the producing stream
 * here (what bench.py and the tests do with torch's current stream). */
int pbs_chunker_set_stream(pbs_chunker *c, void *hip_stream);

/* Number of CUs the persistent scan kernel sizes its grid for (default: all of the
 * device); set it to the CU count of a CU-masked stream given to set_stream. */
int pbs_chunker_set_cu_count(pbs_chunker *c, int cus);

/* Error of the last failed call on this handle, and a message for any code. */
int pbs_chunker_last_error(const pbs_chunker *c);
const char *pbs_strerror(int code);

/* Timing of the last find_cuts / scan device pass (HIP events on the handle's stream). */
typedef struct {
    float scan_ms;      /* main candidate kernel (scan_fused_kernel / scan_main_kernel) */
    float exact_ms;     /* exact block re-evaluation + candidate sort */
    float resolve_ms;   /* min/max resolve over the candidate list */
    float total_ms;     /* first kernel start .. cut list on the host */
    uint64_t bytes;     /* bytes scanned by the pass */
    uint64_t suspects;  /* 128-byte blocks flagged by the main kernel */
    uint64_t candidates;
    uint64_t cuts;
    uint64_t fused;     /* bytes chunked by scan_fused_kernel: the one-launch pass or the scan pass */
    uint64_t scan_pass; /* of those, bytes through the scan pass (no resolver waves; gather +
                         * multi-kernel resolve after it: 64/128 KiB averages) */
} pbs_timing;
int pbs_chunker_last_timing(const pbs_chunker *c, pbs_timing *t);

/* ---- one stream sharded over several GPUs ------------
 * The cut test is a pure function of the 64-byte window (chunker.rs:146: rotl by 64 is
 * the identity), so contiguous ranges of one stream are scanned independently given
 * the 63 bytes before each range (a halo exchanged between neighbours); the sorted
 * per-range candidate lists concatenate into the stream's list (one all-gather), and
 * the min/max rule (chunker.rs:172-183) is resolved once over it. */

/* Phase A over the device range holding stream bytes [base, base + len): every
 * position p in it with p >= 63 whose window hash passes the cut test, ascending and
 * absolute, to `out_dev` (device memory, cap entries).  `pre` holds the
 * pre_len = min(base, 63) stream bytes before `base` (host memory).  *n_out receives
 * the number of candidates, also when it exceeds cap (then PBS_ERR_CAPACITY and
 * nothing is written).  Complete on return; the handle's stream state is untouched. */
int pbs_chunker_candidates_device(pbs_chunker *c, const uint8_t *dev, size_t len,
                                  const uint8_t *pre, size_t pre_len, uint64_t base,
                                  uint64_t *out_dev, size_t cap, size_t *n_out);

/* Phase B: the cut list (chunk END offsets, host `out`, cap >= cuts_bound(c, end))
 * of a stream of `end` bytes from its complete sorted candidate list (device, n
 * entries, all < end), from the stream start; is_final appends the tail like
 * find_cuts.  Restarts the handle's stream (before and after).  last_timing keeps
 * the phase-A fields of the preceding candidates_device call. */
int pbs_chunker_resolve_device(pbs_chunker *c, const uint64_t *cand_dev, size_t n, uint64_t end,
                               int is_final, uint64_t *out, size_t cap, size_t *n_out);

/* ---- helpers for tests and the benchmark harness ------------------------------ */

/* Phase-A hook: every position p (>= 63) of a host buffer whose window hash passes
 * the cut test for `avg` (chunker.rs:185), computed on the GPU; ascending. */
int pbs_candidates_host(const uint8_t *data, size_t len, size_t avg, uint64_t *out, size_t cap,
                        size_t *n_out);

/* Fill a device buffer with a synthetic stream (kind 0 = LE-u32 counter
 * (examples/test_chunk_speed.rs:8-14), 1 = splitmix64 random, 2 = VM-image-like).
 * `len` and `offset` must be multiples of 8. */
int pbs_generate_device(uint8_t *dev, size_t len, int kind, uint64_t seed, uint64_t offset,
                        void *hip_stream);

/* Number of visible HIP devices (0 without a GPU). */
int pbs_device_count(void);

/* Copy of the library's Buzhash table (256 entries), for the digest check. */
int pbs_table_copy(uint32_t *out256);

/* Digest (16 hex digits) of the sources this library was built from (csrc/ and
 * include/); bench.py reports a PMC traffic record only when it was measured on the
 * same build. */
const char *pbs_build_id(void);

/* Device buffers the library's per-device work areas have allocated so far (blob
 * encoding, digests, CRCs, the known-chunk test reuse theirs across calls: a repeated call
 * of the same size allocates nothing). */
uint64_t pbs_debug_arena_allocs(void);

#ifdef __cplusplus
}
#endif
#endif /* PBS_CHUNKER_H */
