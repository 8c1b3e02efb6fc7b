/*
 * Replays, call for call through the C ABI, what the Rust shim rust/chunker_gpu.rs does
 * (a Rust toolchain is not in the image, so the shim itself is never compiled here):
 *
 *   stream <avg> <len> <seed> <read>
 *       Chunker::new(avg) -> pbs_chunker_new; ChunkStream::poll_next
 *       (pbs-client/src/chunk_stream.rs:40-77) over reads of <read> bytes, each
 *       Chunker::scan -> pbs_chunker_scan on buffer[scan_pos..]; Drop -> pbs_chunker_free.
 *       Prints "ends <chunk end offsets...>" (the EOF tail included, :64-68).
 *   badavg
 *       Chunker::new(1000) -> NULL, err PBS_ERR_NOT_POW2 -> the reference's panic text
 *       (chunker.rs:87-89). Prints "panic: <message>".
 *   failed-scan <avg> <len>
 *       A handle whose device wait overran its bound (run with PBS_HOST_WAIT_MS tiny: a
 *       pbs_chunker_find_cuts of <len> host bytes gives up on the kernel) -> the next
 *       Chunker::scan gets SIZE_MAX -> pbs_chunker_last_error -> pbs_strerror -> the
 *       shim's panic message -> Drop -> pbs_chunker_free (which must return). Then a
 *       fresh handle, and the old one after pbs_chunker_reset, chunk again.
 *       Prints "find_cuts <rc>", "panic: <message>", "reset <rc>", "ends ..." lines.
 *   kernel-timeout <avg> <len>
 *       PBS_FUSED_TIMEOUT_TICKS=0 in the environment: the fused pass's resolver fails at
 *       once (status 2) -> pbs_chunker_find_cuts returns PBS_ERR_HIP; the handle is not
 *       lost: scan() still works. Prints "find_cuts <rc> <last_error>", "ends ...".
 *
 * Input: splitmix64 random bytes (oracle.gen_random(len, seed)); failed-scan and
 * kernel-timeout: oracle.gen_random(4 MiB, 7), then zeros up to <len>.
 */
#define _DEFAULT_SOURCE /* usleep */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "pbs_chunker.h"

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint8_t *gen(size_t len, uint64_t seed) {
    uint8_t *d = malloc(len ? len : 1);
    if (!d) exit(3);
    for (size_t x = 0; x < len; ++x) d[x] = (uint8_t)(splitmix64(seed ^ (x >> 3)) >> ((x & 7) * 8));
    return d;
}

/* the shim's Chunker::new: NULL + message where it panics */
static pbs_chunker *shim_new(size_t avg, char *panic_msg, size_t cap) {
    int err = 0;
    pbs_chunker *h = pbs_chunker_new(avg, &err);
    if (!h) {
        if (err == PBS_ERR_NOT_POW2)
            snprintf(panic_msg, cap, "got unexpected chunk size - not a power of two.");
        else
            snprintf(panic_msg, cap, "GPU chunker unavailable: %s", pbs_strerror(err));
    }
    return h;
}

/* the shim's Chunker::scan: 0 + message where it panics */
static int shim_scan(pbs_chunker *h, const uint8_t *data, size_t len, size_t *out, char *panic_msg, size_t cap) {
    const size_t r = pbs_chunker_scan(h, data, len);
    if (r == SIZE_MAX) {
        const int code = pbs_chunker_last_error(h);
        snprintf(panic_msg, cap, "GPU chunker failed: %s", pbs_strerror(code));
        return 0;
    }
    *out = r;
    return 1;
}

/* ChunkStream::poll_next until the input ends; prints the chunk ends; 0 on a panic */
static int chunk_stream(pbs_chunker *h, const uint8_t *data, size_t len, size_t read, char *msg, size_t cap) {
    size_t buf_lo = 0, buf_hi = 0, scan_pos = 0, off = 0, emitted = 0;
    printf("ends");
    for (;;) {
        if (scan_pos < buf_hi - buf_lo) {
            size_t boundary = 0;
            if (!shim_scan(h, data + buf_lo + scan_pos, buf_hi - buf_lo - scan_pos, &boundary, msg, cap)) {
                printf("\n");
                return 0;
            }
            const size_t chunk_size = scan_pos + boundary;
            if (boundary == 0) {
                scan_pos = buf_hi - buf_lo;
            } else if (chunk_size <= buf_hi - buf_lo) {
                buf_lo += chunk_size;
                emitted += chunk_size;
                printf(" %zu", emitted);
                scan_pos = 0;
                continue;
            } else {
                snprintf(msg, cap, "got unexpected chunk boundary from chunker");
                printf("\n");
                return 0;
            }
        }
        if (off >= len) {  /* input ended: the tail is the last chunk */
            scan_pos = 0;
            if (buf_hi > buf_lo) printf(" %zu", emitted + (buf_hi - buf_lo));
            printf("\n");
            return 1;
        }
        const size_t n = len - off < read ? len - off : read;
        off += n;
        buf_hi += n; /* the buffer is a window [buf_lo, buf_hi) of `data` */
    }
}

int main(int argc, char **argv) {
    char msg[256] = "";
    if (argc >= 2 && !strcmp(argv[1], "badavg")) {
        pbs_chunker *h = shim_new(1000, msg, sizeof msg);
        if (h) {
            pbs_chunker_free(h);
            return 1;
        }
        printf("panic: %s\n", msg);
        return 0;
    }
    if (argc == 6 && !strcmp(argv[1], "stream")) {
        const size_t avg = strtoull(argv[2], NULL, 0), len = strtoull(argv[3], NULL, 0);
        const size_t read = strtoull(argv[5], NULL, 0);
        uint8_t *data = gen(len, strtoull(argv[4], NULL, 0));
        pbs_chunker *h = shim_new(avg, msg, sizeof msg);
        if (!h) {
            printf("panic: %s\n", msg);
            return 1;
        }
        const int ok = chunk_stream(h, data, len, read, msg, sizeof msg);
        if (!ok) printf("panic: %s\n", msg);
        pbs_chunker_free(h);
        free(data);
        return ok ? 0 : 1;
    }
    if (argc == 4 && (!strcmp(argv[1], "failed-scan") || !strcmp(argv[1], "kernel-timeout"))) {
        const int lost = !strcmp(argv[1], "failed-scan");
        const size_t avg = strtoull(argv[2], NULL, 0), len = strtoull(argv[3], NULL, 0);
        /* random in the first 4 MiB (the chunk_stream checks), zeros after (a long pass) */
        const size_t head = len < (4u << 20) ? len : (4u << 20);
        uint8_t *data = calloc(len ? len : 1, 1), *rnd = gen(head, 7);
        if (!data) return 3;
        memcpy(data, rnd, head);
        free(rnd);
        pbs_chunker *h = shim_new(avg, msg, sizeof msg);
        if (!h) {
            printf("panic: %s\n", msg);
            return 1;
        }
        const size_t cap = pbs_chunker_cuts_bound(h, len);
        uint64_t *out = malloc(cap * sizeof *out);
        size_t n = 0;
        const int rc = pbs_chunker_find_cuts(h, data, len, 1, out, cap, &n);
        printf("find_cuts %d %d\n", rc, pbs_chunker_last_error(h));
        if (lost) {
            /* the shim's next scan() panics; its Drop frees the handle */
            size_t r = 0;
            if (shim_scan(h, data, 8192, &r, msg, sizeof msg)) {
                printf("scan did not fail: %zu\n", r);
                return 1;
            }
            printf("panic: %s\n", msg);
            printf("reset-while-lost %d\n", pbs_chunker_reset(h)); /* may still run: either way no hang */
            usleep(500 * 1000);                                   /* the overrun kernel retires */
            printf("reset %d\n", pbs_chunker_reset(h));
            if (!chunk_stream(h, data, head, 65536, msg, sizeof msg))
                printf("panic: %s\n", msg);
            pbs_chunker_free(h);
            /* a fresh handle on the same device */
            h = shim_new(avg, msg, sizeof msg);
            if (!h) {
                printf("panic: %s\n", msg);
                return 1;
            }
        } else {
            pbs_chunker_reset(h);
        }
        const int ok = chunk_stream(h, data, head, 65536, msg, sizeof msg);
        if (!ok) printf("panic: %s\n", msg);
        pbs_chunker_free(h);
        free(out);
        free(data);
        printf("freed\n");
        return ok ? 0 : 1;
    }
    fprintf(stderr, "usage: %s stream avg len seed read | badavg | failed-scan avg len | kernel-timeout avg len\n",
            argv[0]);
    return 2;
}
