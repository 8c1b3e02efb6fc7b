/*
 * oracle/chunker_oracle.c -- CPU restatement of proxmox-backup's content-defined
 * chunker, used ONLY as test infrastructure (the checker in tests/, smoke() and the
 * cpu_baseline leg of bench.py).  Nothing in the product library links or calls this
 * file; the product path is the HIP kernels in proxmox-backup_amd/csrc/.
 *
 * Reference followed (read as text; the Rust reference cannot be built here, no
 * cargo/rustc in the image, see DESIGN.md "Parity"):
 *   pbs-datastore/src/chunker.rs:6        CA_CHUNKER_WINDOW_SIZE = 64
 *   pbs-datastore/src/chunker.rs:18-33    struct Chunker state
 *   pbs-datastore/src/chunker.rs:35-68    BUZHASH_TABLE (oracle/buzhash_table_oracle.h)
 *   pbs-datastore/src/chunker.rs:75-106   Chunker::new (thresholds, power-of-two panic)
 *   pbs-datastore/src/chunker.rs:112-168  Chunker::scan (fill phase, roll loop, reset)
 *   pbs-datastore/src/chunker.rs:172-186  Chunker::shall_break
 *   pbs-datastore/src/chunker.rs:202-271  test_chunker1 (feed-granularity invariance)
 *
 * Besides the streaming restatement (ora_new / ora_scan) this file holds:
 *   - ora_chunk_feed: the caller loop of test_chunker1 / ChunkStream
 *     (pbs-client/src/chunk_stream.rs:40-77) for a given feed granularity;
 *   - ora_window_hash / ora_candidates / ora_resolve: the two-phase restatement
 *     (properties 1 and 4) that the GPU design relies on;
 *   - the synthetic stream generators shared by tests and bench (DESIGN.md "Inputs").
 *
 * Rust `usize` arithmetic is restated with uint64_t; `u32` with uint32_t and
 * wrapping semantics (release build) where the reference would wrap.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include "buzhash_table_oracle.h"

#define ORA_WINDOW 64u

typedef struct {
    uint32_t h;
    uint64_t window_size;
    uint64_t chunk_size;
    uint64_t chunk_size_min;
    uint64_t chunk_size_max;
    uint64_t chunk_size_avg;
    uint32_t discriminator; /* computed, unused (chunker.rs:84-85, 101) */
    uint32_t break_test_mask;
    uint32_t break_test_minimum;
    uint8_t window[ORA_WINDOW];
} ora_chunker;

static inline uint32_t rotl32(uint32_t x, unsigned r) {
    r &= 31u;
    return r ? (x << r) | (x >> (32u - r)) : x;
}

uint64_t ora_sizeof_chunker(void) { return sizeof(ora_chunker); }

/* chunker.rs:75-106.  Returns 0 on success, -1 where the reference panics
 * ("got unexpected chunk size - not a power of two."). */
int ora_new(ora_chunker *c, uint64_t chunk_size_avg) {
    double avg = (double)chunk_size_avg;
    uint32_t discriminator = (uint32_t)(avg / (-1.42888852e-7 * avg + 1.33237515));
    if (__builtin_popcountll(chunk_size_avg) != 1) return -1;
    uint32_t break_test_mask = (uint32_t)(chunk_size_avg * 2 - 1);   /* `as u32` truncates */
    uint32_t break_test_minimum = break_test_mask - 2u;                /* wraps for avg == 1 */
    memset(c, 0, sizeof(*c));
    c->chunk_size_min = chunk_size_avg >> 2;
    c->chunk_size_max = chunk_size_avg << 2;
    c->chunk_size_avg = chunk_size_avg;
    c->discriminator = discriminator;
    c->break_test_mask = break_test_mask;
    c->break_test_minimum = break_test_minimum;
    return 0;
}

/* chunker.rs:172-186 */
static inline int ora_shall_break(const ora_chunker *c) {
    if (c->chunk_size >= c->chunk_size_max) return 1;
    if (c->chunk_size < c->chunk_size_min) return 0;
    return (c->h & c->break_test_mask) >= c->break_test_minimum;
}

/* chunker.rs:112-168: returns 0 (no boundary, whole slice consumed into state) or
 * the position just after the cut byte, relative to `data`. */
uint64_t ora_scan(ora_chunker *c, const uint8_t *data, uint64_t data_len) {
    const uint64_t window_len = ORA_WINDOW;
    uint64_t pos = 0;

    if (c->window_size < window_len) {
        uint64_t need = window_len - c->window_size;
        uint64_t copy_len = need < data_len ? need : data_len;
        for (uint64_t i = 0; i < copy_len; i++) {
            uint8_t byte = data[pos];
            c->window[c->window_size] = byte;
            c->h = rotl32(c->h, 1) ^ ORACLE_BUZHASH_TABLE[byte];
            pos += 1;
            c->window_size += 1;
        }
        c->chunk_size += copy_len;
        if (c->window_size < window_len) return 0;
    }

    uint64_t idx = c->chunk_size & 0x3f;
    while (pos < data_len) {
        uint8_t enter = data[pos];
        uint8_t leave = c->window[idx];
        c->h = rotl32(c->h, 1) ^ ORACLE_BUZHASH_TABLE[leave] ^ ORACLE_BUZHASH_TABLE[enter];
        c->chunk_size += 1;
        pos += 1;
        c->window[idx] = enter;
        if (ora_shall_break(c)) {
            c->h = 0;
            c->chunk_size = 0;
            c->window_size = 0;
            return pos;
        }
        idx = c->chunk_size & 0x3f;
    }
    return 0;
}

/*
 * Caller loop in the style of test_chunker1 (chunker.rs:214-226) and ChunkStream
 * (chunk_stream.rs:40-77): the stream arrives in pieces of `feed` bytes (feed == 0:
 * one piece = the whole buffer).  Within a piece the unconsumed remainder is
 * re-submitted after every cut.  Writes the absolute chunk END offsets (exclusive)
 * of every cut; the tail [last, len) is not a cut.  Returns the number of cuts, or
 * -1 for a non-power-of-two avg, -2 if `cap` is too small.
 */
int64_t ora_chunk_feed(uint64_t avg, const uint8_t *data, uint64_t len, uint64_t feed,
                       uint64_t *out_ends, uint64_t cap) {
    ora_chunker c;
    if (ora_new(&c, avg) != 0) return -1;
    if (feed == 0) feed = len ? len : 1;
    uint64_t n = 0;
    for (uint64_t piece = 0; piece < len; piece += feed) {
        uint64_t plen = len - piece < feed ? len - piece : feed;
        uint64_t off = 0;
        while (off < plen) {
            uint64_t k = ora_scan(&c, data + piece + off, plen - off);
            if (k == 0) break;
            off += k;
            if (n >= cap) return -2;
            out_ends[n++] = piece + off;
        }
    }
    return (int64_t)n;
}

/* SURVEY.md section 0 property 1: once the window is full, h at stream byte p is
 * H(p) = XOR_{k=0..63} rotl(T[b[p-k]], k mod 32).  Direct 64-term evaluation. */
uint32_t ora_window_hash(const uint8_t *data, uint64_t p) {
    uint32_t h = 0;
    for (unsigned k = 0; k < ORA_WINDOW; k++)
        h ^= rotl32(ORACLE_BUZHASH_TABLE[data[p - k]], k & 31u);
    return h;
}

/* Phase A restated: every p >= 63 whose full-window hash satisfies the
 * shall_break hash test (chunker.rs:185).  Returns count or -2 on overflow. */
int64_t ora_candidates(uint64_t avg, const uint8_t *data, uint64_t len, uint64_t *out,
                       uint64_t cap) {
    ora_chunker c;
    if (ora_new(&c, avg) != 0) return -1;
    uint64_t n = 0;
    uint32_t h = 0;
    for (uint64_t p = 0; p < len; p++) {
        h = rotl32(h, 1) ^ ORACLE_BUZHASH_TABLE[data[p]];
        if (p >= ORA_WINDOW) h ^= ORACLE_BUZHASH_TABLE[data[p - ORA_WINDOW]];
        if (p + 1 >= ORA_WINDOW && (h & c.break_test_mask) >= c.break_test_minimum) {
            if (n >= cap) return -2;
            out[n++] = p;
        }
    }
    return (int64_t)n;
}

/*
 * Phase B restated (SURVEY.md section 0 property 4): from chunk start s, the next cut
 * is the first candidate c in [s + max(min,65) - 1, s + max(max,65) - 1], else the
 * forced cut at s + max(max,65) - 1.  Writes chunk END offsets (c + 1), the tail is
 * not a cut.  Candidates must be sorted ascending.
 */
int64_t ora_resolve(uint64_t avg, const uint64_t *cand, uint64_t m, uint64_t len,
                    uint64_t *out_ends, uint64_t cap) {
    ora_chunker c;
    if (ora_new(&c, avg) != 0) return -1;
    const uint64_t min_eff = c.chunk_size_min > 65 ? c.chunk_size_min : 65;
    const uint64_t max_eff = c.chunk_size_max > 65 ? c.chunk_size_max : 65;
    uint64_t s = 0, i = 0, n = 0;
    for (;;) {
        uint64_t lo = s + min_eff - 1, hi = s + max_eff - 1;
        while (i < m && cand[i] < lo) i++;
        uint64_t cut;
        if (i < m && cand[i] <= hi) cut = cand[i];
        else if (hi < len) cut = hi;
        else break;
        if (cut >= len) break;
        if (n >= cap) return -2;
        out_ends[n++] = cut + 1;
        s = cut + 1;
    }
    return (int64_t)n;
}

/* ------------------------------------------------------------------------------
 * Synthetic input generators (DESIGN.md "Inputs"); byte x of a stream is a pure
 * function of (seed, x), so host, numpy and device generators agree bytewise.
 * ---------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t ora_splitmix64(uint64_t x) { return splitmix64(x); }

/* test_chunk_speed.rs:8-14: byte[4i+j] = (i >> 8j) & 0xff (LE u32 counter). */
void ora_gen_counter(uint8_t *buf, uint64_t len, uint64_t offset) {
    for (uint64_t k = 0; k < len; k++) {
        uint64_t x = offset + k;
        buf[k] = (uint8_t)(((uint32_t)(x >> 2)) >> ((x & 3) * 8));
    }
}

/* random: byte x = LE byte (x & 7) of splitmix64(seed ^ (x >> 3)). */
void ora_gen_random(uint8_t *buf, uint64_t len, uint64_t seed, uint64_t offset) {
    for (uint64_t k = 0; k < len; k++) {
        uint64_t x = offset + k;
        buf[k] = (uint8_t)(splitmix64(seed ^ (x >> 3)) >> ((x & 7) * 8));
    }
}

#define VM_SEED_PAGE 0x7A65726F50414745ull
#define VM_SEED_WORD 0x52414E44574F5244ull
#define VM_SEED_EXT 0x4558544E54000000ull

/* VM-image-like: one forced all-zero 64 MiB extent per GiB (slot chosen by seed),
 * else 4 KiB pages all-zero with probability 40 %, else random words. */
static inline uint8_t vm_byte(uint64_t seed, uint64_t x) {
    uint64_t g = x >> 30;
    uint64_t ext = (splitmix64(seed ^ VM_SEED_EXT ^ g) & 15u) << 26;
    uint64_t in_g = x & ((1ull << 30) - 1);
    if (in_g >= ext && in_g < ext + (1ull << 26)) return 0;
    if (splitmix64(seed ^ VM_SEED_PAGE ^ (x >> 12)) % 100u < 40u) return 0;
    return (uint8_t)(splitmix64(seed ^ VM_SEED_WORD ^ (x >> 3)) >> ((x & 7) * 8));
}

void ora_gen_vmimage(uint8_t *buf, uint64_t len, uint64_t seed, uint64_t offset) {
    for (uint64_t k = 0; k < len; k++) buf[k] = vm_byte(seed, offset + k);
}

/* The same bytes as ora_gen_{counter,random,vmimage} (kind 0/1/2), a word at a time
 * where the range is 8-byte aligned (one splitmix64 per word instead of per byte;
 * tests/test_oracle.py checks the two agree), for the long streams of
 * tests/golden/make_bench_golden.py. */
static void gen_block(int kind, uint64_t seed, uint8_t *buf, uint64_t len, uint64_t off) {
    if (kind == 0) { ora_gen_counter(buf, len, off); return; }
    uint64_t k = 0;
    for (; k < len && ((off + k) & 7u); k++)
        buf[k] = kind == 1 ? (uint8_t)(splitmix64(seed ^ ((off + k) >> 3)) >> (((off + k) & 7) * 8))
                           : vm_byte(seed, off + k);
    uint64_t page = ~0ull;  /* VM image: the zero decision is made once per 4 KiB page */
    int zero = 0;
    for (; k + 8 <= len; k += 8) {
        uint64_t x = off + k, w;
        if (kind == 1) {
            w = splitmix64(seed ^ (x >> 3));
        } else {
            if ((x >> 12) != page) {
                page = x >> 12;
                uint64_t g = x >> 30, ext = (splitmix64(seed ^ VM_SEED_EXT ^ g) & 15u) << 26;
                uint64_t in_g = x & ((1ull << 30) - 1);
                zero = (in_g >= ext && in_g < ext + (1ull << 26)) ||
                       splitmix64(seed ^ VM_SEED_PAGE ^ page) % 100u < 40u;
            }
            w = zero ? 0 : splitmix64(seed ^ VM_SEED_WORD ^ (x >> 3));
        }
        memcpy(buf + k, &w, 8);  /* little-endian host */
    }
    for (; k < len; k++)
        buf[k] = kind == 1 ? (uint8_t)(splitmix64(seed ^ ((off + k) >> 3)) >> (((off + k) & 7) * 8))
                           : vm_byte(seed, off + k);
}

void ora_gen_block(int kind, uint64_t seed, uint8_t *buf, uint64_t len, uint64_t off) {
    gen_block(kind, seed, buf, len, off);
}

/*
 * The cut list of a whole generated stream (kind 0 counter, 1 random, 2 VM image; `len`
 * bytes from offset 0) as the reference computes it: the stream is generated `piece`
 * bytes at a time and fed through the caller loop of ChunkStream::poll_next
 * (chunk_stream.rs:40-77) around ora_scan (chunker.rs:112-168), so no stream has to
 * fit in memory.  Writes the absolute chunk END offsets, and at EOF the stream end when
 * the tail is non-empty (chunk_stream.rs:64-68) -- the list find_cuts(..., is_final)
 * returns.  Returns the count, -1 for a bad average, -2 if `cap` is too small, -3 when
 * out of memory.
 */
int64_t ora_chunk_generated(int kind, uint64_t seed, uint64_t avg, uint64_t len, uint64_t piece,
                            uint64_t *out, uint64_t cap) {
    ora_chunker c;
    if (ora_new(&c, avg) != 0) return -1;
    if (piece == 0) piece = 16ull << 20;
    uint8_t *buf = (uint8_t *)malloc(piece);
    if (!buf) return -3;
    uint64_t n = 0;
    for (uint64_t base = 0; base < len; base += piece) {
        uint64_t plen = len - base < piece ? len - base : piece;
        gen_block(kind, seed, buf, plen, base);
        uint64_t off = 0;
        while (off < plen) {
            uint64_t k = ora_scan(&c, buf + off, plen - off);
            if (k == 0) break;
            off += k;
            if (n >= cap) { free(buf); return -2; }
            out[n++] = base + off;
        }
    }
    free(buf);
    if (len > 0 && (n == 0 || out[n - 1] != len)) {
        if (n >= cap) return -2;
        out[n++] = len;
    }
    return (int64_t)n;
}

/* The compiler and flags this library was built with (bench.py's cpu_baseline records them
 * beside its rates: a CPU baseline is only comparable across runs with the same build). */
#ifndef ORA_CFLAGS
#define ORA_CFLAGS "(unknown)"
#endif
const char *ora_build_info(void) { return "cc " __VERSION__ "; flags " ORA_CFLAGS; }
