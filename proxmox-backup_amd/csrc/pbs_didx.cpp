// Host side of SURVEY.md 8(f) rank 3: the dynamic index (.didx) image and its checksum.
// Format (pbs-datastore/src/dynamic_index.rs):
//   header (4096 bytes, :28-37): magic [u8; 8] = DYNAMIC_SIZED_CHUNK_INDEX_1_0
//       (file_formats.rs:24), uuid [u8; 16], ctime i64 LE, index_csum [u8; 32],
//       reserved zeros;
//   entries (:61-66): {end_le: u64 LE, digest: [u8; 32]} per chunk, in stream order;
//   index_csum = SHA-256(end1_le || digest1 || end2_le || ...)  (add_chunk :373-391,
//       written into the header by close :347-370).
// The SHA-256 here is a plain FIPS 180-4 host implementation: the checksum covers 40
// bytes per chunk (a few hundred KiB per index), the reference computes it on the host
// too (openssl::sha::Sha256).
#include <stdint.h>

#include <cstring>

#include "pbs_chunker.h"
#include "pbs_digest.h"

namespace {

constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

// DYNAMIC_SIZED_CHUNK_INDEX_1_0 (pbs-datastore/src/file_formats.rs:24)
constexpr uint8_t kDidxMagic[8] = {28, 145, 78, 165, 25, 186, 179, 205};
constexpr size_t kHeader = 4096;
constexpr size_t kEntry = 40;

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Sha256 {
    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint8_t buf[64];
    size_t fill = 0;
    uint64_t total = 0;

    void block(const uint8_t* p) {
        uint32_t w[64];
        for (int t = 0; t < 16; ++t)
            w[t] = (uint32_t)p[4 * t] << 24 | (uint32_t)p[4 * t + 1] << 16 |
                   (uint32_t)p[4 * t + 2] << 8 | p[4 * t + 3];
        for (int t = 16; t < 64; ++t) {
            const uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
            const uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
            w[t] = w[t - 16] + s0 + w[t - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int t = 0; t < 64; ++t) {
            const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) +
                                kK[t] + w[t];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g;
            g = f;
            f = e;
            e = d + t1;
            d = c;
            c = b;
            b = a;
            a = t1 + t2;
        }
        h[0] += a;
        h[1] += b;
        h[2] += c;
        h[3] += d;
        h[4] += e;
        h[5] += f;
        h[6] += g;
        h[7] += hh;
    }
    void update(const uint8_t* p, size_t n) {
        total += n;
        if (fill) {
            const size_t k = n < 64 - fill ? n : 64 - fill;
            std::memcpy(buf + fill, p, k);
            fill += k;
            p += k;
            n -= k;
            if (fill == 64) {
                block(buf);
                fill = 0;
            }
        }
        for (; n >= 64; p += 64, n -= 64) block(p);
        if (n) {
            std::memcpy(buf, p, n);
            fill = n;
        }
    }
    void finish(uint8_t out[32]) {
        const uint64_t bits = total * 8;
        const uint8_t pad = 0x80;
        update(&pad, 1);
        const uint8_t zero[64] = {0};
        update(zero, (fill <= 56 ? 56 - fill : 120 - fill));
        uint8_t len[8];
        for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(len, 8);
        for (int i = 0; i < 8; ++i) {
            out[4 * i] = (uint8_t)(h[i] >> 24);
            out[4 * i + 1] = (uint8_t)(h[i] >> 16);
            out[4 * i + 2] = (uint8_t)(h[i] >> 8);
            out[4 * i + 3] = (uint8_t)h[i];
        }
    }
};

inline void put_le64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

}  // namespace

extern "C" void pbs_sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
    Sha256 s;
    if (len) s.update(data, len);
    s.finish(out);
}

extern "C" size_t pbs_didx_size(size_t n) { return kHeader + kEntry * n; }

extern "C" int pbs_didx_build(const uint64_t* ends, const uint8_t* digests, size_t n,
                              const uint8_t uuid[16], int64_t ctime, uint8_t* out, size_t cap,
                              uint8_t csum_out[32]) {
    if (!out || (n && (!ends || !digests))) return PBS_ERR_INVALID;
    if (cap < pbs_didx_size(n)) return PBS_ERR_CAPACITY;
    std::memset(out, 0, kHeader);
    std::memcpy(out, kDidxMagic, 8);              // magic
    if (uuid) std::memcpy(out + 8, uuid, 16);     // uuid
    put_le64(out + 24, (uint64_t)ctime);          // ctime (i64 LE)
    Sha256 csum;                                  // index_csum at offset 32
    uint8_t* e = out + kHeader;
    for (size_t i = 0; i < n; ++i, e += kEntry) {
        put_le64(e, ends[i]);
        std::memcpy(e + 8, digests + 32 * i, 32);
        csum.update(e, kEntry);
    }
    uint8_t c[32];
    csum.finish(c);
    std::memcpy(out + 32, c, 32);
    if (csum_out) std::memcpy(csum_out, c, 32);
    return PBS_OK;
}
