// Host SHA-256 for the per-chunk digest's long chunks.
//
// The reference hashes every chunk on the host (data_blob.rs:516-536,
// openssl::sha::sha256, SHA-256(chunk || id_key) with a crypt config,
// crypt_config.rs:79-84).  On the GPU one lane walks one chunk's serial chain at
// ~34 MB/s, so a handful of 16 MiB chunks sets the digest stage's makespan (DESIGN.md
// section 10); an x86 core with the SHA extensions walks a chain ~50x faster.  The
// hybrid digest (pbs_digest.hip) therefore gives the longest chunks to host threads
// running this code and the rest to the GPU.
//
// A thread hashes up to four chunks in step (sha256_host_lanes): one message's rounds wait
// on each sha256rnds2's latency, four messages' rounds overlap.
//
// Block function: the SHA-NI form (sha256rnds2 does two rounds on the ABEF/CDGH state
// halves; sha256msg1/msg2 + one alignr extend the schedule four words at a time), with a
// runtime CPUID check and the portable FIPS 180-4 rounds as the fallback.  Padding and
// the appended key follow FIPS 180-4 section 5.1.1 over message = chunk || key.
#include <cpuid.h>
#include <immintrin.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "pbs_chunker.h"
#include "pbs_digest.h"
#include "sha_host.h"

namespace {

alignas(16) constexpr uint32_t kK[64] = {
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

constexpr uint32_t kInit[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                               0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void blocks_portable(uint32_t h[8], const uint8_t* p, size_t nb) {
    for (; nb; --nb, p += 64) {
        uint32_t w[64];
        for (int t = 0; t < 16; ++t)
            w[t] = (uint32_t)p[4 * t] << 24 | (uint32_t)p[4 * t + 1] << 16 | (uint32_t)p[4 * t + 2] << 8 |
                   p[4 * t + 3];
        for (int t = 16; t < 64; ++t)
            w[t] = w[t - 16] + (rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3)) + w[t - 7] +
                   (rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10));
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int t = 0; t < 64; ++t) {
            const uint32_t t1 =
                hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kK[t] + w[t];
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
        h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += hh;
    }
}

// Four schedule words per step: quad q = W[4q .. 4q+3] (+K) feeds two sha256rnds2.  N
// independent messages advance together: one message's chain waits on each sha256rnds2's
// latency, N of them overlap (sha256_host_lanes below).
template <int N>
__attribute__((target("sha,sse4.1,ssse3"), always_inline)) inline void blocks_ni_n(uint32_t* const* h,
                                                                                 const uint8_t* const* pin,
                                                                                 size_t nb) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
    __m128i s0[N], s1[N];
    const uint8_t* p[N];
#pragma GCC unroll 4
    for (int j = 0; j < N; ++j) {
        // state words {a,b,c,d},{e,f,g,h} -> ABEF / CDGH lane order of sha256rnds2
        const __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)h[j]), 0xB1);  // C D A B
        const __m128i e = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)(h[j] + 4)), 0x1B);  // E F G H
        s0[j] = _mm_alignr_epi8(t, e, 8);   // A B E F
        s1[j] = _mm_blend_epi16(e, t, 0xF0);  // C D G H
        p[j] = pin[j];
    }
    for (; nb; --nb) {
        __m128i save0[N], save1[N], m[N][4];
#pragma GCC unroll 4
        for (int j = 0; j < N; ++j) save0[j] = s0[j], save1[j] = s1[j];
#pragma GCC unroll 16
        for (int q = 0; q < 16; ++q) {
#pragma GCC unroll 4
            for (int j = 0; j < N; ++j) {
                __m128i& x = m[j][q & 3];
                if (q < 4) {
                    x = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p[j] + 16 * q)), bswap);
                } else {
                    // W[t] = W[t-16] + s0(W[t-15]) + W[t-7] + s1(W[t-2])
                    const __m128i w7 = _mm_alignr_epi8(m[j][(q - 1) & 3], m[j][(q - 2) & 3], 4);
                    x = _mm_sha256msg2_epu32(_mm_add_epi32(_mm_sha256msg1_epu32(x, m[j][(q - 3) & 3]), w7),
                                             m[j][(q - 1) & 3]);
                }
                const __m128i wk = _mm_add_epi32(x, _mm_load_si128((const __m128i*)(kK + 4 * q)));
                s1[j] = _mm_sha256rnds2_epu32(s1[j], s0[j], wk);
                s0[j] = _mm_sha256rnds2_epu32(s0[j], s1[j], _mm_shuffle_epi32(wk, 0x0E));
            }
        }
#pragma GCC unroll 4
        for (int j = 0; j < N; ++j) {
            s0[j] = _mm_add_epi32(s0[j], save0[j]);
            s1[j] = _mm_add_epi32(s1[j], save1[j]);
            p[j] += 64;
        }
    }
#pragma GCC unroll 4
    for (int j = 0; j < N; ++j) {
        const __m128i t = _mm_shuffle_epi32(s0[j], 0x1B);  // F E B A
        const __m128i u = _mm_shuffle_epi32(s1[j], 0xB1);  // D C H G
        _mm_storeu_si128((__m128i*)h[j], _mm_blend_epi16(t, u, 0xF0));     // D C B A
        _mm_storeu_si128((__m128i*)(h[j] + 4), _mm_alignr_epi8(u, t, 8));  // H G F E
    }
}

__attribute__((target("sha,sse4.1,ssse3"))) void blocks_ni(uint32_t h[8], const uint8_t* p, size_t nb) {
    uint32_t* const hh[1] = {h};
    const uint8_t* const pp[1] = {p};
    blocks_ni_n<1>(hh, pp, nb);
}

// `lanes` (1-4) messages in step, `nb` blocks each
__attribute__((target("sha,sse4.1,ssse3"))) void blocks_ni_lanes(int lanes, uint32_t* const* h, const uint8_t* const* p,
                                                                  size_t nb) {
    switch (lanes) {
        case 1: blocks_ni_n<1>(h, p, nb); break;
        case 2: blocks_ni_n<2>(h, p, nb); break;
        case 3: blocks_ni_n<3>(h, p, nb); break;
        default: blocks_ni_n<4>(h, p, nb); break;
    }
}

using BlockFn = void (*)(uint32_t*, const uint8_t*, size_t);

BlockFn pick_blocks() {
    const char* e = std::getenv("PBS_SHA_HOST_PORTABLE");  // A/B runs and the fallback's tests
    if (e && e[0] == '1') return blocks_portable;
    __builtin_cpu_init();
    unsigned a = 0, b = 0, c = 0, d = 0;  // CPUID leaf 7 subleaf 0: EBX bit 29 = SHA extensions
    const bool sha = __get_cpuid_count(7, 0, &a, &b, &c, &d) && ((b >> 29) & 1);
    return sha && __builtin_cpu_supports("sse4.1") && __builtin_cpu_supports("ssse3") ? blocks_ni
                                                                                      : blocks_portable;
}

BlockFn blocks() {
    static const BlockFn f = pick_blocks();
    return f;
}

}  // namespace

namespace pbs {

void sha256_host_init(HostSha& s) {
    std::memcpy(s.h, kInit, sizeof s.h);
    s.total = 0;
}

void sha256_host_blocks(HostSha& s, const uint8_t* p, size_t nbytes) {
    if (nbytes >= 64) blocks()(s.h, p, nbytes / 64);
    s.total += nbytes / 64 * 64;
}

// The message's last r < 64 bytes, then key, 0x80, zeros and the 64-bit bit length
// (FIPS 180-4 5.1.1) through one to three blocks on the stack.
void sha256_host_final(HostSha& s, const uint8_t* rest, size_t r, const uint8_t* key, size_t key_len,
                       uint8_t out[32]) {
    uint8_t tail[64 * 3] = {0};  // < 64 message bytes + <= 64 key bytes + 0x80 + 8 length bytes
    if (r) std::memcpy(tail, rest, r);
    if (key_len) std::memcpy(tail + r, key, key_len);
    const uint64_t bits = (s.total + r + key_len) * 8;
    r += key_len;
    tail[r] = 0x80;
    const size_t nt = (r + 1 + 8 + 63) / 64;
    for (int i = 0; i < 8; ++i) tail[nt * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    blocks()(s.h, tail, nt);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(s.h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s.h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s.h[i] >> 8);
        out[4 * i + 3] = (uint8_t)s.h[i];
    }
}

void sha256_host_one(const uint8_t* msg, size_t len, const uint8_t* key, size_t key_len, uint8_t out[32]) {
    HostSha s;
    sha256_host_init(s);
    sha256_host_blocks(s, msg, len);
    sha256_host_final(s, msg + len / 64 * 64, len % 64, key, key_len, out);
}

// Up to kShaLanes messages in step per thread: on the EPYC 9575F hosts one message runs at
// 2.47 GB/s (each sha256rnds2 waits for the previous one), two in step at 3.55, four at
// 4.36 (scripts/sha_host_lanes_bench.cpp, profiles/r04/sha_lanes/).  While fewer than four
// are open, the lanes advance kShaStep blocks at a time and then ask for more work.
constexpr int kShaLanes = 4;
constexpr uint64_t kShaStep = 2048;  // 128 KiB

void sha256_host_lanes(const std::function<bool(ShaJob&, bool)>& next, const std::function<void(const ShaJob&)>& done,
                       const uint8_t* key, size_t key_len) {
    struct Lane {
        ShaJob j;
        HostSha s;
        const uint8_t* p;
        uint64_t nb;  // whole blocks left
    };
    Lane L[kShaLanes];
    int act = 0;
    const bool ni = blocks() == blocks_ni;
    const char* e = std::getenv("PBS_SHA_HOST_LANES");  // A/B runs: 1 = one message at a time
    const int lanes = e && *e ? std::max(1, std::min(kShaLanes, std::atoi(e))) : kShaLanes;
    for (;;) {
        while (act < lanes && next(L[act].j, act == 0)) {
            Lane& l = L[act++];
            sha256_host_init(l.s);
            l.p = l.j.p;
            l.nb = l.j.len / 64;
        }
        if (act == 0) return;
        uint64_t k = act < lanes ? kShaStep : ~0ull;
        for (int i = 0; i < act; ++i) k = std::min(k, L[i].nb);
        if (k) {
            uint32_t* h[kShaLanes];
            const uint8_t* p[kShaLanes];
            for (int i = 0; i < act; ++i) h[i] = L[i].s.h, p[i] = L[i].p;
            if (ni)
                blocks_ni_lanes(act, h, p, k);
            else
                for (int i = 0; i < act; ++i) blocks()(h[i], p[i], k);
            for (int i = 0; i < act; ++i) {
                L[i].p += 64 * k;
                L[i].nb -= k;
                L[i].s.total += 64 * k;
            }
        }
        for (int i = 0; i < act;) {  // lanes without a whole block left: tail, key, padding
            if (L[i].nb) {
                ++i;
                continue;
            }
            sha256_host_final(L[i].s, L[i].p, L[i].j.len % 64, key, key_len, L[i].j.out);
            done(L[i].j);
            L[i] = L[--act];
        }
    }
}

// Hashes chunks items[0..n) (indices into bounds) of a host buffer holding stream bytes
// [base, ...) on `threads` threads; items are taken in the given order (longest first
// keeps the threads' finishing times close).
void sha256_host_items(const uint8_t* host, uint64_t base, const uint64_t* bounds, const uint32_t* items,
                       size_t n, const uint8_t* key, size_t key_len, uint8_t* digests, int threads) {
    std::atomic<size_t> next{0};
    auto work = [&] {
        sha256_host_lanes(
            [&](ShaJob& j, bool) {
                const size_t k = next.fetch_add(1, std::memory_order_relaxed);
                if (k >= n) return false;
                const uint32_t i = items ? items[k] : (uint32_t)k;
                j = ShaJob{host + (bounds[i] - base), bounds[i + 1] - bounds[i], digests + 32 * (size_t)i, i};
                return true;
            },
            [](const ShaJob&) {}, key, key_len);
    };
    const int t = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), n));
    std::vector<std::thread> pool;
    for (int j = 1; j < t; ++j) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
}

bool sha256_host_has_ni() { return blocks() == blocks_ni; }

bool all_zero(const uint8_t* p, size_t n) {
    size_t i = 0;
    for (; i < n && ((uintptr_t)(p + i) & 63); ++i)
        if (p[i]) return false;
    for (; i + 64 <= n; i += 64) {  // 64-byte lines, OR-reduced
        uint64_t acc = 0;
        for (int q = 0; q < 8; ++q) {
            uint64_t w;
            std::memcpy(&w, p + i + 8 * q, 8);
            acc |= w;
        }
        if (acc) return false;
    }
    for (; i < n; ++i)
        if (p[i]) return false;
    return true;
}

}  // namespace pbs

extern "C" int pbs_digest_chunks_host(const uint8_t* host_data, size_t data_len, uint64_t base,
                                      const uint64_t* bounds, size_t n, const uint8_t* key,
                                      size_t key_len, uint8_t* digests, int threads) {
    if (n == 0) return PBS_OK;
    if (!bounds || !digests || (data_len && !host_data) || key_len > PBS_DIGEST_MAX_KEY || (key_len && !key))
        return PBS_ERR_INVALID;
    for (size_t i = 0; i < n; ++i)
        if (bounds[i] > bounds[i + 1] || bounds[i] < base || bounds[i + 1] - base > data_len)
            return PBS_ERR_INVALID;
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return bounds[a + 1] - bounds[a] > bounds[b + 1] - bounds[b];
    });
    pbs::sha256_host_items(host_data, base, bounds, order.data(), n, key, key_len, digests,
                           threads > 0 ? threads : (int)std::thread::hardware_concurrency());
    return PBS_OK;
}

extern "C" int pbs_sha256_host_uses_ni(void) { return pbs::sha256_host_has_ni() ? 1 : 0; }
