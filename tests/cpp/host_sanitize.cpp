// Host-only driver of the library's threaded host C++ for the sanitizer builds
// (proxmox-backup_amd/csrc/Makefile `sanitize`: ASan + UBSan, then TSan; no device):
//   - the pipeline's host share (csrc/host_share.h): a producer appends chunk ends and
//     pushes routed indices in bursts while 6 workers hash them four in step, zero chunks
//     memoised per length, flags read by a polling consumer (the upload encoder's role);
//   - the routing rule and the copy-end projection;
//   - pbs_digest_chunks_host (the hybrid digest's host lanes) on 1..8 threads, keyed and not;
//   - pbs_didx_build / pbs_sha256 (the .didx image and its checksum).
// Every digest is checked against the one-message SHA-256 (sha256_host_one), whose own
// known answers are the FIPS 180-4 vectors below.  Exit 0 = all checks passed.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "host_share.h"
#include "pbs_chunker.h"
#include "pbs_digest.h"
#include "sha_host.h"

static int failures = 0;
#define CHECK(x)                                                              \
    do {                                                                      \
        if (!(x)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #x); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

static std::string hex(const uint8_t* d, size_t n) {
    static const char* k = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) {
        s += k[d[i] >> 4];
        s += k[d[i] & 15];
    }
    return s;
}

static void known_answers() {
    uint8_t out[32];
    pbs::sha256_host_one(reinterpret_cast<const uint8_t*>("abc"), 3, nullptr, 0, out);
    CHECK(hex(out, 32) == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
    pbs::sha256_host_one(nullptr, 0, nullptr, 0, out);
    CHECK(hex(out, 32) == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
    const char* m = "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq";
    pbs::sha256_host_one(reinterpret_cast<const uint8_t*>(m), std::strlen(m), nullptr, 0, out);
    CHECK(hex(out, 32) == "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1");
    // pbs_sha256 (the index checksum's hash) agrees
    uint8_t o2[32];
    pbs_sha256(reinterpret_cast<const uint8_t*>(m), std::strlen(m), o2);
    CHECK(std::memcmp(out, o2, 32) == 0);
}

static void host_share(std::mt19937_64& rng, bool keyed) {
    // ~40 MiB: random chunks 0..2 MiB, all-zero chunks of three repeated lengths, empties
    std::vector<uint64_t> lens;
    for (int i = 0; i < 60; ++i) {
        const int kind = (int)(rng() % 5);
        lens.push_back(kind == 0 ? 0 : kind == 1 ? (uint64_t)(1 + rng() % 3) * 65536 + 7 : rng() % (2u << 20));
    }
    uint64_t total = 0;
    for (uint64_t l : lens) total += l;
    std::vector<uint8_t> host(total + 1);
    std::vector<uint64_t> ends(lens.size());
    {
        uint64_t o = 0;
        for (size_t i = 0; i < lens.size(); ++i) {
            const bool zero = lens[i] % 65536 == 7;
            for (uint64_t b = 0; b < lens[i]; ++b) host[o + b] = zero ? 0 : (uint8_t)rng();
            o += lens[i];
            ends[i] = o;
        }
    }
    const uint8_t key[32] = {1, 2, 3};
    const size_t n = lens.size();
    std::vector<uint8_t> dig(32 * n, 0xEE), ref(32 * n);
    for (size_t i = 0; i < n; ++i)
        pbs::sha256_host_one(host.data() + (i ? ends[i - 1] : 0), lens[i], keyed ? key : nullptr, keyed ? 32 : 0,
                             ref.data() + 32 * i);
    std::vector<uint64_t> pub(n, 0);  // the producer's view of `ends`, appended as it goes
    std::vector<uint8_t> mask(n, 0);
    pbs::HostShare hs(host.data(), pub.data(), dig.data(), n, keyed ? key : nullptr, keyed ? 32 : 0,
                      pbs::HostShare::Clock::now());
    std::vector<std::thread> pool;
    for (int t = 0; t < 6; ++t) pool.emplace_back([&] { hs.work(); });
    // a consumer polling the flags of the host-routed chunks (the upload encoder's wait)
    // (it reads the masks of the chunks published so far: the upload worker gets each
    // batch's range under its queue's mutex)
    std::atomic<bool> stop{false};
    std::atomic<size_t> seen{0}, published{0};
    std::thread consumer([&] {
        std::vector<uint8_t> got(n, 0);
        while (!stop.load()) {
            const size_t np = published.load(std::memory_order_acquire);
            for (size_t i = 0; i < np; ++i)
                if (mask[i] && !got[i] && hs.flag(i)) {
                    got[i] = 1;
                    seen += 1;
                }
            std::this_thread::yield();
        }
    });
    // (the mask is written before the push that publishes the chunk, as in the pipeline)
    size_t i0 = 0, host_n = 0;
    while (i0 < n) {
        const size_t i1 = std::min(n, i0 + 1 + (size_t)(rng() % 9));
        for (size_t i = i0; i < i1; ++i) {
            pub[i] = ends[i];
            mask[i] = pbs::route_to_host(6, 1 << 20, 0.0, lens[i], 15e3, 100.0) || lens[i] % 65536 == 7 ? 1 : 0;
            host_n += mask[i];
        }
        hs.push(mask.data(), i0, i1);
        published.store(i1, std::memory_order_release);
        i0 = i1;
        if (rng() % 3 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    hs.finish();
    hs.work();  // the producer joins in, as the pipeline's main thread does
    for (auto& th : pool) th.join();
    stop = true;
    consumer.join();
    CHECK(hs.chunks() == host_n);
    for (size_t i = 0; i < n; ++i)
        if (mask[i]) {
            CHECK(hs.flag(i));
            CHECK(std::memcmp(dig.data() + 32 * i, ref.data() + 32 * i, 32) == 0);
        } else {
            CHECK(dig[32 * i] == 0xEE);  // not the host's: untouched
        }
    std::printf("host_share keyed=%d: %zu chunks, %zu on the host, %llu MiB hashed, consumer saw %zu flags\n",
                (int)keyed, n, host_n, (unsigned long long)(hs.bytes() >> 20), seen.load());
}

static void routing() {
    // deadline rule: a chunk whose chain would end after the projected copy end goes host
    const double t_end = pbs::projected_copy_end(64ull << 30, 4ull << 30, 4, 100.0, 10.0);
    CHECK(t_end > 1600.0 && t_end < 1611.0);  // 64 GiB at 4 GiB per 100 ms, + 10 ms slack
    CHECK(!pbs::route_to_host(8, ~0ull, 100.0, 1 << 20, 15e3, t_end));        // 70 ms chain: GPU
    CHECK(pbs::route_to_host(8, ~0ull, 1590.0, 1 << 20, 15e3, t_end));        // too late: host
    CHECK(!pbs::route_to_host(0, ~0ull, 1590.0, 1 << 20, 15e3, t_end));       // no host threads
    CHECK(pbs::route_to_host(8, 8 << 20, 0.0, 8 << 20, 15e3, 0.0));           // fixed threshold
    CHECK(!pbs::route_to_host(8, 8 << 20, 1e9, (8 << 20) - 1, 15e3, 0.0));
    CHECK(pbs::projected_copy_end(1000, 0, 0, 0.0, 0.0) > 0.0);               // before two pieces
}

static void digest_host(std::mt19937_64& rng) {
    const size_t n = 300;
    std::vector<uint64_t> b(n + 1, 0);
    for (size_t i = 0; i < n; ++i) b[i + 1] = b[i] + (rng() % 7 == 0 ? 0 : rng() % 300000);
    const uint64_t base = 12345;
    std::vector<uint8_t> data(b[n] + 3);
    for (auto& x : data) x = (uint8_t)rng();
    std::vector<uint64_t> abs(n + 1);
    for (size_t i = 0; i <= n; ++i) abs[i] = b[i] + base;
    const uint8_t key[17] = {9, 8, 7};
    for (int keyed = 0; keyed < 2; ++keyed)
        for (int threads : {1, 3, 8}) {
            std::vector<uint8_t> d(32 * n);
            CHECK(pbs_digest_chunks_host(data.data(), data.size(), base, abs.data(), n, keyed ? key : nullptr,
                                         keyed ? 17 : 0, d.data(), threads) == PBS_OK);
            for (size_t i = 0; i < n; ++i) {
                uint8_t r[32];
                pbs::sha256_host_one(data.data() + b[i], b[i + 1] - b[i], keyed ? key : nullptr, keyed ? 17 : 0, r);
                CHECK(std::memcmp(r, d.data() + 32 * i, 32) == 0);
            }
        }
    // argument errors
    uint8_t d[32];
    CHECK(pbs_digest_chunks_host(data.data(), 10, base, abs.data(), 1, nullptr, 0, d, 1) == PBS_ERR_INVALID);
    std::printf("digest_chunks_host: %zu chunks x {1, 3, 8} threads x {plain, keyed}\n", n);
}

static void didx() {
    const size_t n = 1000;
    std::vector<uint64_t> ends(n);
    std::vector<uint8_t> dig(32 * n);
    for (size_t i = 0; i < n; ++i) {
        ends[i] = (i + 1) * 4096 + i;
        for (int k = 0; k < 32; ++k) dig[32 * i + k] = (uint8_t)(i * 31 + k);
    }
    std::vector<uint8_t> img(pbs_didx_size(n));
    uint8_t uuid[16] = {1, 2, 3, 4}, csum[32];
    CHECK(pbs_didx_build(ends.data(), dig.data(), n, uuid, -5, img.data(), img.size(), csum) == PBS_OK);
    // csum = SHA-256 over the 40-byte entries (dynamic_index.rs:373-391)
    uint8_t want[32];
    pbs_sha256(img.data() + 4096, 40 * n, want);
    CHECK(std::memcmp(want, csum, 32) == 0);
    CHECK(std::memcmp(img.data() + 32, csum, 32) == 0);
    CHECK(pbs_didx_build(ends.data(), dig.data(), n, uuid, 0, img.data(), img.size() - 1, csum) != PBS_OK);
    std::printf("didx: %zu entries\n", n);
}

int main() {
    std::mt19937_64 rng(20261018);
    known_answers();
    routing();
    for (int r = 0; r < 3; ++r) {
        host_share(rng, false);
        host_share(rng, true);
    }
    digest_host(rng);
    didx();
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "host_sanitize ok", failures);
    return failures ? 1 : 0;
}
