// Host SHA-256 microbenchmark: N messages in step (N = 1..4) through the block function
// template of pbs_sha_host.cpp (included, so its internal template is visible), 32 MiB each;
// then sha256_host_items (the multi-lane scheduler) over 1 GiB of 1-16 MiB chunks on 1 and
// 14 threads against one chunk at a time per thread.
//   g++ -O2 -std=c++17 -I proxmox-backup_amd/csrc -I include scripts/sha_host_lanes_bench.cpp -o /tmp/sha_lanes -lpthread
#include "../proxmox-backup_amd/csrc/pbs_sha_host.cpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>

template <int N>
__attribute__((target("sha,sse4.1,ssse3"))) void run_n(uint32_t (*h)[8], const uint8_t* const* p, size_t nb) {
    uint32_t* hh[N];
    for (int j = 0; j < N; ++j) hh[j] = h[j];
    blocks_ni_n<N>(hh, p, nb);
}

int main() {
    const size_t L = 32 << 20, nb = L / 64;
    std::vector<std::vector<uint8_t>> m(4, std::vector<uint8_t>(L));
    for (int j = 0; j < 4; ++j)
        for (size_t i = 0; i < L; ++i) m[j][i] = (uint8_t)((i + 977 * j) * 2654435761u >> 13);
    const uint8_t* p[4] = {m[0].data(), m[1].data(), m[2].data(), m[3].data()};
    uint32_t ref[4][8];
    for (int j = 0; j < 4; ++j) {
        std::memcpy(ref[j], kInit, 32);
        blocks_ni(ref[j], p[j], nb);
    }
    for (int rep = 0; rep < 2; ++rep) {
        for (int n = 1; n <= 4; ++n) {
            uint32_t h[4][8];
            for (int j = 0; j < 4; ++j) std::memcpy(h[j], kInit, 32);
            const auto t0 = std::chrono::steady_clock::now();
            if (n == 1) for (int j = 0; j < 4; ++j) run_n<1>(h + j, p + j, nb);
            if (n == 2) { run_n<2>(h, p, nb); run_n<2>(h + 2, p + 2, nb); }
            if (n == 3) { run_n<3>(h, p, nb); run_n<1>(h + 3, p + 3, nb); }
            if (n == 4) run_n<4>(h, p, nb);
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            printf("N=%d  %.2f GB/s per core (4 x 32 MiB)  equal=%d\n", n, 4.0 * L / s / 1e9,
                   !std::memcmp(h, ref, sizeof ref));
        }
    }
    // a chunk list: 1 GiB of chunks 1..16 MiB long (+ ragged tails), longest first
    const size_t T = 1ull << 30;
    std::vector<uint8_t> buf(T);
    for (size_t i = 0; i < T; i += 8) {
        const uint64_t v = (i + 0x9e3779b97f4a7c15ull) * 0xbf58476d1ce4e5b9ull;
        std::memcpy(&buf[i], &v, 8);
    }
    std::vector<uint64_t> bounds{0};
    uint64_t x = 88172645463325252ull;
    while (bounds.back() < T) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        bounds.push_back(std::min<uint64_t>(T, bounds.back() + (1u << 20) + x % (15u << 20) + x % 61));
    }
    const size_t n = bounds.size() - 1;
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return bounds[a + 1] - bounds[a] > bounds[b + 1] - bounds[b]; });
    std::vector<uint8_t> d1(32 * n), d2(32 * n);
    for (int threads : {1, 14}) {
        for (int rep = 0; rep < 2; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            std::atomic<size_t> nx{0};
            std::vector<std::thread> pool;
            for (int t = 0; t < threads; ++t)
                pool.emplace_back([&] {
                    for (size_t k; (k = nx.fetch_add(1)) < n;) {
                        const uint32_t i = order[k];
                        pbs::sha256_host_one(buf.data() + bounds[i], bounds[i + 1] - bounds[i], nullptr, 0, &d1[32 * i]);
                    }
                });
            for (auto& th : pool) th.join();
            auto t1 = std::chrono::steady_clock::now();
            pbs::sha256_host_items(buf.data(), 0, bounds.data(), order.data(), n, nullptr, 0, d2.data(), threads);
            auto t2 = std::chrono::steady_clock::now();
            printf("%zu chunks, %d threads: one at a time %.2f GB/s, lanes %.2f GB/s, equal=%d\n", n, threads,
                   T / std::chrono::duration<double>(t1 - t0).count() / 1e9,
                   T / std::chrono::duration<double>(t2 - t1).count() / 1e9, d1 == d2);
        }
    }
}
