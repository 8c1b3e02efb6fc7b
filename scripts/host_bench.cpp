// Host-path throughput of the drop-in surface, without Python:
//   stream <piece>   pbs::ChunkStream over `piece`-byte input pieces (chunk_stream.rs:40-77;
//                    pxar feeds 256 KiB pieces)
//   scan             Chunker::scan loop over the whole buffer (test_chunk_speed.rs:25-36)
//   batch <piece>    find_cuts per piece (is_final on the last)
// Input: the VM-image generator, pageable host memory.
// build: g++ -O2 -std=c++17 -I include -I proxmox-backup_amd/host scripts/host_bench.cpp \
//          -L proxmox-backup_amd/csrc -lpbschunk -Wl,-rpath,proxmox-backup_amd/csrc -o host_bench
// run:   ./host_bench [GiB=1] [avg=4194304]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pbs_chunker.hpp"

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void gen_vmimage(std::vector<uint8_t>& d, uint64_t seed) {
    uint64_t* w = reinterpret_cast<uint64_t*>(d.data());
    const size_t nw = d.size() / 8;
    for (size_t k = 0; k < nw; ++k) {
        const uint64_t x = k << 3, g = x >> 30;
        const uint64_t ext = (splitmix64(seed ^ 0x4558544E54000000ull ^ g) & 15u) << 26;
        const uint64_t in_g = x & ((1ull << 30) - 1);
        uint64_t v = 0;
        if (!(in_g >= ext && in_g < ext + (1ull << 26)) &&
            splitmix64(seed ^ 0x7A65726F50414745ull ^ (x >> 12)) % 100u >= 40u)
            v = splitmix64(seed ^ 0x52414E44574F5244ull ^ k);
        w[k] = v;
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 1.0;
    const size_t avg = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : (4u << 20);
    const size_t len = (size_t)(gib * (1ull << 30)) / 8 * 8;
    std::vector<uint8_t> data(len);
    gen_vmimage(data, 0x5EED0003ull);
    const double G = (double)len / (1ull << 30);
    try {
        {  // warm-up (allocations, code objects)
            pbs::Chunker c(avg);
            c.find_cuts(data.data(), std::min<size_t>(len, 64u << 20), true);
        }
        for (size_t piece : {64u << 10, 256u << 10, 1u << 20, 4u << 20, 16u << 20}) {
            size_t off = 0, nch = 0;
            pbs::ChunkStream s([&](std::vector<uint8_t>& out) {
                if (off >= len) return false;
                const size_t n = std::min(piece, len - off);
                out.assign(data.begin() + off, data.begin() + off + n);
                off += n;
                return true;
            }, avg);
            const double t0 = now();
            while (auto ch = s.next()) ++nch;
            const double t = now() - t0;
            std::printf("stream piece=%zu KiB: %.3f GiB/s (%zu chunks, %.1f us/piece)\n", piece >> 10,
                        G / t, nch, t * 1e6 / ((len + piece - 1) / piece));
            std::fflush(stdout);
        }
        {
            pbs::Chunker c(avg);
            size_t pos = 0, nch = 0;
            const double t0 = now();
            while (pos < len) {
                const size_t k = c.scan(data.data() + pos, len - pos);
                if (k == 0) break;
                pos += k;
                ++nch;
            }
            const double t = now() - t0;
            std::printf("scan loop (whole buffer): %.3f GiB/s (%zu cuts)\n", G / t, nch);
        }
        for (size_t piece : {256u << 10, 4u << 20, 64u << 20, 1024u << 20}) {
            pbs::Chunker c(avg);
            size_t nch = 0;
            const double t0 = now();
            for (size_t off = 0; off < len; off += piece) {
                const size_t n = std::min(piece, len - off);
                nch += c.find_cuts(data.data() + off, n, off + n >= len).size();
            }
            const double t = now() - t0;
            std::printf("find_cuts piece=%zu KiB: %.3f GiB/s (%zu cuts)\n", piece >> 10, G / t, nch);
            std::fflush(stdout);
        }
    } catch (const std::exception& e) {
        std::printf("error %s\n", e.what());
        return 1;
    }
    return 0;
}
