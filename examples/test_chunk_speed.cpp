// Port of examples/test_chunk_speed.rs onto the C++ host mirror (drop-in Chunker):
// an 80 MiB LE-u32 counter buffer (:8-14), Chunker::new(64 KiB) (:15), five passes of
// the scan loop with the chunker state carried across passes (:21-36), then the speed
// line (:40-50).  usage: test_chunk_speed [u32 count = 20 Mi] [passes = 5]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pbs_chunker.hpp"

int main(int argc, char** argv) {
    const size_t words = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 20u * 1024 * 1024;
    const int count = argc > 2 ? std::atoi(argv[2]) : 5;
    std::vector<uint8_t> buffer;
    buffer.reserve(words * 4);
    for (size_t i = 0; i < words; ++i)
        for (int j = 0; j < 4; ++j) buffer.push_back((uint8_t)((i >> (j << 3)) & 0xff));
    try {
        pbs::Chunker chunker(64 * 1024);
        const auto start = std::chrono::steady_clock::now();
        size_t chunk_count = 0;
        for (int i = 0; i < count; ++i) {
            size_t pos = 0;
            while (pos < buffer.size()) {
                const size_t k = chunker.scan(buffer.data() + pos, buffer.size() - pos);
                if (k == 0) break;
                pos += k;
                ++chunk_count;
            }
        }
        const double elapsed =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
        const double mbytecount = (double)count * (double)buffer.size() / (1024.0 * 1024.0);
        const double avg_chunk_size = mbytecount / (double)chunk_count;
        std::printf("SPEED = %g MB/s, avg chunk size = %g KB\n", mbytecount / elapsed,
                    avg_chunk_size * 1024.0);
        std::printf("CHUNKS %zu\n", chunk_count);
    } catch (const std::exception& e) {
        std::printf("error %s\n", e.what());
        return 1;
    }
    return 0;
}
