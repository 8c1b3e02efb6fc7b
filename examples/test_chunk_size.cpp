// Port of examples/test_chunk_size.rs onto the C++ host mirror: a Write adapter around
// Chunker::new(4 MiB) records each chunk size with Welford's running mean/variance
// (:38-64) and prints one line per chunk; input: 64 KiB buffers (:98-113) of the seeded
// random stream (examples/common.hpp) instead of /dev/urandom, until more than 1 GiB.
// usage: test_chunk_size [limit bytes = 1 GiB] [avg = 4194304]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.hpp"
#include "pbs_chunker.hpp"

struct ChunkWriter {
    explicit ChunkWriter(size_t chunk_size) : chunker(chunk_size) {}
    pbs::Chunker chunker;
    size_t last_chunk = 0, chunk_offset = 0, chunk_count = 0;
    double m_old = 0, m_new = 0, s_old = 0, s_new = 0;

    void record_stat(double chunk_size) {
        ++chunk_count;
        if (chunk_count == 1) {
            m_old = m_new = chunk_size;
            s_old = 0.0;
        } else {
            m_new = m_old + (chunk_size - m_old) / (double)chunk_count;
            s_new = s_old + (chunk_size - m_old) * (chunk_size - m_new);
            m_old = m_new;
            s_old = s_new;
        }
        const double variance = chunk_count > 1 ? s_new / (double)(chunk_count - 1) : 0.0;
        const double deviation_per = std::sqrt(variance) * 100.0 / m_new;
        std::printf("COUNT %10zu SIZE %10zu MEAN %10zu DEVIATION %3zu%%\n", chunk_count,
                    (size_t)chunk_size, (size_t)m_new, (size_t)deviation_per);
    }

    // Write::write (:70-88): consumed bytes
    size_t write(const uint8_t* data, size_t len) {
        const size_t pos = chunker.scan(data, len);
        if (pos > 0) {
            chunk_offset += pos;
            record_stat((double)(chunk_offset - last_chunk));
            last_chunk = chunk_offset;
            return pos;
        }
        chunk_offset += len;
        return len;
    }
    void write_all(const uint8_t* data, size_t len) {
        while (len) {
            const size_t k = write(data, len);
            data += k;
            len -= k;
        }
    }
};

int main(int argc, char** argv) {
    const uint64_t limit = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (1ull << 30);
    const size_t avg = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 4096 * 1024;
    try {
        ChunkWriter writer(avg);
        std::vector<uint8_t> buffer(64 * 1024);
        uint64_t bytes = 0;
        for (;;) {
            random_bytes(0x5EED0001ull, bytes, buffer.data(), buffer.size());
            bytes += buffer.size();
            writer.write_all(buffer.data(), buffer.size());
            if (bytes > limit) break;
        }
    } catch (const std::exception& e) {
        std::printf("error %s\n", e.what());
        return 1;
    }
    return 0;
}
