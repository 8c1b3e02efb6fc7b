// Port of examples/test_chunk_speed2.rs onto the C++ host mirror: ChunkStream with the
// default average (4 MiB) over a file read in pieces (tokio FramedRead + BytesCodec,
// 8 KiB reads), printing every chunk and the summary lines (:44-60).  Without a file
// argument the input is 1 GiB of the seeded random stream (examples/common.hpp),
// generated before the clock starts (the reference reads random-test.dat, i.e. from the
// page cache): each read is a memcpy of the next piece.
// min_scan = 0 is the unchanged caller of chunk_stream.rs:40-77 (one Chunker::scan per
// read); the default gathers 4 MiB per scan (pbs::ChunkStream::set_min_scan).
// usage: test_chunk_speed2 [random-test.dat | -] [bytes = 1 GiB] [piece = 8192] [avg = 4 MiB]
//                          [min_scan = 4 MiB] [quiet = 0]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "pbs_chunker.hpp"

int main(int argc, char** argv) {
    const char* path = argc > 1 && std::strcmp(argv[1], "-") ? argv[1] : nullptr;
    const uint64_t total = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : (1ull << 30);
    const size_t piece = argc > 3 ? std::strtoull(argv[3], nullptr, 0) : 8192;
    const size_t avg = argc > 4 ? std::strtoull(argv[4], nullptr, 0) : 4096 * 1024;
    const size_t min_scan = argc > 5 ? std::strtoull(argv[5], nullptr, 0) : (4u << 20);
    const bool quiet = argc > 6 && std::atoi(argv[6]) != 0;
    std::FILE* f = path ? std::fopen(path, "rb") : nullptr;
    if (path && !f) {
        std::printf("error cannot open %s\n", path);
        return 1;
    }
    uint64_t off = 0;
    std::vector<uint8_t> input;
    if (!f) {
        input.resize(total);
        random_bytes(0x5EED0001ull, 0, input.data(), total);
    }
    try {
        pbs::ChunkStream stream([&](std::vector<uint8_t>& out) {
            out.resize(piece);
            size_t n = 0;
            if (f) {
                n = std::fread(out.data(), 1, piece, f);
            } else if (off < total) {
                n = (size_t)std::min<uint64_t>(piece, total - off);
                std::memcpy(out.data(), input.data() + off, n);
            }
            off += n;
            out.resize(n);
            return n > 0;
        }, avg);
        stream.set_min_scan(min_scan);
        const auto start = std::chrono::steady_clock::now();
        uint64_t repeat = 0, stream_len = 0;
        while (auto chunk = stream.next()) {
            if (chunk->size() > 16u * 1024 * 1024) {
                std::printf("error Chunk too large %zu\n", chunk->size());
                return 1;
            }
            ++repeat;
            stream_len += chunk->size();
            if (!quiet) std::printf("Got chunk %zu\n", chunk->size());
        }
        const double us = std::chrono::duration<double, std::micro>(
                              std::chrono::steady_clock::now() - start).count();
        std::printf("Uploaded %llu chunks in %llu seconds (%llu MB/s).\n",
                    (unsigned long long)repeat, (unsigned long long)(us / 1e6),
                    (unsigned long long)((double)stream_len / (1024.0 * 1024.0) / (us / 1e6)));
        if (repeat)
            std::printf("Average chunk size was %llu bytes.\n",
                        (unsigned long long)(stream_len / repeat));
        if (repeat)
            std::printf("time per request: %llu microseconds.\n",
                        (unsigned long long)(us / (double)repeat));
    } catch (const std::exception& e) {
        std::printf("error %s\n", e.what());
        return 1;
    }
    if (f) std::fclose(f);
    return 0;
}
