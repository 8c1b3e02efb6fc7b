// Port of examples/test_chunk_speed2.rs onto the C++ host mirror: ChunkStream with the
// default average (4 MiB) over a file read in pieces (tokio FramedRead + BytesCodec,
// 8 KiB reads), printing every chunk and the summary lines (:44-60).  Without a file
// argument the input is 1 GiB of the seeded random stream (examples/common.hpp),
// generated before the clock starts (the reference reads random-test.dat, i.e. from the
// page cache): each read is a memcpy of the next piece.
// min_scan = 0 (the default) is the unchanged caller of chunk_stream.rs:40-77 (one
// Chunker::scan per read); min_scan > 0 gathers that many bytes per scan
// (pbs::ChunkStream::set_min_scan).  The reference's lines are printed for the chosen
// mode, then the same input runs once more in the other mode (0 <-> 4 MiB) and one
// "beside:" line gives its rate, so a gathering number is never quoted without the
// unchanged caller's.
// usage: test_chunk_speed2 [random-test.dat | -] [bytes = 1 GiB] [piece = 8192] [avg = 4 MiB]
//                          [min_scan = 0] [quiet = 0]
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
    const size_t min_scan = argc > 5 ? std::strtoull(argv[5], nullptr, 0) : 0;
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
    struct Run {
        uint64_t chunks = 0, bytes = 0;
        double us = 0;
    };
    // one pass over the input with the given min_scan; false on a chunk over 16 MiB
    auto run = [&](size_t gather, bool print, Run& r) {
        off = 0;
        if (f) std::rewind(f);
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
        stream.set_min_scan(gather);
        const auto start = std::chrono::steady_clock::now();
        while (auto chunk = stream.next()) {
            if (chunk->size() > 16u * 1024 * 1024) {
                std::printf("error Chunk too large %zu\n", chunk->size());
                return false;
            }
            ++r.chunks;
            r.bytes += chunk->size();
            if (print) std::printf("Got chunk %zu\n", chunk->size());
        }
        r.us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - start).count();
        return true;
    };
    auto mbs = [](const Run& r) {
        return (unsigned long long)((double)r.bytes / (1024.0 * 1024.0) / (r.us / 1e6));
    };
    try {
        Run a;
        if (!run(min_scan, !quiet, a)) return 1;
        std::printf("Uploaded %llu chunks in %llu seconds (%llu MB/s).\n", (unsigned long long)a.chunks,
                    (unsigned long long)(a.us / 1e6), mbs(a));
        if (a.chunks)
            std::printf("Average chunk size was %llu bytes.\n", (unsigned long long)(a.bytes / a.chunks));
        if (a.chunks)
            std::printf("time per request: %llu microseconds.\n", (unsigned long long)(a.us / (double)a.chunks));
        const size_t other = min_scan ? 0 : (4u << 20);
        Run b;
        if (!run(other, false, b)) return 1;
        std::printf("beside: min_scan %zu (%s): %llu chunks, %llu MB/s%s\n", other,
                    other ? "4 MiB gathered per scan" : "unchanged caller, one scan() per read",
                    (unsigned long long)b.chunks, mbs(b),
                    b.chunks == a.chunks && b.bytes == a.bytes ? "" : " -- DIFFERENT chunk count");
        if (b.chunks != a.chunks || b.bytes != a.bytes) return 1;
    } catch (const std::exception& e) {
        std::printf("error %s\n", e.what());
        return 1;
    }
    if (f) std::fclose(f);
    return 0;
}
