// Drives the C++ host mirror (proxmox-backup_amd/host/pbs_chunker.hpp) the way the
// reference's callers do, and prints the chunk END offsets per caller, one line each:
//   scan <ends...>      Chunker::scan loop of test_chunker1's test2 (chunker.rs:246-257)
//   stream <ends...>    ChunkStream over pieces of `piece` bytes (chunk_stream.rs:40-77)
//   stream0 <ends...>   the same, scanning every piece as it arrives (min_scan 0)
//   writer <ends...>    DynamicChunkWriter via write_all (dynamic_index.rs:493-515)
//   batch <ends...>     find_cuts(is_final)
//   crc <crcs...>       host CRC-32 of the writer's chunks (DataBlob::compute_crc)
//   blob0 <hex>         first 16 bytes of the first chunk's uncompressed blob
//   index <csum hex>    DynamicIndexWriter over the writer's chunks (host SHA-256
//                       digests), written to $HOST_MIRROR_DIDX when set
//   pipe <ends...>      pipeline_host over the buffer in `piece`-byte pieces
//   pipedig <hex>       SHA-256 over the pipeline's digests in chunk order (and its crcs:
//   pipecrc <crcs...>   the blob CRC-32s); hostdig <hex>: the same over digest_chunks_host
// usage: host_mirror <avg> <len> <seed> <piece>   (input: splitmix64 random stream)
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

static void print(const char* tag, const std::vector<uint64_t>& v) {
    std::printf("%s", tag);
    for (uint64_t e : v) std::printf(" %llu", (unsigned long long)e);
    std::printf("\n");
}

int main(int argc, char** argv) {
    if (argc != 5) {
        std::fprintf(stderr, "usage: %s avg len seed piece\n", argv[0]);
        return 2;
    }
    const size_t avg = std::strtoull(argv[1], nullptr, 0), len = std::strtoull(argv[2], nullptr, 0);
    const uint64_t seed = std::strtoull(argv[3], nullptr, 0);
    const size_t piece = std::strtoull(argv[4], nullptr, 0);
    std::vector<uint8_t> data(len);
    for (size_t x = 0; x < len; ++x) data[x] = (uint8_t)(splitmix64(seed ^ (x >> 3)) >> ((x & 7) * 8));
    try {
        {
            pbs::Chunker c(avg);
            std::vector<uint64_t> ends;
            size_t pos = 0;
            while (pos < len) {
                const size_t k = c.scan(data.data() + pos, len - pos);
                if (k == 0) break;
                pos += k;
                ends.push_back(pos);
            }
            print("scan", ends);
        }
        for (size_t min_scan : {(size_t)0, (size_t)4 << 20}) {
            size_t off = 0;
            pbs::ChunkStream s([&](std::vector<uint8_t>& out) {
                if (off >= len) return false;
                const size_t n = std::min(piece, len - off);
                out.assign(data.begin() + off, data.begin() + off + n);
                off += n;
                return true;
            }, avg);
            s.set_min_scan(min_scan);
            std::vector<uint64_t> ends;
            uint64_t total = 0;
            while (auto ch = s.next()) {
                total += ch->size();
                ends.push_back(total);
            }
            print(min_scan ? "stream" : "stream0", ends);
        }
        {
            std::vector<uint64_t> ends;
            const char* didx = std::getenv("HOST_MIRROR_DIDX");
            pbs::DynamicIndexWriter index(didx ? didx : "/dev/null", {}, 1234);
            std::vector<uint64_t> crcs;
            std::vector<uint8_t> blob0;
            pbs::DynamicChunkWriter w([&](uint64_t end, const std::vector<uint8_t>& chunk) {
                ends.push_back(end);
                index.add_chunk(end, pbs::sha256(chunk.data(), chunk.size()));
                crcs.push_back(pbs::crc32(chunk.data(), chunk.size()));
                if (blob0.empty())
                    blob0 = pbs::blob_encode_uncompressed(chunk.data(), chunk.size(), (uint32_t)crcs.back());
            }, avg);
            for (size_t off = 0; off < len; off += piece)
                w.write_all(data.data() + off, std::min(piece, len - off));
            w.close();
            print("writer", ends);
            print("crc", crcs);
            std::printf("blob0 ");
            for (size_t k = 0; k < blob0.size() && k < 16; ++k) std::printf("%02x", blob0[k]);
            std::printf("\n");
            if (didx) {
                const pbs::Digest csum = index.close();
                std::printf("index ");
                for (uint8_t b : csum) std::printf("%02x", b);
                std::printf("\n");
            }
        }
        {
            pbs::Chunker c(avg);
            print("batch", c.find_cuts(data.data(), len, true));
        }
        {
            const pbs::PipelineResult r = pbs::pipeline_host(data.data(), len, avg, piece);
            print("pipe", r.ends);
            std::vector<uint64_t> crcs(r.crcs.begin(), r.crcs.end());
            print("pipecrc", crcs);
            std::vector<uint8_t> all;
            for (const auto& d : r.digests) all.insert(all.end(), d.begin(), d.end());
            const pbs::Digest h = pbs::sha256(all.data(), all.size());
            std::printf("pipedig ");
            for (uint8_t b : h) std::printf("%02x", b);
            std::printf("\n");
            std::vector<uint64_t> bounds{0};
            bounds.insert(bounds.end(), r.ends.begin(), r.ends.end());
            const std::vector<pbs::Digest> hd = pbs::digest_chunks_host(data.data(), len, 0, bounds, {}, 3);
            std::vector<uint8_t> all2;
            for (const auto& d : hd) all2.insert(all2.end(), d.begin(), d.end());
            const pbs::Digest h2 = pbs::sha256(all2.data(), all2.size());
            std::printf("hostdig ");
            for (uint8_t b : h2) std::printf("%02x", b);
            std::printf("\n");
        }
        try {
            pbs::Chunker bad(avg + 1 == 2 ? 3 : avg + 1);
            std::printf("badavg accepted\n");
        } catch (const std::invalid_argument& e) {
            std::printf("badavg %s\n", e.what());
        }
    } catch (const std::exception& e) {
        std::printf("error %s\n", e.what());
        return 1;
    }
    return 0;
}
