// C++ host mirror of proxmox-backup's chunker interface over the C ABI
// (include/pbs_chunker.h).  Header-only; link with libpbschunk.so.
//
//   pbs::Chunker            pbs-datastore/src/chunker.rs:18-186   (new / scan)
//   pbs::ChunkStream        pbs-client/src/chunk_stream.rs:12-78  (pull iterator of chunks)
//   pbs::DynamicChunkWriter pbs-datastore/src/dynamic_index.rs:397-523 (write / close)
//   pbs::DynamicIndexWriter pbs-datastore/src/dynamic_index.rs:297-391 (add_chunk / close)
//   pbs::digest_chunks_device  DataChunkBuilder::digest (data_blob.rs:516-536) per chunk, GPU
//   pbs::sha256             openssl::sha::sha256 (host; index checksum)
//   pbs::crc32_chunks_device DataBlob::compute_crc (data_blob.rs:70-75) per chunk, GPU
//   pbs::crc32 / pbs::blob_encode_uncompressed  crc32fast::Hasher, DataBlob::encode(.., false)
//   pbs::digest_chunks_host  the per-chunk digest on host cores (SHA extensions)
//   pbs::pipeline_host      ChunkStream + the upload stream's per-chunk digest
//                           (chunk_stream.rs:40-77, backup_writer.rs:671-678) over a host buffer
//
// Same names, argument meaning and error behaviour as the reference: a non-power-of-two
// average throws std::invalid_argument with the reference's panic text; `scan` is
// infallible in the reference, so a device error throws std::runtime_error (the Rust
// shim in INTEGRATION.md panics at the same point).  The hash scan runs on the GPU.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <functional>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "pbs_chunker.h"
#include "pbs_blob.h"
#include "pbs_digest.h"

namespace pbs {

class Chunker {
  public:
    explicit Chunker(size_t chunk_size_avg) {
        int err = 0;
        h_ = pbs_chunker_new(chunk_size_avg, &err);
        if (!h_) {
            if (err == PBS_ERR_NOT_POW2)
                throw std::invalid_argument("got unexpected chunk size - not a power of two.");
            throw std::runtime_error(std::string("pbs_chunker_new: ") + pbs_strerror(err));
        }
    }
    Chunker(const Chunker&) = delete;
    Chunker& operator=(const Chunker&) = delete;
    Chunker(Chunker&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
    Chunker& operator=(Chunker&& o) noexcept {
        if (this != &o) {
            reset_handle();
            h_ = std::exchange(o.h_, nullptr);
        }
        return *this;
    }
    ~Chunker() { reset_handle(); }

    // chunker.rs:112 -- 0 if no boundary in `data` (all consumed), else the position
    // just after the cut byte, relative to `data`.
    size_t scan(const uint8_t* data, size_t len) {
        const size_t r = pbs_chunker_scan(h_, data, len);
        if (r == SIZE_MAX)
            throw std::runtime_error(std::string("pbs_chunker_scan: ") +
                                     pbs_strerror(pbs_chunker_last_error(h_)));
        return r;
    }
    size_t scan(const std::vector<uint8_t>& v) { return scan(v.data(), v.size()); }

    // All chunk END offsets (absolute) decided inside `data`; with is_final the tail too.
    std::vector<uint64_t> find_cuts(const uint8_t* data, size_t len, bool is_final = false) {
        std::vector<uint64_t> out(pbs_chunker_cuts_bound(h_, len));
        size_t n = 0;
        const int rc = pbs_chunker_find_cuts(h_, data, len, is_final ? 1 : 0, out.data(),
                                             out.size(), &n);
        if (rc != PBS_OK)
            throw std::runtime_error(std::string("pbs_chunker_find_cuts: ") + pbs_strerror(rc));
        out.resize(n);
        return out;
    }

    pbs_chunker* handle() const { return h_; }

  private:
    void reset_handle() {
        if (h_) pbs_chunker_free(h_);
        h_ = nullptr;
    }
    pbs_chunker* h_ = nullptr;
};

// ChunkStream: `next()` pulls input pieces from `source` (returns false at EOF) and
// yields chunks; the remainder is yielded at EOF (chunk_stream.rs:64-68).
class ChunkStream {
  public:
    using Source = std::function<bool(std::vector<uint8_t>&)>;
    explicit ChunkStream(Source source, std::optional<size_t> chunk_size = std::nullopt)
        : source_(std::move(source)), chunker_(chunk_size.value_or(4 * 1024 * 1024)) {}

    std::optional<std::vector<uint8_t>> next() {
        for (;;) {
            // gather at least min_scan unscanned bytes before a scan: each scan is a
            // host->device round trip (~30 us), so scanning every 8 KiB read piece would
            // cap the stream near 250 MB/s.  The cuts are those of the whole stream either
            // way (the chunker is a pure function of the bytes); only latency changes.
            while (!eof_ && buffer_.size() - head_ - scan_pos_ < std::max<size_t>(min_scan_, 1)) pull();
            const size_t avail = buffer_.size() - head_;
            if (scan_pos_ < avail) {
                const uint8_t* base = buffer_.data() + head_;
                const size_t boundary = chunker_.scan(base + scan_pos_, avail - scan_pos_);
                const size_t chunk_size = scan_pos_ + boundary;
                if (boundary == 0) {
                    scan_pos_ = avail;
                } else if (chunk_size <= avail) {
                    // BytesMut::split_to (chunk_stream.rs:51) is O(1): advance a head
                    // offset instead of moving the remainder
                    std::vector<uint8_t> out(base, base + chunk_size);
                    head_ += chunk_size;
                    scan_pos_ = 0;
                    return out;
                } else {
                    throw std::logic_error("got unexpected chunk boundary from chunker");
                }
                continue;
            }
            // everything buffered is scanned and the source is exhausted: the tail
            scan_pos_ = 0;
            if (head_ == buffer_.size()) return std::nullopt;
            std::vector<uint8_t> out(buffer_.begin() + (ptrdiff_t)head_, buffer_.end());
            buffer_.clear();
            head_ = 0;
            return out;
        }
    }

    // bytes gathered per device scan (default 4 MiB; 0 scans every piece as it arrives)
    void set_min_scan(size_t bytes) { min_scan_ = bytes; }

  private:
    Source source_;
    Chunker chunker_;
    std::vector<uint8_t> buffer_;
    size_t head_ = 0;      // bytes of buffer_ already handed out
    size_t scan_pos_ = 0;  // relative to head_
    size_t min_scan_ = 4u << 20;
    bool eof_ = false;

    void pull() {
        std::vector<uint8_t> piece;
        if (!source_(piece)) {
            eof_ = true;
            return;
        }
        if (head_ && head_ * 2 >= buffer_.size()) {  // compact before growing
            buffer_.erase(buffer_.begin(), buffer_.begin() + (ptrdiff_t)head_);
            head_ = 0;
        }
        buffer_.insert(buffer_.end(), piece.begin(), piece.end());
    }
};

// DynamicChunkWriter: `write` returns the bytes consumed (the caller re-submits the
// rest, as write_all does); every finished chunk goes to sink(chunk_end_offset, bytes)
// in place of the digest/compress/insert/add_chunk step (dynamic_index.rs:444-490).
class DynamicChunkWriter {
  public:
    using Sink = std::function<void(uint64_t, const std::vector<uint8_t>&)>;
    DynamicChunkWriter(Sink sink, size_t chunk_size) : sink_(std::move(sink)), chunker_(chunk_size) {
        chunk_buffer_.reserve(chunk_size * 4);
    }

    size_t write(const uint8_t* data, size_t len) {
        const size_t pos = chunker_.scan(data, len);
        if (pos > 0) {
            chunk_buffer_.insert(chunk_buffer_.end(), data, data + pos);
            chunk_offset_ += pos;
            write_chunk_buffer();
            return pos;
        }
        chunk_offset_ += len;
        chunk_buffer_.insert(chunk_buffer_.end(), data, data + len);
        return len;
    }

    void write_all(const uint8_t* data, size_t len) {
        while (len) {
            const size_t k = write(data, len);
            data += k;
            len -= k;
        }
    }

    void close() {
        if (closed_) return;
        closed_ = true;
        write_chunk_buffer();
    }

    uint64_t chunk_count() const { return chunk_count_; }

  private:
    void write_chunk_buffer() {
        if (chunk_buffer_.empty()) return;
        if (chunk_offset_ - last_chunk_ != chunk_buffer_.size())
            throw std::logic_error("wrong chunk size");
        ++chunk_count_;
        last_chunk_ = chunk_offset_;
        sink_(chunk_offset_, chunk_buffer_);
        chunk_buffer_.clear();
    }

    Sink sink_;
    Chunker chunker_;
    std::vector<uint8_t> chunk_buffer_;
    uint64_t chunk_offset_ = 0, last_chunk_ = 0, chunk_count_ = 0;
    bool closed_ = false;
};

using Digest = std::array<uint8_t, 32>;

inline Digest sha256(const uint8_t* data, size_t len) {
    Digest d;
    pbs_sha256(data, len, d.data());
    return d;
}

// SHA-256 of every chunk [bounds[i], bounds[i+1]) of a device-resident stream (stream
// bytes [base, base + len) at dev), optionally keyed (SHA-256(chunk || id_key)).
inline std::vector<Digest> digest_chunks_device(const uint8_t* dev, size_t len, uint64_t base,
                                                const std::vector<uint64_t>& bounds,
                                                const std::vector<uint8_t>& key = {},
                                                void* hip_stream = nullptr) {
    const size_t n = bounds.size() > 1 ? bounds.size() - 1 : 0;
    std::vector<Digest> out(n);
    if (!n) return out;
    const int rc = pbs_digest_chunks_device(dev, len, base, bounds.data(), n,
                                            key.empty() ? nullptr : key.data(), key.size(),
                                            out[0].data(), hip_stream);
    if (rc != PBS_OK) throw std::runtime_error(std::string("pbs_digest_chunks_device: ") + pbs_strerror(rc));
    return out;
}

// CRC-32 (crc32fast) of every chunk [bounds[i], bounds[i+1]) of a device-resident stream:
// the blob CRC of an uncompressed chunk blob (DataBlob::compute_crc, data_blob.rs:70-75).
inline std::vector<uint32_t> crc32_chunks_device(const uint8_t* dev, size_t len, uint64_t base,
                                                 const std::vector<uint64_t>& bounds,
                                                 void* hip_stream = nullptr) {
    const size_t n = bounds.size() > 1 ? bounds.size() - 1 : 0;
    std::vector<uint32_t> out(n);
    if (!n) return out;
    const int rc = pbs_crc32_chunks_device(dev, len, base, bounds.data(), n, out.data(), hip_stream);
    if (rc != PBS_OK) throw std::runtime_error(std::string("pbs_crc32_chunks_device: ") + pbs_strerror(rc));
    return out;
}

// Host CRC-32, continuable like crc32fast::Hasher::update (crc = 0 to start).
inline uint32_t crc32(const uint8_t* data, size_t len, uint32_t crc = 0) { return pbs_crc32(crc, data, len); }

// DataBlob::encode(data, None, compress = false) (data_blob.rs:159-174) with a known CRC:
// UNCOMPRESSED_BLOB_MAGIC_1_0 || crc LE || data; throws above MAX_BLOB_SIZE like the
// reference's bail! (data_blob.rs:92-94).
inline std::vector<uint8_t> blob_encode_uncompressed(const uint8_t* data, size_t len, uint32_t crc) {
    std::vector<uint8_t> out(len + PBS_BLOB_HEADER_SIZE);
    if (pbs_blob_encode_uncompressed(data, len, crc, out.data(), out.size()) != out.size())
        throw std::invalid_argument("data blob too large (" + std::to_string(len) + " bytes).");
    return out;
}

// SHA-256 of every chunk [bounds[i], bounds[i+1]) of a host buffer (stream bytes
// [base, base + len)) on `threads` host threads (0: all), optionally keyed.
inline std::vector<Digest> digest_chunks_host(const uint8_t* data, size_t len, uint64_t base,
                                              const std::vector<uint64_t>& bounds,
                                              const std::vector<uint8_t>& key = {}, int threads = 0) {
    const size_t n = bounds.size() > 1 ? bounds.size() - 1 : 0;
    std::vector<Digest> out(n);
    if (!n) return out;
    const int rc = pbs_digest_chunks_host(data, len, base, bounds.data(), n, key.empty() ? nullptr : key.data(),
                                          key.size(), out[0].data(), threads);
    if (rc != PBS_OK) throw std::runtime_error(std::string("pbs_digest_chunks_host: ") + pbs_strerror(rc));
    return out;
}

// The client's upload path over a whole host buffer (pbs_pipeline_host): chunk END
// offsets (the tail included), the per-chunk digests and, with crc, the uncompressed
// blobs' CRC-32s; copies to HBM, chunking and digests overlapped on the GPU and host cores.
struct PipelineResult {
    std::vector<uint64_t> ends;
    std::vector<Digest> digests;
    std::vector<uint32_t> crcs;
    pbs_pipeline_timing timing;
};
inline PipelineResult pipeline_host(const uint8_t* data, size_t len, size_t avg, size_t piece = (size_t)1 << 30,
                                    const std::vector<uint8_t>& key = {}, bool crc = true, int digest_cus = 64) {
    // pbs_chunker_cuts_bound without a handle: every chunk but the tail >= max(avg / 4, 65)
    const size_t cap = len / std::max<size_t>(avg >> 2, 65) + 4;
    PipelineResult r;
    r.ends.resize(cap);
    r.digests.resize(cap);
    if (crc) r.crcs.resize(cap);
    size_t n = 0;
    const int rc = pbs_pipeline_host(avg, data, len, piece, key.empty() ? nullptr : key.data(), key.size(),
                                     digest_cus, r.ends.data(), r.digests[0].data(),
                                     crc ? r.crcs.data() : nullptr, cap, &n, &r.timing);
    if (rc == PBS_ERR_NOT_POW2) throw std::invalid_argument("chunk size is not a power of two");
    if (rc != PBS_OK) throw std::runtime_error(std::string("pbs_pipeline_host: ") + pbs_strerror(rc));
    r.ends.resize(n);
    r.digests.resize(n);
    if (crc) r.crcs.resize(n);
    return r;
}

// DynamicIndexWriter (dynamic_index.rs:297-391): add_chunk(end offset, digest) per chunk,
// close() writes the .didx file (tmp file + rename) and returns index_csum.
class DynamicIndexWriter {
  public:
    explicit DynamicIndexWriter(std::string path, std::array<uint8_t, 16> uuid = {},
                                int64_t ctime = (int64_t)std::time(nullptr))
        : path_(std::move(path)), uuid_(uuid), ctime_(ctime) {}

    void add_chunk(uint64_t offset, const Digest& digest) {
        if (closed_) throw std::runtime_error("cannot write to closed dynamic index file " + path_);
        ends_.push_back(offset);
        digests_.insert(digests_.end(), digest.begin(), digest.end());
    }

    Digest close() {
        if (closed_) throw std::runtime_error("cannot close already closed archive index file " + path_);
        closed_ = true;
        std::vector<uint8_t> image(pbs_didx_size(ends_.size()));
        Digest csum;
        const int rc = pbs_didx_build(ends_.data(), digests_.data(), ends_.size(), uuid_.data(),
                                      ctime_, image.data(), image.size(), csum.data());
        if (rc != PBS_OK) throw std::runtime_error(std::string("pbs_didx_build: ") + pbs_strerror(rc));
        std::string tmp = path_;
        const size_t dot = tmp.find_last_of('.');
        tmp = (dot == std::string::npos ? tmp : tmp.substr(0, dot)) + ".tmp_didx";
        std::FILE* f = std::fopen(tmp.c_str(), "wb");
        if (!f) throw std::runtime_error("cannot create " + tmp);
        const bool ok = std::fwrite(image.data(), 1, image.size(), f) == image.size();
        if (std::fclose(f) != 0 || !ok) throw std::runtime_error("write failed: " + tmp);
        if (std::rename(tmp.c_str(), path_.c_str()) != 0)
            throw std::runtime_error("Atomic rename file " + path_ + " failed");
        return csum;
    }

  private:
    std::string path_;
    std::array<uint8_t, 16> uuid_;
    int64_t ctime_;
    std::vector<uint64_t> ends_;
    std::vector<uint8_t> digests_;
    bool closed_ = false;
};

}  // namespace pbs
