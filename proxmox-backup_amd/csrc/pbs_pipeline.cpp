// Client upload path on a host-resident stream: ChunkStream's
// chunking (pbs-client/src/chunk_stream.rs:40-77) and the per-chunk digest of the upload
// stream (pbs-client/src/backup_writer.rs:671-678), overlapped on one MI355X:
//
//   copy thread   pageable host pieces -> HBM (hipMemcpyAsync on its own stream; the DMA
//                 engines, no CUs)
//   main thread   chunker over each resident piece (find_cuts_device on a stream
//                 CU-masked to CUs [digest_cus, n)); the completed chunks go to per-chunk
//                 SHA-256 launches on four digest streams CU-masked to CUs [0, digest_cus)
//
// The CU split keeps the persistent scan kernel and the long-running digest workgroups
// apart: a scan workgroup (130 KiB LDS, 2 x 208 VGPRs per SIMD) cannot share a CU with a
// digest workgroup, and a digest launch lasts as long as its longest chunk's serial
// hash (~0.6 s for a 16 MiB chunk), so without the split a scan launch would wait for it.
// The chunks are digested in a few large launches (a quarter of the stream, at most
// 16 GiB each), which overlap on the four digest streams and with the later copies.
//   host threads  the LONG chunks (>= PBS_PIPE_HOST_MIN, default 8 MiB) are hashed on the
//                 host cores straight from the caller's buffer (SHA extensions,
//                 pbs_sha_host.cpp; all-zero chunks once per length), because one GPU
//                 lane walks a chunk's serial chain at ~30 MB/s: a 16 MiB chunk in the
//                 last launch kept the GPU busy ~0.6 s after the last copy.  The GPU keeps
//                 the short chunks (and every chunk's CRC).
// C ABI: include/pbs_digest.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#include "pbs_blob.h"
#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"
#include "pbs_digest.h"
#include "sha_host.h"

namespace {

using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

hipError_t masked_stream(hipStream_t* s, int first, int count, int ncu) {
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    for (int cu = first; cu < first + count && cu < ncu; ++cu) mask[cu / 32] |= 1u << (cu % 32);
    return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

constexpr int kDigestStreams = 4;

uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::strtoull(e, nullptr, 0) : dflt;
}

}  // namespace

extern "C" int pbs_pipeline_host(size_t avg, const uint8_t* host, size_t len, size_t piece,
                                 const uint8_t* key, size_t key_len, int digest_cus,
                                 uint64_t* ends, uint8_t* digests, uint32_t* crcs, size_t cap,
                                 size_t* n_out, pbs_pipeline_timing* timing) {
    if (!n_out || (len && !host) || piece == 0 || (cap && (!ends || !digests)) ||
        key_len > PBS_DIGEST_MAX_KEY || (key_len && !key))
        return PBS_ERR_INVALID;
    *n_out = 0;
    if (timing) std::memset(timing, 0, sizeof(*timing));
    if (len == 0) return PBS_OK;
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return PBS_ERR_NO_DEVICE;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 16)
        return PBS_ERR_HIP;
    const int dig = std::min(std::max(digest_cus, 4), ncu - 8);
    int err = PBS_OK;
    pbs_chunker* c = pbs_chunker_new(avg, &err);
    if (!c) return err;
    if (cap < pbs_chunker_cuts_bound(c, len)) {
        pbs_chunker_free(c);
        return PBS_ERR_CAPACITY;
    }
    const size_t npieces = (len + piece - 1) / piece;
    hipStream_t s_copy = nullptr, s_scan = nullptr, s_dig[kDigestStreams] = {};
    uint8_t* d_data = nullptr;
    uint8_t* d_dig = nullptr;
    uint64_t* d_bounds = nullptr;
    uint32_t* d_order = nullptr;
    uint32_t* d_crc = nullptr;
    std::vector<hipEvent_t> ev_copied(npieces, nullptr);
    int rc = PBS_OK;
    auto hip_ok = [&](hipError_t e) {
        if (e != hipSuccess && rc == PBS_OK) rc = PBS_ERR_HIP;
        return e == hipSuccess;
    };
    bool ok = hip_ok(hipStreamCreateWithFlags(&s_copy, hipStreamNonBlocking)) &&
              hip_ok(masked_stream(&s_scan, dig, ncu - dig, ncu));
    for (auto& s : s_dig) ok = ok && hip_ok(masked_stream(&s, 0, dig, ncu));
    for (auto& e : ev_copied) ok = ok && hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // device: the stream, the digests, and per-launch bounds/order (<= cap + npieces + 1)
    if (ok && (hipMalloc(&d_data, len) != hipSuccess || hipMalloc(&d_dig, cap * 32) != hipSuccess ||
               hipMalloc(&d_bounds, (cap + npieces + 1) * 8) != hipSuccess ||
               hipMalloc(&d_order, std::max<size_t>(cap, 1) * 4) != hipSuccess ||
               (crcs && hipMalloc(&d_crc, std::max<size_t>(cap, 1) * 4) != hipSuccess))) {
        ok = false;
        rc = PBS_ERR_NOMEM;
    }
    ok = ok && pbs_chunker_set_stream(c, s_scan) == PBS_OK &&
         pbs_chunker_set_cu_count(c, ncu - dig) == PBS_OK;
    if (!ok && rc == PBS_OK) rc = PBS_ERR_HIP;

    const Clock::time_point t0 = Clock::now();
    std::atomic<size_t> copied{0};
    std::atomic<bool> copy_failed{false};
    std::mutex mu;
    std::condition_variable cv;
    double h2d_ms = 0;
    std::thread copier;
    if (ok) {
        copier = std::thread([&] {
            const Clock::time_point tc = Clock::now();
            for (size_t k = 0; k < npieces; ++k) {
                const size_t off = k * piece, n = std::min(piece, len - off);
                if (hipMemcpyAsync(d_data + off, host + off, n, hipMemcpyHostToDevice, s_copy) !=
                        hipSuccess ||
                    hipEventRecord(ev_copied[k], s_copy) != hipSuccess) {
                    copy_failed = true;
                    break;
                }
                {
                    std::lock_guard<std::mutex> g(mu);
                    copied = k + 1;
                }
                cv.notify_one();
            }
            (void)hipStreamSynchronize(s_copy);
            h2d_ms = ms_since(tc);
            cv.notify_one();
        });
    }

    // host share: long chunks, hashed from `host` by a pool fed in stream order
    const uint64_t host_min = env_u64("PBS_PIPE_HOST_MIN", 8ull << 20);
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int hthreads = host_min ? (int)env_u64("PBS_PIPE_HOST_THREADS", (uint64_t)std::max(1, std::min(hw, 16) - 2)) : 0;
    std::deque<uint64_t> hq;  // chunk indices
    std::mutex hmu;
    std::condition_variable hcv;
    bool hdone = false;
    std::atomic<uint64_t> host_chunks{0}, host_bytes{0};
    double host_done_at = 0;
    std::vector<uint8_t> hmask;  // 1 = digest computed on the host
    std::map<uint64_t, std::array<uint8_t, 32>> zero_dig;  // digest of an all-zero chunk per length
    std::vector<std::thread> hpool;
    if (ok && hthreads > 0) {
        hmask.assign(cap, 0);
        for (int j = 0; j < hthreads; ++j)
            hpool.emplace_back([&] {
                for (;;) {
                    uint64_t i;
                    {
                        std::unique_lock<std::mutex> g(hmu);
                        hcv.wait(g, [&] { return hdone || !hq.empty(); });
                        if (hq.empty()) return;
                        i = hq.front();
                        hq.pop_front();
                    }
                    const uint64_t s0 = i ? ends[i - 1] : 0, e0 = ends[i], cl = e0 - s0;
                    uint8_t* out = digests + 32 * i;
                    const bool zero = pbs::all_zero(host + s0, cl);
                    if (zero) {  // zero extents: one hash per length
                        bool hit = false;
                        {
                            std::lock_guard<std::mutex> g(hmu);
                            auto it = zero_dig.find(cl);
                            if (it != zero_dig.end()) {
                                std::memcpy(out, it->second.data(), 32);
                                hit = true;
                            }
                        }
                        if (hit) {
                            host_chunks += 1;
                            continue;
                        }
                    }
                    pbs::sha256_host_one(host + s0, cl, key, key_len, out);
                    if (zero) {
                        std::lock_guard<std::mutex> g(hmu);
                        std::memcpy(zero_dig[cl].data(), out, 32);
                    }
                    host_chunks += 1;
                    host_bytes += e0 - s0;
                }
            });
    }
    double chunk_ms = 0, last_chunk_at = 0;
    size_t n = 0, nb = 0, launches = 0, launched = 0;
    uint64_t start = 0;  // start of the first chunk not yet digested
    // bytes of completed chunks per digest launch: a quarter of the stream, at most 16 GiB
    const uint64_t dbatch = std::max<uint64_t>(std::min<uint64_t>(len / 4, 16ull << 30), piece);
    std::vector<uint64_t> tmp(ok ? pbs_chunker_cuts_bound(c, std::min(piece, len)) + 1 : 0);
    std::vector<std::vector<uint64_t>> hb;  // host bounds/order stay alive until the end
    std::vector<std::vector<uint32_t>> ho;
    for (size_t k = 0; ok && rc == PBS_OK && k < npieces; ++k) {
        {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return copied.load() > k || copy_failed.load(); });
        }
        if (copy_failed) {
            rc = PBS_ERR_HIP;
            break;
        }
        const size_t off = k * piece, pn = std::min(piece, len - off);
        if (!hip_ok(hipStreamWaitEvent(s_scan, ev_copied[k], 0))) break;
        const Clock::time_point tk = Clock::now();
        size_t m = 0;
        const int r = pbs_chunker_find_cuts_device(c, d_data + off, pn, k + 1 == npieces, tmp.data(),
                                                   tmp.size(), &m);
        chunk_ms += ms_since(tk);
        if (r != PBS_OK) {
            rc = r;
            break;
        }
        if (n + m > cap) {
            rc = PBS_ERR_CAPACITY;
            break;
        }
        if (m) {
            std::memcpy(ends + n, tmp.data(), m * 8);
            n += m;
        }
        // digest the chunks completed since the last launch once they cover dbatch bytes
        // (or at the end): a launch lasts as long as its longest chunk's serial hash, so
        // few large launches, overlapping on the digest streams, keep the CUs busy
        const uint64_t done_to = n ? ends[n - 1] : 0;
        const bool last = k + 1 == npieces;
        if (n > launched && (done_to - start >= dbatch || last)) {
            const size_t mm = n - launched;
            hb.emplace_back(mm + 1);
            ho.emplace_back(mm);
            std::vector<uint64_t>& b = hb.back();
            std::vector<uint32_t>& o = ho.back();
            b[0] = start;
            std::memcpy(b.data() + 1, ends + launched, mm * 8);
            std::iota(o.begin(), o.end(), 0u);
            std::stable_sort(o.begin(), o.end(), [&](uint32_t x, uint32_t y) {
                return b[x + 1] - b[x] > b[y + 1] - b[y];
            });
            // the longest chunks (a prefix of o) go to the host threads
            size_t nh = 0;
            if (hthreads > 0) {
                while (nh < mm && b[o[nh] + 1] - b[o[nh]] >= host_min) ++nh;
                if (nh) {
                    {
                        std::lock_guard<std::mutex> g(hmu);
                        for (size_t q = 0; q < nh; ++q) {
                            hq.push_back(launched + o[q]);
                            hmask[launched + o[q]] = 1;
                        }
                    }
                    hcv.notify_all();
                }
            }
            hipStream_t sd = s_dig[launches % kDigestStreams];
            // o sorted longest first: the CRC launch takes all of it, the digest launch
            // the suffix after the host's prefix
            if (!hip_ok(hipMemcpyAsync(d_bounds + nb, b.data(), (mm + 1) * 8, hipMemcpyHostToDevice, sd)) ||
                !hip_ok(hipMemcpyAsync(d_order + launched, o.data(), mm * 4, hipMemcpyHostToDevice, sd)))
                break;
            if (mm > nh) {
                const int dr = pbs_digest_chunks_async(d_data, len, 0, d_bounds + nb, d_order + launched + nh,
                                                       mm - nh, key, key_len, d_dig + 32 * launched, sd);
                if (dr != PBS_OK) {
                    rc = dr;
                    break;
                }
            }
            if (crcs) {  // the blob CRC of the same chunks, behind the digests on that stream
                const int cr = pbs_crc32_chunks_async(d_data, len, 0, d_bounds + nb, d_order + launched, mm,
                                                      d_crc + launched, sd);
                if (cr != PBS_OK) {
                    rc = cr;
                    break;
                }
            }
            ++launches;
            nb += mm + 1;
            launched = n;
            start = done_to;
        }
        last_chunk_at = ms_since(t0);
    }
    if (copier.joinable()) copier.join();
    {
        std::lock_guard<std::mutex> g(hmu);
        hdone = true;
    }
    hcv.notify_all();
    std::vector<uint8_t> gdig;
    if (rc == PBS_OK && ok) {
        for (auto& s : s_dig) hip_ok(hipStreamSynchronize(s));
        if (rc == PBS_OK && n) {
            if (hpool.empty()) {
                hip_ok(hipMemcpy(digests, d_dig, n * 32, hipMemcpyDeviceToHost));
            } else {  // the GPU's digests, merged around the host's
                gdig.resize(n * 32);
                if (hip_ok(hipMemcpy(gdig.data(), d_dig, n * 32, hipMemcpyDeviceToHost))) {
                    for (auto& th : hpool) th.join();
                    hpool.clear();
                    host_done_at = ms_since(t0);
                    for (size_t i = 0; i < n; ++i)
                        if (!hmask[i]) std::memcpy(digests + 32 * i, gdig.data() + 32 * i, 32);
                }
            }
        }
        if (rc == PBS_OK && n && crcs) hip_ok(hipMemcpy(crcs, d_crc, n * 4, hipMemcpyDeviceToHost));
    }
    for (auto& th : hpool) th.join();  // error paths
    if (!host_done_at && host_chunks) host_done_at = ms_since(t0);
    const double total = ms_since(t0);
    if (timing) {
        timing->total_ms = total;
        timing->h2d_ms = h2d_ms;
        timing->chunk_ms = chunk_ms;
        timing->drain_ms = total - last_chunk_at;
        timing->bytes = len;
        timing->chunks = n;
        timing->pieces = npieces;
        timing->host_chunks = host_chunks;
        timing->host_bytes = host_bytes;
        timing->host_done_ms = host_done_at;
        timing->host_threads = hthreads;
    }
    *n_out = n;
    for (auto& e : ev_copied)
        if (e) (void)hipEventDestroy(e);
    for (void* p : {(void*)d_data, (void*)d_dig, (void*)d_bounds, (void*)d_order, (void*)d_crc})
        if (p) (void)hipFree(p);
    pbs_chunker_free(c);  // before its stream goes away
    if (s_copy) (void)hipStreamDestroy(s_copy);
    if (s_scan) (void)hipStreamDestroy(s_scan);
    for (auto& s : s_dig)
        if (s) {
            pbs::release_stream_counter(s);
            (void)hipStreamDestroy(s);
        }
    return rc;
}
