// Client upload path on a host-resident stream: ChunkStream's
// chunking (pbs-client/src/chunk_stream.rs:40-77) and the per-chunk digest of the upload
// stream (pbs-client/src/backup_writer.rs:671-678), overlapped on one MI355X:
//
//   copy thread   pageable host pieces -> HBM (hipMemcpyAsync on its own stream; the DMA
//                 engines, no CUs)
//   main thread   chunker over each resident piece (find_cuts_device on a stream
//                 CU-masked to CUs [digest_cus, n)); every completed chunk is routed at
//                 once: to the GPU's digest queue -- a persistent grid on CUs
//                 [0, digest_cus) that takes jobs as they are published
//                 (pbs_digest.hip sha256_queue_kernel) -- or to the host threads
//
// The CU split keeps the persistent scan kernel and the long-running digest workgroups
// apart: a scan workgroup (130 KiB LDS, 2 x 208 VGPRs per SIMD) cannot share a CU with a
// digest workgroup, and a digest launch lasts as long as its longest chunk's serial
// hash (~0.6 s for a 16 MiB chunk), so without the split a scan launch would wait for it.
//   routing       one GPU lane walks a chunk's serial SHA-256 chain at ~25-35 MB/s, a host
//                 thread (SHA extensions, pbs_sha_host.cpp) at ~2.5 GB/s per chunk, ~4.4
//                 with four chunks in step, but there are only ~14 of them.  A chunk goes to
//                 the GPU when its chain ends before the copy does (now + len / 15 MB/s <=
//                 the copy's projected end + slack; the assumed rate is below the lane's so
//                 the host takes more of the late chunks), else to
//                 the host threads (straight from the caller's buffer; all-zero chunks once
//                 per length).  So early chunks of any length hash on the GPU under the
//                 copy, and only the long chunks found near the end load the host
//                 (round 3 sent every chunk >= 8 MiB to the host and digested the rest in
//                 four quarter-stream launches: the last launch's 8 MiB chains and the
//                 host's quarter-sized bursts ran ~240 ms past the last copy;
//                 scripts/pipe_sim.py models both).  PBS_PIPE_HOST_MIN=<bytes> restores the
//                 fixed length threshold.
// The blob CRC-32 of every chunk (HBM-bound, milliseconds) still runs as a few large
// launches on the other digest streams.
// C ABI: include/pbs_digest.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <memory>
#include <thread>
#include <unordered_set>
#include <vector>

#include "pbs_blob.h"
#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"
#include "dev_arena.h"
#include "host_share.h"
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

// Everything a call sets up, kept per device between calls (pbs_pipeline_release frees the
// idle ones): the device buffers (a stream-sized one among them -- allocating 64 GiB right
// after freeing 64 GiB cost 2.5 s, profiles/r04/pipeline/sweep_r04j.log), the chunker
// handle, the CU-masked streams, the copy events and the pinned job array.  Setting these
// up and tearing them down cost ~75 ms per 64 GiB call beside its 1.4 s (r04k bench.log:
// wall 1471 ms, total_ms 1395).
struct PipeArea {
    explicit PipeArea(int d) : dev(d), mem(d) {}
    ~PipeArea() {
        if (c) pbs_chunker_free(c);  // before its stream goes away
        drop_streams();
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (hq) (void)hipHostFree(hq);
    }
    void drop_streams() {
        if (s_copy) (void)hipStreamDestroy(s_copy);
        if (s_scan) (void)hipStreamDestroy(s_scan);
        if (s_up) (void)hipStreamDestroy(s_up);
        if (s_dh) (void)hipStreamDestroy(s_dh);
        if (s_full) (void)hipStreamDestroy(s_full);
        s_up = s_dh = s_full = nullptr;
        for (auto& s : s_dig)
            if (s) {
                pbs::release_stream_counter(s);
                (void)hipStreamDestroy(s);
            }
        s_copy = s_scan = nullptr;
        for (auto& s : s_dig) s = nullptr;
        dig = -1;
    }
    int dev;
    pbs::DevArena mem;  // slots: 0 stream, 1 digests, 2 bounds, 3 order, 4 CRCs, 5 queue state
    pbs_chunker* c = nullptr;
    size_t avg = 0;
    int dig = -1;  // digest CUs the streams are masked for
    hipStream_t s_copy = nullptr, s_scan = nullptr, s_up = nullptr, s_dh = nullptr, s_full = nullptr,
                s_dig[kDigestStreams] = {};
    std::vector<hipEvent_t> ev;
    uint8_t* hq = nullptr;
    size_t hq_bytes = 0;
};

struct PipePool {
    std::mutex mu;
    std::map<int, std::vector<PipeArea*>> idle;
};

PipePool& pipe_pool() {
    static PipePool* p = [] {
        pbs::add_reclaim_hook(&pbs_pipeline_release);  // idle work areas go when memory runs out
        return new PipePool();  // never destroyed: no HIP calls at exit
    }();
    return *p;
}

PipeArea* pipe_acquire(int dev) {
    PipePool& p = pipe_pool();
    {
        std::lock_guard<std::mutex> g(p.mu);
        std::vector<PipeArea*>& v = p.idle[dev];
        if (!v.empty()) {
            PipeArea* a = v.back();
            v.pop_back();
            return a;
        }
    }
    return new PipeArea(dev);
}

// back to the pool after a good call; after a failed one (state unknown) it is freed
void pipe_release(PipeArea* a, bool good) {
    if (!good) {
        delete a;
        return;
    }
    PipePool& p = pipe_pool();
    std::lock_guard<std::mutex> g(p.mu);
    p.idle[a->dev].push_back(a);
}

}  // namespace

extern "C" void pbs_pipeline_release(void) {
    PipePool& p = pipe_pool();
    std::map<int, std::vector<PipeArea*>> v;
    {
        std::lock_guard<std::mutex> g(p.mu);
        v.swap(p.idle);
    }
    int cur = -1;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    for (auto& kv : v)
        for (PipeArea* a : kv.second)
            if (hipSetDevice(kv.first) == hipSuccess) delete a;
    if (have) (void)hipSetDevice(cur);
}

namespace {

// pbs_upload_stream_host's part after the digests (see upload_stage)
struct UploadExt {
    const uint8_t* known;
    size_t n_known;
    int compress;
    uint8_t* known_out;
    uint8_t* blobs;
    size_t blobs_cap;
    uint64_t* blob_offsets;
    uint8_t* compressed;
    pbs_upload_timing* t;
    // `spec`: the known test, the encoding and the blobs' copy run per piece beside the
    // copies (pipeline_run's upload worker); upload_stage then only checks and counts
    bool spec = false;
    uint8_t* d_blobs = nullptr;
    size_t n_done = 0;  // chunks whose known flag, blob range and compressed flag are out
    double known_ms = 0, enc_ms = 0, d2h_ms = 0;
    pbs_blob_encode_timing enc_t{};
    int enc_rc = PBS_OK;
};

int upload_stage(UploadExt& x, pbs::DevArena* area, const uint8_t* d_data, size_t len, const uint64_t* ends,
                 const uint8_t* digests, size_t n, hipStream_t st);

int pipeline_run(size_t avg, const uint8_t* host, size_t len, size_t piece, const uint8_t* key, size_t key_len,
                 int digest_cus, uint64_t* ends, uint8_t* digests, uint32_t* crcs, size_t cap, size_t* n_out,
                 pbs_pipeline_timing* timing, UploadExt* ext) {
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
    if (__builtin_popcountll(avg) != 1) return PBS_ERR_NOT_POW2;  // as pbs_chunker_new
    if (cap < len / std::max<size_t>(avg >> 2, 65) + 3) return PBS_ERR_CAPACITY;  // pbs_chunker_cuts_bound
    const size_t npieces = (len + piece - 1) / piece;
    int rc = PBS_OK;
    auto hip_ok = [&](hipError_t e) {
        if (e != hipSuccess && rc == PBS_OK) rc = PBS_ERR_HIP;
        return e == hipSuccess;
    };
    // the device's work area (the first call on a device, or after pbs_pipeline_release,
    // creates it); returned to the pool when this call ends
    PipeArea* A = pipe_acquire(dev);
    struct Return {
        PipeArea* a;
        const int& rc;
        ~Return() { pipe_release(a, rc == PBS_OK); }
    } give_back{A, rc};
    if (!A->c || A->avg != avg) {
        if (A->c) pbs_chunker_free(A->c);
        int err = PBS_OK;
        A->c = pbs_chunker_new(avg, &err);
        A->avg = A->c ? avg : 0;
        if (!A->c) return rc = err;
    } else if (pbs::chunker_rewind(A->c) != PBS_OK) {
        return rc = PBS_ERR_HIP;
    }
    pbs_chunker* const c = A->c;
    bool ok = true;
    if (A->dig != dig) {  // CU masks for this split
        A->drop_streams();
        ok = hip_ok(hipStreamCreateWithFlags(&A->s_copy, hipStreamNonBlocking)) &&
             hip_ok(masked_stream(&A->s_scan, dig, ncu - dig, ncu)) &&
             hip_ok(masked_stream(&A->s_up, dig, ncu - dig, ncu)) &&
             hip_ok(hipStreamCreateWithFlags(&A->s_dh, hipStreamNonBlocking)) &&
             hip_ok(hipStreamCreateWithFlags(&A->s_full, hipStreamNonBlocking));
        for (auto& s : A->s_dig) ok = ok && hip_ok(masked_stream(&s, 0, dig, ncu));
        if (ok) A->dig = dig;
    }
    while (ok && A->ev.size() < npieces) {
        hipEvent_t e = nullptr;
        ok = hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (ok) A->ev.push_back(e);
    }
    hipStream_t const s_copy = A->s_copy, s_scan = A->s_scan;
    hipStream_t* const s_dig = A->s_dig;
    const std::vector<hipEvent_t>& ev_copied = A->ev;
    // device: the stream, the digests, and per-launch bounds/order (<= cap + npieces + 1)
    pbs::DevArena* const area = &A->mem;
    uint8_t* d_data = nullptr;
    uint8_t* d_dig = nullptr;
    uint64_t* d_bounds = nullptr;
    uint32_t* d_order = nullptr;
    uint32_t* d_crc = nullptr;
    if (ok) {
        d_data = area->get<uint8_t>(0, len, false);
        d_dig = area->get<uint8_t>(1, cap * 32);
        d_bounds = area->get<uint64_t>(2, (cap + npieces + 1) * 8);
        d_order = area->get<uint32_t>(3, std::max<size_t>(cap, 1) * 4);
        if (crcs) d_crc = area->get<uint32_t>(4, std::max<size_t>(cap, 1) * 4);
        if (!d_data || !d_dig || !d_bounds || !d_order || (crcs && !d_crc)) {
            ok = false;
            rc = PBS_ERR_NOMEM;
        }
    }
    ok = ok && pbs_chunker_set_stream(c, s_scan) == PBS_OK &&
         pbs_chunker_set_cu_count(c, ncu - dig) == PBS_OK;
    if (!ok && rc == PBS_OK) rc = PBS_ERR_HIP;
    // the digest queue: control word + jobs in pinned coherent host memory (the GPU reads
    // them over PCIe), its claim counter and mirror in device memory
    uint64_t* q_ctl = nullptr;
    pbs::DigestJob* q_jobs = nullptr;
    pbs::DigestQueueDev* d_q = nullptr;
    std::atomic<bool> q_running{false};
    const size_t hq_need = 64 + std::max<size_t>(cap, 1) * sizeof(pbs::DigestJob);
    if (ok && A->hq_bytes < hq_need) {
        if (A->hq) (void)hipHostFree(A->hq);
        A->hq = nullptr;
        A->hq_bytes = 0;
        if (hipHostMalloc((void**)&A->hq, hq_need, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess)
            A->hq_bytes = hq_need;
        else
            A->hq = nullptr;
    }
    uint8_t* const hqmem = A->hq;
    if (ok && (!hqmem || !(d_q = area->get<pbs::DigestQueueDev>(5, sizeof(pbs::DigestQueueDev))))) {
        ok = false;
        rc = PBS_ERR_NOMEM;
    }
    uint64_t* q_ctl_dev = nullptr;
    pbs::DigestJob* q_jobs_dev = nullptr;
    if (ok) {
        q_ctl = reinterpret_cast<uint64_t*>(hqmem);
        q_jobs = reinterpret_cast<pbs::DigestJob*>(hqmem + 64);
        __atomic_store_n(q_ctl, 0ull, __ATOMIC_RELEASE);
        ok = hip_ok(hipHostGetDevicePointer((void**)&q_ctl_dev, q_ctl, 0)) &&
             hip_ok(hipHostGetDevicePointer((void**)&q_jobs_dev, q_jobs, 0)) &&
             hip_ok(hipMemsetAsync(d_q, 0, sizeof(pbs::DigestQueueDev), s_dig[0]));
        q_running = ok;
    }
    // two workgroups (48 KiB LDS each) per digest CU.  The grid stays resident until the final
    // count -- nothing on this path may wait for the whole device meanwhile (the chunker's
    // buffers retire instead of hipFree, the CRC tables load on their own stream) -- or until
    // PBS_PIPE_IDLE_MS (50 ms) pass without a new job; it is launched again when jobs come
    // after such an exit, and jobs it never took are hashed on the host at the end.  The
    // queue's stream is a blocking one (CU-masked streams take no flags), so null-stream work
    // of another thread waits for the grid while the grid waits for this thread's next
    // publish, which may wait for that work (a blocking scan stream): the idle exit bounds
    // such a cycle to 50 ms (round 4's 10 s turned it into a stall;
    // tests/test_gpu_digest.py::test_pipeline_beside_null_stream_work)
    const int q_wgs = (int)env_u64("PBS_PIPE_QUEUE_WGS", (uint64_t)dig * 2);
    const uint64_t q_idle = env_u64("PBS_PIPE_IDLE_MS", 50) * 100000ull;  // wall_clock64: 100 MHz
    std::atomic<uint64_t> q_launches{0};
    // a launch skipped because the grid was still resident: it may have been on its idle
    // exit and leave the jobs just published, so the next tries (the next piece, the upload
    // worker's wait, the final drain) launch it again once it has gone
    std::atomic<bool> relaunch_due{false};
    std::mutex qmu;  // launches come from this thread and the upload worker
    auto q_launch_locked = [&]() {
        if (!q_running) return;
        if (q_launches && hipStreamQuery(s_dig[0]) == hipErrorNotReady) {  // still resident
            relaunch_due = true;
            return;
        }
        relaunch_due = false;
        if (pbs::launch_sha256_queue(d_data, key, key_len, q_jobs_dev, q_ctl_dev, d_q, d_dig, q_wgs, q_idle,
                                     s_dig[0]) == hipSuccess)
            ++q_launches;
        else
            q_running = false;  // the host hashes what the queue did not take
    };
    auto q_launch = [&]() {
        std::lock_guard<std::mutex> g(qmu);
        q_launch_locked();
    };
    uint64_t nj = 0;  // jobs published

    const Clock::time_point t0 = Clock::now();
    const bool dbg = std::getenv("PBS_PIPE_DEBUG") != nullptr;
    std::vector<std::pair<uint64_t, double>> pubs;  // debug (PBS_PIPE_DEBUG)
    auto publish = [&](bool final) {
        pubs.emplace_back(nj | (final ? pbs::kDigestQueueFinal : 0ull), ms_since(t0));
        // the job records before the count, and the count out of the store buffers at once
        // (without the fences the GPU's polls saw a count published ms earlier for the rest
        // of the run)
        __builtin_ia32_sfence();
        __atomic_store_n(q_ctl, nj | (final ? pbs::kDigestQueueFinal : 0ull), __ATOMIC_SEQ_CST);
        __builtin_ia32_sfence();
    };
    std::atomic<size_t> copied{0};
    std::atomic<bool> copy_failed{false};
    std::mutex mu;
    std::condition_variable cv;
    double h2d_ms = 0;
    // host share: the chunks routed to the host threads, hashed from `host` by a pool fed
    // in stream order.  Routing (see the top): PBS_PIPE_HOST_MIN = a fixed length threshold
    // instead (0: no host share); PBS_PIPE_GPU_MBS = the GPU lane rate the routing assumes
    // (15; a lane runs ~25 MB/s beside the scan and the copies, 36 alone: the lower figure
    // hands the host more of the late chunks, which it hashes four in step per thread);
    // PBS_PIPE_SLACK_MS = how far past the copy's projected end a GPU chain may run (10).
    // Same-process sweeps over the 64 GiB stream (scripts/pipe_sweep.py): with one chunk at a
    // time per host thread (profiles/r04/pipeline/) 25/20 -> 1329 ms, 30/20 -> 1385, 35/40 ->
    // 1490, 20/0 -> 1353, the fixed 8 MiB threshold 1528; with four in step
    // (profiles/r04/sha_lanes/) 25/20 -> 1321-1326, 20/0 -> 1279, 10-17 MB/s with 0-10 ms ->
    // 1240-1256
    const uint64_t host_min = env_u64("PBS_PIPE_HOST_MIN", ~0ull);
    const double gpu_bpms = (double)env_u64("PBS_PIPE_GPU_MBS", 15) * 1e3;  // bytes per ms
    const double slack_ms = (double)env_u64("PBS_PIPE_SLACK_MS", 10);
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int hthreads = host_min ? (int)env_u64("PBS_PIPE_HOST_THREADS", (uint64_t)std::max(1, std::min(hw, 16) - 2)) : 0;
    double host_done_at = 0;
    std::vector<uint8_t> hmask;  // 1 = digest computed on the host
    std::vector<std::thread> hpool;
    hmask.assign(ok ? cap : 0, 0);
    // the host threads' queue and zero-chunk memo (host_share.h); the upload path's encoder
    // waits per chunk for its digest: a host-routed chunk's flag there, a GPU job's `done` in
    // the job record; dig_final once every digest is in `digests`
    pbs::HostShare hs(host, ends, digests, ok ? cap : 0, key, key_len, t0);
    std::vector<uint64_t> jobof(ok ? cap : 0, 0);
    std::atomic<bool> dig_final{false};
    auto host_work = [&] { hs.work(); };
    if (ok && hthreads > 0)
        for (int j = 0; j < hthreads; ++j) hpool.emplace_back(host_work);
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
            // the copies have landed: this thread hashes host-routed chunks too
            if (hthreads > 0) host_work();
        });
    }

    // the upload's per-piece stage (UploadExt::spec): for each piece's chunks, as the main
    // loop finds them -- wait for their digests, the known-chunk test against the previous
    // index and the earlier chunks of the stream (the client's HashSet, backup_writer.rs:
    // 677-697), encode the new chunks' blobs on the scan partition's CUs (its own stream,
    // after the piece's copy), and copy them out to their final place in the caller's buffer;
    // all of it beside the next pieces' copies.  PBS_UPLOAD_SPEC=0: the whole stage after the
    // pipeline (upload_stage's other path).
    std::deque<std::array<size_t, 3>> upq;  // {first chunk, end chunk, piece}
    std::mutex upmu;
    std::condition_variable upcv;
    bool updone = false;
    std::thread upw;
    if (ok && ext && env_u64("PBS_UPLOAD_SPEC", 1) != 0) {
        // every chunk's blob (the early encode writes the whole batch: <= len + 12 per chunk)
        // plus up to 15 bytes of alignment per batch (a batch holds >= 1 chunk): 27 per chunk
        const size_t bcap = len + 28 * cap + 64;
        ext->d_blobs = area->get<uint8_t>(9, bcap, false);
        if (ext->d_blobs) {
            ext->spec = true;
            hipStream_t const su_masked = A->s_up, sdh = A->s_dh, su_full = A->s_full;
            upw = std::thread([&, bcap, su_masked, sdh, su_full] {
                (void)hipSetDevice(dev);
                struct DigHash {
                    size_t operator()(const std::array<uint8_t, 32>& d) const {
                        uint64_t h;
                        std::memcpy(&h, d.data(), 8);
                        return (size_t)h;
                    }
                };
                std::unordered_set<std::array<uint8_t, 32>, DigHash> seen, prev;
                for (size_t q = 0; q < ext->n_known; ++q) {
                    std::array<uint8_t, 32> d;
                    std::memcpy(d.data(), ext->known + 32 * q, 32);
                    prev.insert(d);
                }
                uint64_t hoff = 0;  // the caller's buffer: bytes of blobs so far
                uint64_t dbase = 0;  // the device area: where this batch's blobs go (the copies
                                     // out of earlier batches may still be running on sdh)
                std::vector<uint64_t> spans, offm;
                std::vector<uint8_t> compm, gdig;
                std::vector<size_t> fresh;
                ext->blob_offsets[0] = 0;
                for (;;) {
                    std::array<size_t, 3> b;
                    {
                        std::unique_lock<std::mutex> g(upmu);
                        upcv.wait(g, [&] { return updone || !upq.empty(); });
                        if (upq.empty()) break;
                        b = upq.front();
                        upq.pop_front();
                    }
                    if (ext->enc_rc != PBS_OK) continue;  // drain after an error
                    if (dbase > bcap) {  // (cannot happen with the bound above; never wrap bcap - dbase)
                        ext->enc_rc = PBS_ERR_CAPACITY;
                        continue;
                    }
                    const size_t i0 = b[0], i1 = b[1], m = i1 - i0;
                    // the scan partition's CUs while the digest queue holds the others; every CU
                    // once all digests are in (compressible streams encode past the copies' end)
                    hipStream_t const su = dig_final.load(std::memory_order_acquire) ? su_full : su_masked;
                    // encode: every chunk of the batch before its digests are in when there is
                    // no previous index (a full backup: nearly all new; the blobs are ready when
                    // the test is), else only the new ones after the test
                    auto encode = [&](const std::vector<uint64_t>& sp, size_t cnt) -> int {
                        offm.assign(cnt + 1, 0);
                        compm.assign(std::max<size_t>(cnt, 1), 0);
                        if (!cnt) return PBS_OK;
                        const Clock::time_point te = Clock::now();
                        pbs_blob_encode_timing bt{};
                        int r = hipStreamWaitEvent(su, ev_copied[b[2]], 0) == hipSuccess ? PBS_OK : PBS_ERR_HIP;
                        if (r == PBS_OK)
                            r = pbs_blob_encode_spans_device(d_data, len, 0, sp.data(), cnt, ext->compress,
                                                             ext->d_blobs + dbase, bcap - dbase, offm.data(), nullptr,
                                                             compm.data(), &bt, su);
                        ext->enc_ms += ms_since(te);
                        ext->enc_t.compress_ms += bt.compress_ms;
                        ext->enc_t.assemble_ms += bt.assemble_ms;
                        ext->enc_t.crc_ms += bt.crc_ms;
                        ext->enc_t.bytes_in += bt.bytes_in;
                        ext->enc_t.bytes_out += bt.bytes_out;
                        ext->enc_t.blocks += bt.blocks;
                        return r;
                    };
                    const bool early = ext->n_known == 0;
                    if (early) {
                        spans.resize(2 * m);
                        for (size_t k = 0; k < m; ++k) {
                            spans[2 * k] = i0 + k ? ends[i0 + k - 1] : 0;
                            spans[2 * k + 1] = ends[i0 + k];
                        }
                        const int r = encode(spans, m);
                        if (r != PBS_OK) {
                            ext->enc_rc = r;
                            continue;
                        }
                    }
                    // the batch's digests: host-routed ones by their flags, GPU jobs by theirs
                    const Clock::time_point tw = Clock::now();
                    bool fin = false;
                    for (unsigned spin = 0;; ++spin) {
                        fin = dig_final.load(std::memory_order_acquire);
                        if (fin) break;
                        if (spin % 64 == 63 && relaunch_due.load(std::memory_order_relaxed)) q_launch();
                        bool all = true;
                        for (size_t i = i0; i < i1 && all; ++i)
                            all = hmask[i] ? hs.flag(i)
                                           : __atomic_load_n(&q_jobs[jobof[i]].done, __ATOMIC_ACQUIRE) != 0;
                        if (all) break;
                        std::this_thread::sleep_for(std::chrono::microseconds(20));
                    }
                    if (!fin) {  // the GPU's digests of the batch from device memory
                        gdig.resize(m * 32);
                        if (hipMemcpyAsync(gdig.data(), d_dig + 32 * i0, m * 32, hipMemcpyDeviceToHost, su) != hipSuccess ||
                            hipStreamSynchronize(su) != hipSuccess) {
                            ext->enc_rc = PBS_ERR_HIP;
                            continue;
                        }
                    }
                    fresh.clear();
                    std::vector<uint64_t> fsp;
                    for (size_t i = i0; i < i1; ++i) {
                        std::array<uint8_t, 32> d;
                        std::memcpy(d.data(), (fin || hmask[i]) ? digests + 32 * i : gdig.data() + 32 * (i - i0), 32);
                        const bool kn = prev.count(d) || !seen.insert(d).second;
                        ext->known_out[i] = kn ? 1 : 0;
                        if (!kn) {
                            fresh.push_back(i);
                            fsp.push_back(i ? ends[i - 1] : 0);
                            fsp.push_back(ends[i]);
                        }
                    }
                    ext->known_ms += ms_since(tw);
                    const size_t mf = fresh.size();
                    int r = PBS_OK;
                    std::vector<uint64_t> dev_off(mf), blen(mf);  // the new blobs in the device area
                    std::vector<uint8_t> bcomp(mf);
                    if (early) {
                        for (size_t q = 0; q < mf; ++q) {
                            const size_t k = fresh[q] - i0;
                            dev_off[q] = offm[k];
                            blen[q] = offm[k + 1] - offm[k];
                            bcomp[q] = compm[k];
                        }
                    } else {
                        r = encode(fsp, mf);
                        for (size_t q = 0; q < mf && r == PBS_OK; ++q) {
                            dev_off[q] = offm[q];
                            blen[q] = offm[q + 1] - offm[q];
                            bcomp[q] = compm[q];
                        }
                    }
                    uint64_t bytes = 0;
                    for (size_t q = 0; q < mf; ++q) bytes += blen[q];
                    if (r == PBS_OK && hoff + bytes > ext->blobs_cap) r = PBS_ERR_CAPACITY;
                    // out in runs of blobs adjacent in the device area, to their final place, on
                    // their own stream (the encoder has synced su: the blobs are complete), not
                    // waited for here -- the next batch encodes beside them
                    const Clock::time_point td = Clock::now();
                    uint64_t h = hoff;
                    for (size_t q = 0; q < mf && r == PBS_OK;) {
                        size_t e = q + 1;
                        while (e < mf && dev_off[e] == dev_off[e - 1] + blen[e - 1]) ++e;
                        const uint64_t nbytes = dev_off[e - 1] + blen[e - 1] - dev_off[q];
                        if (nbytes && hipMemcpyAsync(ext->blobs + h, ext->d_blobs + dbase + dev_off[q], nbytes,
                                                     hipMemcpyDeviceToHost, sdh) != hipSuccess)
                            r = PBS_ERR_HIP;
                        h += nbytes;
                        q = e;
                    }
                    ext->d2h_ms += ms_since(td);
                    dbase = (dbase + offm.back() + 15) & ~15ull;
                    if (r != PBS_OK) {
                        ext->enc_rc = r;
                        continue;
                    }
                    size_t k = 0;
                    uint64_t run = hoff;
                    for (size_t i = i0; i < i1; ++i) {
                        const bool fr = k < mf && fresh[k] == i;
                        if (fr) run += blen[k];
                        ext->blob_offsets[i + 1] = run;
                        if (ext->compressed) ext->compressed[i] = fr ? bcomp[k] : 0;
                        k += fr ? 1 : 0;
                    }
                    hoff = run;
                    ext->n_done = i1;
                }
                const Clock::time_point td = Clock::now();
                if (hipStreamSynchronize(sdh) != hipSuccess && ext->enc_rc == PBS_OK) ext->enc_rc = PBS_ERR_HIP;
                ext->d2h_ms += ms_since(td);
            });
        }
    }
    auto up_finish = [&] {  // every path: the encoder thread ends before its state does
        if (!upw.joinable()) return;
        {
            std::lock_guard<std::mutex> g(upmu);
            updone = true;
        }
        upcv.notify_all();
        upw.join();
    };

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
        if (dbg && ms_since(tk) > 20.0) {
            pbs_timing tt{};
            pbs_chunker_last_timing(c, &tt);
            std::fprintf(stderr, "piece %zu: find_cuts_device %.3f ms (at %.3f ms; scan %.3f fused %llu scan_pass %llu)\n",
                         k, ms_since(tk), ms_since(t0), tt.scan_ms, (unsigned long long)tt.fused,
                         (unsigned long long)tt.scan_pass);
        }
        if (r != PBS_OK) {
            rc = r;
            break;
        }
        if (n + m > cap) {
            rc = PBS_ERR_CAPACITY;
            break;
        }
        const size_t n0 = n;
        if (m) {
            std::memcpy(ends + n, tmp.data(), m * 8);
            n += m;
        }

        // route the chunks completed in this piece: the GPU's digest queue when the chain
        // ends before the copy's projected end (+ slack), else the host threads
        if (n > n0) {
            const double now = ms_since(t0);
            // projected end of the copy: the rate at which pieces have become resident so
            // far (this loop waits for each piece's copy), ~55 GB/s before two pieces
            const double t_end = pbs::projected_copy_end(len, off + pn, k, now, slack_ms);
            size_t nh = 0;
            for (size_t i = n0; i < n; ++i) {
                const uint64_t s0 = i ? ends[i - 1] : 0, cl = ends[i] - s0;
                const bool to_host = pbs::route_to_host(hthreads, host_min, now, cl, gpu_bpms, t_end);
                if (to_host) {
                    hmask[i] = 1;
                    ++nh;
                } else {
                    q_jobs[nj].start = s0;
                    q_jobs[nj].len = cl;
                    q_jobs[nj].idx = i;
                    q_jobs[nj].done = 0;
                    jobof[i] = nj;
                    ++nj;
                }
            }
            publish(false);  // the jobs above were written before the count (release)
            if (nj) q_launch();  // (again, if the grid went idle and exited)
            if (nh) hs.push(hmask.data(), n0, n);
        }
        // the upload's encoder takes this piece's chunks (routed: their digests will come)
        if (upw.joinable() && n > n0) {
            {
                std::lock_guard<std::mutex> g(upmu);
                upq.push_back({n0, n, k});
            }
            upcv.notify_one();
        }
        // the blob CRC of the chunks completed since the last launch once they cover dbatch
        // bytes (or at the end), on the digest streams other than the queue's
        const uint64_t done_to = n ? ends[n - 1] : 0;
        const bool last = k + 1 == npieces;
        if (crcs && n > launched && (done_to - start >= dbatch || last)) {
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
            hipStream_t sd = s_dig[1 + launches % (kDigestStreams - 1)];
            if (!hip_ok(hipMemcpyAsync(d_bounds + nb, b.data(), (mm + 1) * 8, hipMemcpyHostToDevice, sd)) ||
                !hip_ok(hipMemcpyAsync(d_order + launched, o.data(), mm * 4, hipMemcpyHostToDevice, sd)))
                break;
            const int cr = pbs_crc32_chunks_async(d_data, len, 0, d_bounds + nb, d_order + launched, mm,
                                                  d_crc + launched, sd);
            if (cr != PBS_OK) {
                rc = cr;
                break;
            }
            ++launches;
            nb += mm + 1;
            launched = n;
            start = done_to;
        }
        last_chunk_at = ms_since(t0);
    }
    if (q_running) publish(true);  // every path: the queue grid drains
    if (relaunch_due) q_launch();
    if (q_launches && rc != PBS_OK) (void)hipStreamSynchronize(s_dig[0]);  // before its memory goes
    hs.finish();
    // the routing is done: this thread hashes what is left of the host share, beside the
    // pool and the copy thread (16 threads in the drain instead of 14)
    if (hthreads > 0 && rc == PBS_OK) host_work();
    if (copier.joinable()) copier.join();
    std::vector<uint8_t> gdig;
    double gpu_done_at = 0;
    if (rc == PBS_OK && ok) {
        for (int i = 0; i < kDigestStreams; ++i) hip_ok(hipStreamSynchronize(s_dig[i]));
        {
            // no launch after this point; one still due (the grid exited before the final
            // count and left jobs) runs now, drained, before the digests are read
            std::lock_guard<std::mutex> g(qmu);
            if (relaunch_due) {
                q_launch_locked();
                hip_ok(hipStreamSynchronize(s_dig[0]));
            }
            q_running = false;
        }
        gpu_done_at = ms_since(t0);
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
    // error paths too: nothing of this call may still run when the work area returns to
    // the pool (no hipFree any more to wait for it), and the upload worker launches nothing
    // from here on
    {
        std::lock_guard<std::mutex> g(qmu);
        q_running = false;
    }
    for (hipStream_t s : {s_copy, s_scan, s_dig[0], s_dig[1], s_dig[2], s_dig[3]})
        if (s) (void)hipStreamSynchronize(s);
    if (!host_done_at && hs.chunks()) host_done_at = ms_since(t0);
    pbs::DigestQueueDev qd{};
    if (q_launches) (void)hipMemcpy(&qd, d_q, sizeof qd, hipMemcpyDeviceToHost);
    // jobs the queue grid never took (it drains after stall_ticks without a new job, e.g.
    // a caller stalled between pieces for that long): hashed here, so no digest is lost
    if (rc == PBS_OK && qd.next < nj) {
        std::atomic<uint64_t> nx{qd.next};
        auto work = [&] {
            for (uint64_t j; (j = nx.fetch_add(1)) < nj;)
                pbs::sha256_host_one(host + q_jobs[j].start, q_jobs[j].len, key, key_len, digests + 32 * q_jobs[j].idx);
        };
        std::vector<std::thread> fb;
        for (int t = 1; t < std::max(1, hthreads); ++t) fb.emplace_back(work);
        work();
        for (auto& th : fb) th.join();
    }
    dig_final.store(true, std::memory_order_release);
    up_finish();
    // the upload's part after the digests: known-chunk test and blobs, from the HBM copy
    // (on the copy stream: not CU-masked, idle since the last piece landed)
    if (ext && rc == PBS_OK) rc = upload_stage(*ext, area, d_data, len, ends, digests, n, s_copy);
    const double total = ms_since(t0);
    if (timing) {
        timing->total_ms = total;
        timing->h2d_ms = h2d_ms;
        timing->chunk_ms = chunk_ms;
        timing->drain_ms = total - last_chunk_at;
        timing->bytes = len;
        timing->chunks = n;
        timing->pieces = npieces;
        timing->host_chunks = hs.chunks();
        timing->host_bytes = hs.bytes();
        timing->host_done_ms = host_done_at;
        timing->host_threads = hthreads;
        timing->gpu_jobs = nj;
        timing->gpu_claimed = qd.next;
        timing->queue_launches = q_launches;
        timing->gpu_done_ms = gpu_done_at;
        timing->host_work_ms = hs.last_done_us() / 1000.0;
        if (std::getenv("PBS_PIPE_DEBUG")) {
            std::fprintf(stderr, "digest queue: jobs %llu claimed %llu launches %llu mirror %llx polls %llu last_h %llx; seen:",
                         (unsigned long long)nj, qd.next, (unsigned long long)q_launches.load(), qd.mirror, qd.polls,
                         qd.last_h);
            for (unsigned long long i = 0; i < qd.nseen && i < 16; ++i)
                std::fprintf(stderr, " %llx@%.3fms", qd.seen[i], (qd.seen_t[i] - qd.seen_t[0]) / 1e5);
            std::fprintf(stderr, " | host publishes:");
            for (auto& pr : pubs) std::fprintf(stderr, " %llx@%.3fms", (unsigned long long)pr.first, pr.second);
            std::fprintf(stderr, " | last chunk at %.3f ms\n", last_chunk_at);
        }
    }
    *n_out = n;
    return rc;  // the work area goes back to the pool (give_back)
}

// backup_writer.rs:677-706 for every chunk of the stream, on the GPU from the HBM copy the
// pipeline made: the known-chunk test (previous index + earlier chunks of this stream), then
// DataBlob::encode(chunk, None, compress) of the new chunks (data_blob.rs:139-176), their
// blobs copied back to back into the caller's host buffer in chunk order; a known chunk's
// blob is empty.  UploadStats (backup_writer.rs:56-64): size_compressed = the blobs' raw
// sizes (`chunk.raw_size()`, :699).
int upload_stage(UploadExt& x, pbs::DevArena* area, const uint8_t* d_data, size_t len, const uint64_t* ends,
                 const uint8_t* digests, size_t n, hipStream_t st) {
    pbs_upload_timing* const t = x.t;
    if (x.spec) {
        // done per piece beside the copies (pipeline_run's upload worker): count it up
        if (x.enc_rc != PBS_OK) return x.enc_rc;
        if (x.n_done != n) return PBS_ERR_HIP;
        uint64_t size_reused = 0, compressed_chunks = 0, reused = 0;
        for (size_t i = 0; i < n; ++i) {
            if (x.known_out[i]) {
                size_reused += ends[i] - (i ? ends[i - 1] : 0);
                ++reused;
            }
            if (x.compressed) compressed_chunks += x.compressed[i];
        }
        if (t) {
            t->known_ms = x.known_ms;  // (these three beside the copies, summed per piece)
            t->encode_ms = x.enc_ms;
            t->d2h_ms = x.d2h_ms;
            t->blob = x.enc_t;
            t->chunk_count = n;
            t->chunk_reused = reused;
            t->size = len;
            t->size_reused = size_reused;
            t->size_compressed = x.blob_offsets[n];
            t->compressed_chunks = compressed_chunks;
        }
        return PBS_OK;
    }
    const Clock::time_point t0 = Clock::now();
    uint8_t* const d_dig = area->get<uint8_t>(6, std::max<size_t>(n, 1) * 32);
    uint8_t* const d_kn = area->get<uint8_t>(7, std::max<size_t>(x.n_known, 1) * 32);
    uint8_t* const d_fl = area->get<uint8_t>(8, std::max<size_t>(n, 1));
    if (!d_dig || !d_kn || !d_fl) return PBS_ERR_NOMEM;
    if (hipMemcpyAsync(d_dig, digests, n * 32, hipMemcpyHostToDevice, st) != hipSuccess ||
        (x.n_known && hipMemcpyAsync(d_kn, x.known, x.n_known * 32, hipMemcpyHostToDevice, st) != hipSuccess))
        return PBS_ERR_HIP;
    size_t reused = 0;
    int rc = pbs_known_chunks_device(d_dig, n, x.n_known ? d_kn : nullptr, x.n_known, d_fl, &reused, st);
    if (rc != PBS_OK) return rc;
    if (hipMemcpyAsync(x.known_out, d_fl, n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return PBS_ERR_HIP;
    const Clock::time_point t1 = Clock::now();
    // the new chunks as spans of the stream
    std::vector<uint64_t> spans;
    std::vector<size_t> idx;
    uint64_t size_reused = 0, new_bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t a = i ? ends[i - 1] : 0, b = ends[i];
        if (x.known_out[i]) {
            size_reused += b - a;
            continue;
        }
        spans.push_back(a);
        spans.push_back(b);
        idx.push_back(i);
        new_bytes += b - a;
    }
    const size_t m = idx.size();
    const size_t bound = 12 * m + new_bytes;
    uint8_t* const d_blobs = area->get<uint8_t>(9, std::max<size_t>(bound, 1), false);
    if (!d_blobs) return PBS_ERR_NOMEM;
    std::vector<uint64_t> offm(m + 1, 0);
    std::vector<uint8_t> compm(std::max<size_t>(m, 1), 0);
    rc = pbs_blob_encode_spans_device(d_data, len, 0, spans.data(), m, x.compress, d_blobs, bound, offm.data(),
                                      nullptr, compm.data(), t ? &t->blob : nullptr, st);
    if (rc != PBS_OK) return rc;
    const Clock::time_point t2 = Clock::now();
    if (offm[m] > x.blobs_cap) return PBS_ERR_CAPACITY;
    if (offm[m] && (hipMemcpyAsync(x.blobs, d_blobs, offm[m], hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess))
        return PBS_ERR_HIP;
    // every chunk's blob range (a known chunk's is empty) and compressed flag
    size_t k = 0;
    x.blob_offsets[0] = 0;
    uint64_t compressed_chunks = 0;
    for (size_t i = 0; i < n; ++i) {
        const bool fresh = k < m && idx[k] == i;
        x.blob_offsets[i + 1] = fresh ? offm[k + 1] : x.blob_offsets[i];
        if (x.compressed) x.compressed[i] = fresh ? compm[k] : 0;
        compressed_chunks += fresh ? compm[k] : 0;
        k += fresh ? 1 : 0;
    }
    if (t) {
        t->known_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        t->encode_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
        t->d2h_ms = ms_since(t2);
        t->chunk_count = n;
        t->chunk_reused = reused;
        t->size = len;
        t->size_reused = size_reused;
        t->size_compressed = offm[m];
        t->compressed_chunks = compressed_chunks;
    }
    return PBS_OK;
}

}  // namespace

extern "C" int pbs_pipeline_host(size_t avg, const uint8_t* host, size_t len, size_t piece,
                                 const uint8_t* key, size_t key_len, int digest_cus,
                                 uint64_t* ends, uint8_t* digests, uint32_t* crcs, size_t cap,
                                 size_t* n_out, pbs_pipeline_timing* timing) {
    return pipeline_run(avg, host, len, piece, key, key_len, digest_cus, ends, digests, crcs, cap, n_out, timing,
                        nullptr);
}

extern "C" int pbs_upload_stream_host(size_t avg, const uint8_t* host, size_t len, size_t piece,
                                      const uint8_t* key, size_t key_len, int digest_cus,
                                      const uint8_t* known, size_t n_known, int compress, uint64_t* ends,
                                      uint8_t* digests, uint8_t* is_known, size_t cap, size_t* n_out,
                                      uint8_t* blobs, size_t blobs_cap, uint64_t* blob_offsets,
                                      uint8_t* compressed, pbs_upload_timing* timing) {
    if (!is_known || !blob_offsets || (n_known && !known) || (blobs_cap && !blobs)) return PBS_ERR_INVALID;
    if (timing) std::memset(timing, 0, sizeof(*timing));
    blob_offsets[0] = 0;
    const Clock::time_point t0 = Clock::now();
    UploadExt x{known, n_known, compress, is_known, blobs, blobs_cap, blob_offsets, compressed, timing};
    const int rc = pipeline_run(avg, host, len, piece, key, key_len, digest_cus, ends, digests, nullptr, cap, n_out,
                                timing ? &timing->pipe : nullptr, len ? &x : nullptr);
    if (timing) timing->total_ms = ms_since(t0);
    return rc;
}
