// The host share of the pipeline's per-chunk digests (pbs_pipeline.cpp): the routing rule
// and the pool of host threads that hash the chunks routed to them, straight from the
// caller's buffer.  Plain C++ (no HIP types), so the threaded part links and runs without
// a device -- the sanitizer builds (Makefile `sanitize`, tests/cpp/host_sanitize.cpp)
// drive it with ASan + UBSan and TSan.
//
// The reference gets this safety from the type system: the chunker and the upload stream
// are moved into tokio tasks (proxmox-backup-client/src/main.rs:206-211) and the digest
// is computed per chunk on the stream (pbs-client/src/backup_writer.rs:671-678).
#pragma once
#include <stdint.h>

#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>

#include "sha_host.h"

namespace pbs {

// Routing of a completed chunk of `cl` bytes, found `now_ms` after the call began: to the
// host threads when its serial GPU chain (at gpu_bpms bytes per ms) would end after the
// copy's projected end t_end_ms (deadline rule), or -- host_min != ~0, PBS_PIPE_HOST_MIN --
// when it is at least host_min bytes long.  Without host threads everything goes to the GPU.
inline bool route_to_host(int host_threads, uint64_t host_min, double now_ms, uint64_t cl, double gpu_bpms,
                          double t_end_ms) {
    if (host_threads <= 0) return false;
    if (host_min == ~0ull) return now_ms + (double)cl / gpu_bpms > t_end_ms;
    return cl >= host_min;
}

// The copy's projected end (ms after the call began): the rate at which pieces became
// resident so far (`resident` bytes at now_ms, k pieces in), ~55 GB/s before two pieces,
// plus the slack a GPU chain may run past it.
inline double projected_copy_end(uint64_t len, uint64_t resident, size_t k, double now_ms, double slack_ms) {
    const double rate = k >= 1 && now_ms > 0 ? (double)resident / now_ms : 55e6;  // bytes per ms
    return (double)len / rate + slack_ms;
}

// Chunk i of the stream is [ends[i - 1], ends[i]) (ends[-1] = 0) of `host`; its digest
// goes to digests + 32 i.  The producer (the pipeline's main thread) appends to `ends`
// and then push()es the routed indices; workers (work(), any number of threads) take them
// in stream order until finish() and an empty queue, up to four in step per thread
// (sha256_host_lanes); an all-zero chunk is hashed once per length and copied after that.
// flag(i) turns 1 (release) once chunk i's digest is written -- the upload's encoder waits
// on it.
class HostShare {
public:
    using Clock = std::chrono::steady_clock;
    HostShare(const uint8_t* host, const uint64_t* ends, uint8_t* digests, size_t cap, const uint8_t* key,
              size_t key_len, Clock::time_point t0)
        : host_(host), ends_(ends), digests_(digests), key_(key), key_len_(key_len), t0_(t0),
          flag_(new std::atomic<uint8_t>[cap ? cap : 1]()) {}

    // chunks [i0, i1) of which mask[i] != 0 are the host's
    void push(const uint8_t* mask, size_t i0, size_t i1) {
        {
            std::lock_guard<std::mutex> g(mu_);
            for (size_t i = i0; i < i1; ++i)
                if (mask[i]) q_.push_back(i);
        }
        cv_.notify_all();
    }
    // the routing is done: workers return once the queue is empty
    void finish() {
        {
            std::lock_guard<std::mutex> g(mu_);
            done_ = true;
        }
        cv_.notify_all();
    }
    // one worker (returns after finish() once nothing is left)
    void work() {
        auto next = [&](ShaJob& j, bool block) {
            for (;;) {
                uint64_t i;
                {
                    std::unique_lock<std::mutex> g(mu_);
                    if (block) cv_.wait(g, [&] { return done_ || !q_.empty(); });
                    if (q_.empty()) return false;
                    i = q_.front();
                    q_.pop_front();
                }
                const uint64_t s0 = i ? ends_[i - 1] : 0, cl = ends_[i] - s0;
                uint8_t* out = digests_ + 32 * i;
                const bool zero = all_zero(host_ + s0, cl);
                if (zero) {
                    std::lock_guard<std::mutex> g(mu_);
                    auto it = zero_dig_.find(cl);
                    if (it != zero_dig_.end()) {
                        std::memcpy(out, it->second.data(), 32);
                        chunks_ += 1;
                        flag_[i].store(1, std::memory_order_release);
                        continue;
                    }
                }
                j = ShaJob{host_ + s0, cl, out, zero ? 1ull : 0ull};
                return true;
            }
        };
        auto done = [&](const ShaJob& j) {
            if (j.tag) {
                std::lock_guard<std::mutex> g(mu_);
                std::memcpy(zero_dig_[j.len].data(), j.out, 32);
            }
            chunks_ += 1;
            bytes_ += j.len;
            flag_[(size_t)(j.out - digests_) / 32].store(1, std::memory_order_release);
            const uint64_t us =
                (uint64_t)(std::chrono::duration<double, std::micro>(Clock::now() - t0_).count());
            for (uint64_t cur = work_us_.load(); us > cur && !work_us_.compare_exchange_weak(cur, us);) {
            }
        };
        sha256_host_lanes(next, done, key_, key_len_);
    }
    bool flag(size_t i) const { return flag_[i].load(std::memory_order_acquire) != 0; }
    uint64_t chunks() const { return chunks_.load(); }
    uint64_t bytes() const { return bytes_.load(); }
    uint64_t last_done_us() const { return work_us_.load(); }  // the last digest (us after t0)

private:
    const uint8_t* host_;
    const uint64_t* ends_;
    uint8_t* digests_;
    const uint8_t* key_;
    size_t key_len_;
    Clock::time_point t0_;
    std::unique_ptr<std::atomic<uint8_t>[]> flag_;
    std::deque<uint64_t> q_;  // chunk indices
    std::mutex mu_;
    std::condition_variable cv_;
    bool done_ = false;
    std::map<uint64_t, std::array<uint8_t, 32>> zero_dig_;  // digest of an all-zero chunk per length
    std::atomic<uint64_t> chunks_{0}, bytes_{0}, work_us_{0};
};

}  // namespace pbs
