// Per-device work areas reused across calls of the synchronous device entry points
// (blob encoding, digests, CRCs, the known-chunk test): a call leases an arena of the
// stream's device, takes its buffers by slot (grown with hipMalloc only when the call
// needs more than the arena holds), and returns the arena when it has synchronised its
// stream.  So in steady state a call makes no hipMalloc / hipFree (hipFree synchronises
// the whole device, stalling every other handle's stream), concurrent calls on one device
// get different arenas (no process-wide lock around the work), and calls on different
// devices never touch each other's memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <map>
#include <mutex>
#include <vector>

namespace pbs {

// every arena buffer allocation of the process (pbs_debug_arena_allocs: tests check that a
// repeated call allocates nothing)
inline std::atomic<uint64_t> g_arena_allocs{0};

class ArenaPool;
// Every pool of the process, and other keepers of idle device memory (the pipeline's work
// areas): when an allocation fails, the idle memory of all of them is freed and the
// allocation tried once more -- one large call (a 64 GiB pipeline or blob stage) must not
// make the next, different call fail until someone calls a *_release.
struct Reclaimers {
    std::mutex mu;
    std::vector<ArenaPool*> pools;
    std::vector<void (*)()> hooks;
};
inline Reclaimers& reclaimers() {
    static Reclaimers* r = new Reclaimers;  // never destroyed
    return *r;
}
inline void add_reclaim_hook(void (*f)()) {
    Reclaimers& r = reclaimers();
    std::lock_guard<std::mutex> g(r.mu);
    for (auto h : r.hooks)
        if (h == f) return;
    r.hooks.push_back(f);
}
inline void reclaim_idle_device_memory();  // below ArenaPool

class DevArena {
public:
    explicit DevArena(int dev) : dev_(dev) {}
    ~DevArena() { free_all(); }
    int dev() const { return dev_; }
    // slot `i`'s buffer of at least `bytes` (the calling thread's current device must be
    // dev()); grows by 1/8 headroom so slowly growing calls do not reallocate every time
    // (`headroom` false: exactly `bytes`, for stream-sized slots of tens of GiB)
    template <typename T>
    T* get(unsigned i, size_t bytes, bool headroom = true) {
        if (bytes == 0) bytes = 1;
        if (bufs_.size() <= i) bufs_.resize(i + 1);
        Buf& b = bufs_[i];
        if (b.cap < bytes) {
            if (b.p) (void)hipFree(b.p);
            b.p = nullptr;
            b.cap = 0;
            const size_t want = headroom ? bytes + bytes / 8 : bytes;
            if (hipMalloc(&b.p, want) != hipSuccess) {
                (void)hipGetLastError();
                // (this arena is leased: not among the idle ones).  The hipFrees wait for the
                // whole device: inside a pipeline run that includes its own resident digest
                // queue grid, which drains on its idle exit (50 ms) -- a stall, taken only
                // when device memory has run out, instead of a failed call
                reclaim_idle_device_memory();
                if (hipMalloc(&b.p, want) != hipSuccess) {
                    (void)hipGetLastError();
                    b.p = nullptr;
                    return nullptr;
                }
            }
            b.cap = want;
            ++grows_;
            g_arena_allocs.fetch_add(1, std::memory_order_relaxed);
        }
        return static_cast<T*>(b.p);
    }
    // timing events, created once per arena
    hipEvent_t event(unsigned i) {
        if (ev_.size() <= i) ev_.resize(i + 1, nullptr);
        if (!ev_[i] && hipEventCreate(&ev_[i]) != hipSuccess) ev_[i] = nullptr;
        return ev_[i];
    }
    uint64_t grows() const { return grows_; }
    size_t bytes() const {
        size_t s = 0;
        for (const Buf& b : bufs_) s += b.cap;
        return s;
    }
    void free_all() {
        for (Buf& b : bufs_)
            if (b.p) (void)hipFree(b.p);
        bufs_.clear();
        for (hipEvent_t e : ev_)
            if (e) (void)hipEventDestroy(e);
        ev_.clear();
    }

private:
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
    };
    int dev_;
    std::vector<Buf> bufs_;
    std::vector<hipEvent_t> ev_;
    uint64_t grows_ = 0;
};

// The idle arenas of one kind of call, per device.
class ArenaPool {
public:
    ArenaPool() {
        Reclaimers& r = reclaimers();
        std::lock_guard<std::mutex> g(r.mu);
        r.pools.push_back(this);
    }
    DevArena* acquire(int dev) {
        {
            std::lock_guard<std::mutex> g(mu_);
            std::vector<DevArena*>& v = idle_[dev];
            if (!v.empty()) {
                DevArena* a = v.back();
                v.pop_back();
                ++leased_;
                return a;
            }
            ++leased_;
        }
        return new DevArena(dev);
    }
    void release(DevArena* a) {
        std::lock_guard<std::mutex> g(mu_);
        idle_[a->dev()].push_back(a);
        --leased_;
    }
    // frees every idle arena, each on its own device (arenas leased by running calls are
    // not touched: they return to the pool afterwards)
    void clear() {
        std::map<int, std::vector<DevArena*>> v;
        {
            std::lock_guard<std::mutex> g(mu_);
            v.swap(idle_);
        }
        int cur = -1;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        for (auto& kv : v)
            for (DevArena* a : kv.second) {
                if (hipSetDevice(kv.first) == hipSuccess) delete a;
            }
        if (have) (void)hipSetDevice(cur);
    }
    size_t idle(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        return idle_[dev].size();
    }

private:
    std::mutex mu_;
    std::map<int, std::vector<DevArena*>> idle_;
    long leased_ = 0;
};

inline void reclaim_idle_device_memory() {
    std::vector<ArenaPool*> pools;
    std::vector<void (*)()> hooks;
    {
        Reclaimers& r = reclaimers();
        std::lock_guard<std::mutex> g(r.mu);
        pools = r.pools;
        hooks = r.hooks;
    }
    for (ArenaPool* p : pools) p->clear();
    for (auto h : hooks) h();
}

// Scoped lease: the arena goes back to the pool at the end of the call.
class ArenaLease {
public:
    ArenaLease(ArenaPool& p, int dev) : p_(p), a_(p.acquire(dev)) {}
    ~ArenaLease() { p_.release(a_); }
    DevArena* operator->() { return a_; }
    DevArena& operator*() { return *a_; }

private:
    ArenaPool& p_;
    DevArena* a_;
};

}  // namespace pbs
