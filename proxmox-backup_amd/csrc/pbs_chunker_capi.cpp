// C ABI (include/pbs_chunker.h) and host pipeline of the MI355X chunker.
//
// Reference interface replaced: pbs_datastore::Chunker (pbs-datastore/src/chunker.rs:18-186)
// and the caller loops around it (pbs-client/src/chunk_stream.rs:40-77,
// pbs-datastore/src/dynamic_index.rs:493-515, examples/test_chunk_speed.rs:25-36).
//
// Pipeline for a range of new stream bytes (DESIGN.md "Pipeline"):
//   1. scan_main_kernel   flags 128-byte blocks holding a hash candidate (HBM-bound scan)
//   2. scan_exact_kernel  exact candidate positions in flagged blocks, the stream head
//                         block and the tail that does not fill a wave tile
//   3. resolve            min/max chunk-size rule -> cut list (pointer doubling):
//                         up to kSmallResolveMax candidates one workgroup sorts and
//                         resolves in LDS and writes the cuts into mapped pinned memory;
//                         above that the in-house radix sort (pbs_sort.hip) + the
//                         multi-kernel resolve; batches >= 1 MiB at averages >= 128 KiB
//                         take the one-launch pass instead (scan_fused.h)
// Steps 1-3 run on the handle's HIP stream with ONE host sync per batch (spec_batch:
// the one-workgroup resolve reads the candidate count on the device and stands down
// when it does not fit; the host then takes the two-sync path); only the counts, the
// cut list, the open chunk's candidates and the 63-byte warm-up tail come back.
//
// `Chunker::scan` semantics (stateful, 0 or the boundary relative to the slice) are
// kept by tracking absolute offsets: consumed (caller position), chunk_start (open
// chunk), scanned_end (bytes whose candidates are known).  Re-submitted bytes are
// never rescanned.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <new>
#include <vector>

#include "buzhash_table.h"
#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"

using namespace pbs;

namespace {

// A device buffer that grows on demand.  The buffer it outgrows is retired, not freed:
// hipFree waits for the whole device (every stream of the process, e.g. the host
// pipeline's persistent digest queue), so buffers are freed only with the handle; growth
// at least doubles, so the retired ones sum to less than the live one.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    std::vector<void*> retired;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        size_t want = bytes + bytes / 4 + 256;
        if (p) {
            retired.push_back(p);
            want = std::max(want, 2 * cap);
        }
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    // the outgrown buffers (the handle is idle: no launch of it can still read them)
    void drop_retired() {
        for (void* r : retired) (void)hipFree(r);
        retired.clear();
    }
    void release() {
        drop_retired();
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

struct Params {
    uint64_t avg = 0, min = 0, max = 0, min_eff = 0, max_eff = 0;
    uint32_t mask = 0, minimum = 0, rot = 0, thr = 0;
    bool hash_cuts = false;  // false when no hash test can pass (avg == 1)
};

// chunker.rs:75-106 (+ the rotated-threshold form used by scan_main_kernel)
int make_params(uint64_t avg, Params* p) {
    if (__builtin_popcountll(avg) != 1) return PBS_ERR_NOT_POW2;
    p->avg = avg;
    p->mask = (uint32_t)(avg * 2 - 1);
    p->minimum = p->mask - 2u;
    p->min = avg >> 2;
    p->max = avg << 2;
    p->min_eff = std::max<uint64_t>(p->min, 65);  // first test at chunk_size 65 (fill phase)
    p->max_eff = std::max<uint64_t>(p->max, 65);
    p->hash_cuts = p->minimum <= p->mask;
    const int n = __builtin_popcount(p->mask);  // mask = 2^n - 1
    p->rot = (uint32_t)(32 - n) & 31u;
    if (!p->hash_cuts) {
        p->thr = 0xFFFFFFFFu;
    } else if (kScanFrame == 1) {
        // h' = rotl(h, rot): the mask bits sit on top, (h & mask) >= mask-2 <=> h' >= thr
        p->thr = p->minimum << p->rot;
    } else {
        // parity frame: odd bytes hold rotl(h, rot), even bytes
        // rotl(h, rot + 1).  A candidate has bits 2..n-1 of h set and bits 1..0 != 0, so in
        // both frames the top n-1 bits read >= 2^(n-1) - 3: one screening threshold (twice
        // the exact candidate rate; scan_exact_kernel applies the exact test)
        p->thr = n < 3 ? 0u : ((1u << (n - 1)) - 3u) << ((33u - (uint32_t)n) & 31u);
    }
    return PBS_OK;
}

inline uint32_t rotl32(uint32_t x, uint32_t r) {
    r &= 31u;
    return r ? (x << r) | (x >> (32u - r)) : x;
}

}  // namespace

// Host side of the scan server (scan_server.h): the mailbox (acknowledgement, candidates)
// in fine-grained pinned host memory; the request record and slot in fine-grained VRAM
// written through the BAR (dev_req), or in pinned host memory when the host has no
// mapping of it; the kernel on its own stream.
struct ScanServer {
    ServerMailbox* mb = nullptr;  // host view (mapped)
    ServerMailbox* mb_dev = nullptr;
    ServerReq* req = nullptr;  // host view of the request record (the mailbox's, or in VRAM)
    ServerReq* req_dev = nullptr;
    ServerDispatch* disp_dev = nullptr;  // split requests (in the VRAM allocation; none without it)
    uint8_t* slot = nullptr;  // host view
    uint8_t* slot_dev = nullptr;
    uint8_t* hslot = nullptr;  // pinned host slot (the slot itself without VRAM; else the
    uint8_t* hslot_dev = nullptr;  // requests over kServerVramMax)
    void* vram = nullptr;  // the VRAM allocation of record + slot (dev_req)
    bool dev_req = true;   // PBS_SERVER_VRAM=0: record + slot in pinned host memory (A/B)
    hipStream_t stream = nullptr;
    uint64_t seq = 0;
    bool running = false;
    bool enabled = true;  // PBS_SCAN_SERVER=0: every scan() takes the batch path (A/B)
    bool broken = false;  // a request timed out: never used again by this handle
    uint32_t n_wg = kSrvDefaultWgs;  // PBS_SERVER_WGS: workgroups (1 = the one-workgroup server)
    uint32_t epoch = 0;              // launches so far (ServerDispatch tags)
    uint64_t vram_max = kServerVramMax;  // PBS_SERVER_VRAM_MAX: longer requests use the pinned slot (A/B)
    uint32_t flags = 0;  // PBS_SERVER_POLL=4: lane 0 of every wave polls, staggered (A/B; no faster)
    // PBS_SERVER_PROBE=1: requests, host round trip (us) and the kernel's phases (ticks of
    // 10 ns: request seen -> staged -> hashed -> acknowledged), printed when the handle is freed
    uint64_t probe_n = 0;
    double probe_rtt_us = 0;
    uint64_t probe_ticks[3] = {0, 0, 0};
};

struct pbs_chunker {
    Params prm;
    // stream state (absolute offsets)
    uint64_t consumed = 0;
    uint64_t chunk_start = 0;
    uint64_t scanned_end = 0;
    uint8_t carry[64];
    uint32_t carry_len = 0;
    std::vector<uint64_t> pending;  // sorted candidates >= chunk_start, < scanned_end
    size_t pend_head = 0;
    // device
    int device = 0;
    int cu = 256;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    DevBuf d_table, d_pre, d_counters, d_susp, d_cand, d_C, d_sort_tmp, d_nxt, d_jtmp, d_nf, d_on,
        d_cnt, d_off, d_scan_tmp, d_cuts, d_res, d_in, d_stage, d_hits, d_rec, d_scratch;
    uint32_t rec_epoch = 0;  // fused pass: tile-record epoch of the last launch (16 bits)
    // fused pass returns on the resolver's status word, before its kernel has retired:
    // its scan time (ev[0] -> ev[1]) and the call's total (ev[5] -> ev[4]) are read from
    // the events when last_timing asks for them
    bool timing_pending = false;
    bool fused = true;        // PBS_FUSED=0: multi-launch path for every batch (A/B)
    bool fused_force = false; // PBS_FUSED=1: the fused pass for every batch it can serve (tests)
    bool scan_pass = true;    // PBS_SCAN_PASS=0: small averages take scan_main + exact + sort (A/B)
    uint64_t fused_min_avg = 0;
    int balance = 1;           // PBS_BALANCE=0: no priority trading between SIMD partners (A/B)
    bool direct_out = true;    // PBS_DIRECT_OUT=0: the multi-kernel resolve always copies its cuts (A/B)
    // the direct resolve's one host sync: 1 = on the event behind its last kernel, 0 = the
    // stream (PBS_SYNC_MODE, A/B: the event wait returned 10-20 us sooner per 64 GiB pass at
    // 64 / 128 KiB, profiles/r04/scanpass/sync_ab.log)
    int sync_mode = 1;
    int scan_dyn_env = -1;         // PBS_SCAN_DYN=0/1: force the static / dynamic tile order
    uint64_t fused_min_bytes = 0;  // smallest batch for the fused pass (PBS_FUSED_MIN_BYTES)  // smallest average served by the fused pass (PBS_FUSED_MIN_AVG: A/B)
    uint64_t susp_cap = 0, cand_cap = 0;
    uint64_t batch_limit = 0;  // bytes per batch (0 = batch_max); shrunk when a batch is too
                               // dense, reset at the start of every find_cuts / scan call
    bool too_dense = false;    // the last scan found more than kMaxBatchCand candidates
    uint64_t* h_small = nullptr;  // pinned + mapped: [0] counters, [8..19] results, [24..31] tail
    uint64_t* h_cuts = nullptr;   // pinned + mapped: cut list of the small resolve
    uint64_t* h_keep = nullptr;   // pinned + mapped: open-chunk candidates of the small resolve
    uint64_t* h_cand = nullptr;   // pinned + mapped: candidates of a small scan() batch
    uint8_t* h_stage = nullptr;   // pinned: carry | pending | input of a small batch
    size_t h_stage_cap = 0;
    // events: 0/1 main scan, 2 exact end, 3/4 resolve, 5 call start
    hipEvent_t ev[6] = {};
    pbs_timing timing{};
    int last_error = 0;
    bool debug_phases = false;  // PBS_DEBUG_PHASES=1: small-resolve phase times to stderr
    ScanServer srv;
    // The fused pass's resolver gives up after fused_timeout_ticks (wall_clock64, 100 MHz;
    // PBS_FUSED_TIMEOUT_TICKS, tests) and stores status 2; the host's spin on that status
    // word gives up host_wait_s after the launch (PBS_HOST_WAIT_MS; default: the kernel's
    // bound + 10 s), so a device wait that escapes the kernel's own bound fails the call
    // with PBS_ERR_HIP instead of hanging the caller.  The handle is then `lost`: a kernel
    // of it may still be running, so every call but reset / free fails with PBS_ERR_HIP,
    // reset succeeds once the handle's stream has drained, and free leaks the device
    // memory of a handle whose kernel still runs rather than wait for it.
    uint64_t fused_timeout_ticks = 100000000ull * 20;
    double host_wait_s = 0;
    bool lost = false;
};

namespace {

int fail(pbs_chunker* c, int code) {
    if (c) c->last_error = code;
    return code;
}

#define HIP_TRY(c, x)                                   \
    do {                                                \
        if ((x) != hipSuccess) return fail(c, PBS_ERR_HIP); \
    } while (0)

constexpr uint64_t kHostCuts = 1ull << 20;  // h_cuts entries (8 MiB)
constexpr uint64_t kHostKeep = 1ull << 16;  // h_keep entries
constexpr size_t kSmallBytes = 256;         // h_small bytes

// Candidates one batch may hold (the lists and the multi-kernel resolve's node arrays,
// ~60 B per candidate, stay < 8 GiB).  Candidates are bounded by the bytes, not by the
// average: data whose window hash passes the test with a short period makes every
// period-th byte one, so a denser batch is redone at a quarter of its length.
constexpr uint64_t kMaxBatchCand = 1ull << 27;

uint64_t batch_max(const pbs_chunker* c) {
    const uint64_t cap = c->prm.avg >= 4096 ? 1ull << 40 : 1ull << 30;
    return c->batch_limit ? std::min(cap, c->batch_limit) : cap;
}

// Phase A over d_data[0..len) (stream offset `base`): scan_main_kernel flags blocks,
// scan_exact_kernel writes exact candidate positions (unsorted) to c->d_cand.  The
// handle's carry (the <= 63 stream bytes before `base`) is the warm-up history.
// scan_launch only enqueues (counters -> h_small[0] as two u32); scan_collect reads them
// after the caller's sync and reports whether the suspect/candidate capacities held.
struct ScanPlan {
    uint64_t ntiles = 0, ext_first = 0, ext_count = 0, blocks = 0;
    int seg = 0, head = 0;
    bool dyn = false;        // dynamic tile order (scan_main_plan)
    uint64_t t_big = 0;      // tiles >= t_big are small (segments of seg / 4)
};

ScanPlan plan_scan(pbs_chunker* c, uint64_t len) {
    const Params& p = c->prm;
    ScanPlan sp;
    sp.seg = scan_main_plan(len, c->cu, &sp.ntiles, &sp.dyn, &sp.t_big);
    const uint64_t covered = scan_main_covered(sp.ntiles, sp.t_big, sp.seg);
    sp.head = sp.ntiles > 0 ? 1 : 0;
    sp.ext_first = covered / kBlockBytes;
    sp.ext_count = (len - covered + kBlockBytes - 1) / kBlockBytes;
    sp.blocks = (len + kBlockBytes - 1) / kBlockBytes;
    const uint64_t expected = len / p.avg * 3 / 2 + 1;
    const uint64_t want_s = std::min<uint64_t>(sp.blocks + 2, expected * 4 + 4096);
    const uint64_t want_c =
        std::min<uint64_t>(std::min<uint64_t>(len + 1, expected * 2 + 8192), kMaxBatchCand);
    c->susp_cap = std::max(c->susp_cap, want_s);
    c->cand_cap = std::max(c->cand_cap, want_c);
    return sp;
}

int scan_launch(pbs_chunker* c, const uint8_t* d_data, uint64_t len, uint64_t base,
                const ScanPlan& sp, bool copy_counts = true) {
    const Params& p = c->prm;
    HIP_TRY(c, c->d_pre.ensure(64));
    if (c->carry_len)
        HIP_TRY(c, hipMemcpyAsync(c->d_pre.p, c->carry, c->carry_len, hipMemcpyHostToDevice,
                                  c->stream));
    HIP_TRY(c, c->d_susp.ensure((size_t)c->susp_cap * 8));
    HIP_TRY(c, c->d_cand.ensure((size_t)c->cand_cap * 8));
    // counters: [0] suspects, [1] candidates (u64), [2] scan_main's tile counter (u32)
    HIP_TRY(c, c->d_counters.ensure(24));
    HIP_TRY(c, hipMemsetAsync(c->d_counters.p, 0, 24, c->stream));
    unsigned long long* d_nsusp = c->d_counters.as<unsigned long long>();
    unsigned long long* d_ncand = d_nsusp + 1;
    HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(c, launch_scan_main(d_data, sp.ntiles, sp.seg, c->d_table.as<uint32_t>(), p.thr,
                                c->d_susp.as<uint64_t>(), d_nsusp, c->susp_cap, c->cu, c->stream,
                                reinterpret_cast<uint32_t*>(d_nsusp + 2), sp.dyn, sp.t_big, c->balance != 0 && !sp.dyn));
    HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
    const uint64_t max_items = c->susp_cap + 1 + sp.ext_count;
    HIP_TRY(c, launch_scan_exact(d_data, len, c->d_pre.as<uint8_t>(), c->carry_len,
                                 c->d_susp.as<uint64_t>(), d_nsusp, c->susp_cap, sp.ext_first,
                                 sp.ext_count, sp.head, p.mask, p.minimum, base,
                                 c->d_cand.as<uint64_t>(), d_ncand, c->cand_cap, max_items,
                                 c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
    // (the speculative batch has resolve_small write them instead: one copy less)
    if (copy_counts)
        HIP_TRY(c, hipMemcpyAsync(c->h_small, c->d_counters.p, 16, hipMemcpyDeviceToHost, c->stream));
    return PBS_OK;
}

// After the sync: *ok = false (and the capacities grown) when a list overflowed.
int scan_collect(pbs_chunker* c, uint64_t len, const ScanPlan& sp, uint64_t* nsusp_out,
                 uint64_t* ncand_out, bool* ok) {
    const uint64_t nsusp = c->h_small[0], ncand = c->h_small[1];
    *ok = true;
    if (ncand > kMaxBatchCand) {  // the caller redoes the batch shorter (too_dense)
        c->too_dense = true;
        *ok = false;
        *nsusp_out = nsusp;
        *ncand_out = ncand;
        return PBS_OK;
    }
    if (nsusp > c->susp_cap) {
        c->susp_cap = std::min<uint64_t>(nsusp * 2 + 1024, sp.blocks + 2);
        *ok = false;
    }
    if (ncand > c->cand_cap) {
        c->cand_cap = std::min<uint64_t>(ncand * 2 + 1024, kMaxBatchCand);
        *ok = false;
    }
    *nsusp_out = nsusp;
    *ncand_out = ncand;
    if (!*ok) return PBS_OK;
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    c->timing.scan_ms += ms;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
    c->timing.exact_ms += ms;
    c->timing.bytes += len;
    c->timing.suspects += nsusp;
    c->timing.candidates += ncand;
    return PBS_OK;
}

int scan_candidates(pbs_chunker* c, const uint8_t* d_data, uint64_t len, uint64_t base,
                    uint64_t* ncand_out) {
    *ncand_out = 0;
    if (!c->prm.hash_cuts || len == 0) return PBS_OK;
    const ScanPlan sp = plan_scan(c, len);
    for (int attempt = 0;; ++attempt) {
        int rc = scan_launch(c, d_data, len, base, sp);
        if (rc) return rc;
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        uint64_t nsusp = 0;
        bool ok = false;
        rc = scan_collect(c, len, sp, &nsusp, ncand_out, &ok);
        if (rc) return rc;
        if (ok) return PBS_OK;
        if (c->too_dense) return PBS_OK;  // caller shrinks the batch
        if (attempt > 4) return fail(c, PBS_ERR_NOMEM);
    }
}

// Radix-sort c->d_cand[0..n) into dst (device).
int sort_candidates(pbs_chunker* c, uint64_t n, uint64_t* dst, uint64_t key_end) {
    if (n == 0) return PBS_OK;
    // keys are stream offsets < key_end: radix passes only over the bits in use
    // (36 bits for a 64 GiB stream: 5 passes instead of 8)
    const int end_bit = key_end > 1 ? 64 - __builtin_clzll(key_end - 1) : 1;
    size_t tb = 0;
    HIP_TRY(c, sort_u64(nullptr, &tb, c->d_cand.as<uint64_t>(), dst, (uint32_t)n, end_bit, c->stream));
    HIP_TRY(c, c->d_sort_tmp.ensure(tb));
    tb = c->d_sort_tmp.cap;
    HIP_TRY(c, sort_u64(c->d_sort_tmp.p, &tb, c->d_cand.as<uint64_t>(), dst, (uint32_t)n, end_bit,
                        c->stream));
    return PBS_OK;
}

// Keep the last <= 63 stream bytes before scanned_end as warm-up history.
void update_carry(pbs_chunker* c, const uint8_t* tail, uint64_t tail_len) {
    const uint32_t W = kWindow - 1;
    if (tail_len >= W) {
        std::memcpy(c->carry, tail + tail_len - W, W);
        c->carry_len = W;
        return;
    }
    uint8_t tmp[128];
    std::memcpy(tmp, c->carry, c->carry_len);
    std::memcpy(tmp + c->carry_len, tail, tail_len);
    const uint32_t tot = c->carry_len + (uint32_t)tail_len;
    const uint32_t keep = tot < W ? tot : W;
    std::memcpy(c->carry, tmp + tot - keep, keep);
    c->carry_len = keep;
}

// Upper bound on the cuts a resolve from chunk_start over m candidates up to `end` can
// emit: at most one per candidate plus the forced cuts, and at most one per 65 bytes.
uint64_t cut_bound(const pbs_chunker* c, uint64_t m, uint64_t end) {
    const uint64_t span = end > c->chunk_start ? end - c->chunk_start : 0;
    return std::min<uint64_t>(span / 65, m + span / c->prm.max_eff) + 2;
}

// After a resolve: move chunk_start to the open chunk; pending = the open chunk's
// candidates ++ older pending entries at/after `end` (not uploaded).
int finish_resolve(pbs_chunker* c, uint64_t s_open, uint64_t end, std::vector<uint64_t>& keep,
                   uint64_t ncut) {
    c->chunk_start = s_open;
    for (size_t i = c->pend_head; i < c->pending.size(); ++i)
        if (c->pending[i] >= end) keep.push_back(c->pending[i]);
    c->pending.swap(keep);
    c->pend_head = 0;
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[3], c->ev[4]));
    c->timing.resolve_ms += ms;
    c->timing.cuts += ncut;
    return PBS_OK;
}

// Resolve the min/max rule over c->d_C[0..m) (sorted, absolute) from chunk_start with
// bytes known up to `end`.  Appends cut END offsets to host `out` at *n, moves
// chunk_start to the open chunk and keeps the open chunk's candidates pending.
int ensure_small_host_bufs(pbs_chunker* c);
template <class T>
int mapped(pbs_chunker* c, T* host, T** dev);

// The device address of a host cut array the GPU can write (pinned / registered memory),
// or nullptr (pageable: the cuts go through a device buffer and a copy).  Asked every call
// (a cached answer would outlive the caller's buffer).
uint64_t* out_device_view(uint64_t* out) {
    if (!out) return nullptr;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, out) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer)
        return static_cast<uint64_t*>(at.devicePointer);
    (void)hipGetLastError();  // pageable memory: not an error here
    return nullptr;
}

// Device buffers of a multi-kernel resolve over up to m nodes.
int resolve_buffers(pbs_chunker* c, uint32_t m) {
    const uint32_t nodes = m + 2;
    HIP_TRY(c, c->d_C.ensure((size_t)nodes * 8));  // no-op: d_C already holds m entries
    HIP_TRY(c, c->d_nxt.ensure((size_t)nodes * 4));
    HIP_TRY(c, c->d_jtmp.ensure((size_t)nodes * 8));
    HIP_TRY(c, c->d_nf.ensure((size_t)nodes * 8));
    HIP_TRY(c, c->d_on.ensure((size_t)nodes * 4));
    HIP_TRY(c, c->d_cnt.ensure((size_t)nodes * 8));
    HIP_TRY(c, c->d_off.ensure((size_t)nodes * 8));
    HIP_TRY(c, c->d_res.ensure(32));
    size_t tb = 0;
    HIP_TRY(c, exclusive_sum_u64(nullptr, &tb, c->d_cnt.as<uint64_t>(), c->d_off.as<uint64_t>(), m + 1, c->stream));
    HIP_TRY(c, c->d_scan_tmp.ensure(tb));
    return PBS_OK;
}

// The multi-kernel resolve into a cut array the GPU can write (out_dev: pinned host memory):
// the emit kernel writes the cuts there, the results and the open chunk's candidates go to
// mapped host memory, and the host syncs once (the copying path: device buffers, a sync,
// copies, a second sync).  m_dev != nullptr: the node count is m_base + *m_dev on the device
// (m its upper bound) and m_base + *m_host after the sync -- the scan pass launches this
// right behind its gather, whose overflow flag (*overflow, h_small[1]) is read after the
// sync: set, nothing changed and the caller takes another path.
int resolve_direct(pbs_chunker* c, uint32_t m, const uint64_t* m_dev, uint32_t m_base,
                   const volatile uint64_t* m_host, uint64_t end, uint64_t* out_dev, size_t cap, size_t* n,
                   bool* overflow) {
    const Params& p = c->prm;
    int rc = resolve_buffers(c, m);
    if (rc) return rc;
    uint64_t *small_dev = nullptr, *keep_dev = nullptr;
    if ((rc = ensure_small_host_bufs(c)) || (rc = mapped(c, c->h_small, &small_dev)) ||
        (rc = mapped(c, c->h_keep, &keep_dev)))
        return rc;
    const uint64_t room = std::min<uint64_t>(cut_bound(c, m, end), cap - *n);
    ResolveParams rp{p.min_eff, p.max_eff, end, c->chunk_start};
    volatile uint64_t* r = c->h_small + 4;
    r[0] = r[1] = r[2] = r[3] = 0;
    HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    HIP_TRY(c, launch_resolve(c->d_C.as<uint64_t>(), m, rp, c->d_nxt.as<uint32_t>(), c->d_jtmp.as<uint32_t>(),
                              c->d_nf.as<uint64_t>(), c->d_on.as<uint32_t>(), c->d_cnt.as<uint64_t>(),
                              c->d_off.as<uint64_t>(), c->d_scan_tmp.p, c->d_scan_tmp.cap, out_dev + *n, room,
                              small_dev + 4, c->stream, m_dev, m_base));
    HIP_TRY(c, launch_resolve_keep(c->d_C.as<uint64_t>(), m, small_dev + 4, keep_dev, kHostKeep, m_dev, m_base,
                                   c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
    if (c->sync_mode == 1)
        HIP_TRY(c, hipEventSynchronize(c->ev[4]));
    else
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (overflow && (*overflow = c->h_small[1] != 0)) return PBS_OK;
    const uint64_t mm = m_dev ? m_base + *m_host : m;
    const uint64_t ncut = r[0], s_open = r[1], idx = r[2], keep_over = r[3];
    if (ncut > room) return fail(c, PBS_ERR_CAPACITY);
    std::vector<uint64_t> keep(mm > idx ? mm - idx : 0);
    if (!keep.empty()) {
        if (!keep_over) {
            std::memcpy(keep.data(), c->h_keep, keep.size() * 8);
        } else {
            HIP_TRY(c, hipMemcpyAsync(keep.data(), c->d_C.as<uint64_t>() + idx, keep.size() * 8,
                                      hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
        }
    }
    *n += ncut;
    return finish_resolve(c, s_open, end, keep, ncut);
}

int run_resolve(pbs_chunker* c, uint32_t m, uint64_t end, uint64_t* out, size_t cap, size_t* n) {
    const Params& p = c->prm;
    // a cut array the GPU can write (pinned, as bench.py hands it): resolve_direct
    uint64_t* const out_dev = c->direct_out ? out_device_view(out) : nullptr;
    if (out_dev && cap > *n) return resolve_direct(c, m, nullptr, 0, nullptr, end, out_dev, cap, n, nullptr);
    int rc = resolve_buffers(c, m);
    if (rc) return rc;
    const uint64_t out_cap = cut_bound(c, m, end);
    ResolveParams rp{p.min_eff, p.max_eff, end, c->chunk_start};
    HIP_TRY(c, c->d_cuts.ensure(out_cap * 8));
    HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    HIP_TRY(c, launch_resolve(c->d_C.as<uint64_t>(), m, rp, c->d_nxt.as<uint32_t>(),
                              c->d_jtmp.as<uint32_t>(), c->d_nf.as<uint64_t>(),
                              c->d_on.as<uint32_t>(), c->d_cnt.as<uint64_t>(),
                              c->d_off.as<uint64_t>(), c->d_scan_tmp.p, c->d_scan_tmp.cap,
                              c->d_cuts.as<uint64_t>(), out_cap, c->d_res.as<uint64_t>(),
                              c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->h_small, c->d_res.p, 24, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const uint64_t ncut = c->h_small[0], s_open = c->h_small[1], idx = c->h_small[2];
    if (*n + ncut > cap || ncut > out_cap) return fail(c, PBS_ERR_CAPACITY);
    if (ncut)
        HIP_TRY(c, hipMemcpyAsync(out + *n, c->d_cuts.p, ncut * 8, hipMemcpyDeviceToHost,
                                  c->stream));
    std::vector<uint64_t> keep(m > idx ? m - idx : 0);
    if (!keep.empty())
        HIP_TRY(c, hipMemcpyAsync(keep.data(), c->d_C.as<uint64_t>() + idx, keep.size() * 8,
                                  hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    *n += ncut;
    return finish_resolve(c, s_open, end, keep, ncut);
}

int ensure_small_host_bufs(pbs_chunker* c) {
    if (!c->h_cuts) HIP_TRY(c, hipHostMalloc((void**)&c->h_cuts, kHostCuts * 8, hipHostMallocMapped));
    if (!c->h_keep) HIP_TRY(c, hipHostMalloc((void**)&c->h_keep, kHostKeep * 8, hipHostMallocMapped));
    return PBS_OK;
}

template <class T>
int mapped(pbs_chunker* c, T* host, T** dev) {
    HIP_TRY(c, hipHostGetDevicePointer((void**)dev, host, 0));
    return PBS_OK;
}

// After a single-workgroup resolve (synchronized): cut list and open-chunk candidates
// from the mapped buffers (device copies when they did not fit).
int small_finish(pbs_chunker* c, uint32_t m, uint64_t out_cap, uint64_t end, uint64_t* out,
                 size_t cap, size_t* n) {
    const uint64_t ncut = c->h_small[8], s_open = c->h_small[9], idx = c->h_small[10];
    if (c->debug_phases)
        std::fprintf(stderr,
                     "resolve_small m=%u hist %.1f bscan %.1f scatter %.1f isort %.1f next %.1f "
                     "double %.1f scan %.1f emit %.1f copy %.1f us\n",
                     m, c->h_small[11] / 100.0, c->h_small[12] / 100.0, c->h_small[13] / 100.0,
                     c->h_small[14] / 100.0, c->h_small[15] / 100.0, c->h_small[16] / 100.0,
                     c->h_small[17] / 100.0, c->h_small[18] / 100.0, c->h_small[19] / 100.0);
    if (*n + ncut > cap || ncut > out_cap) return fail(c, PBS_ERR_CAPACITY);
    const uint64_t nkeep = m > idx ? m - idx : 0;
    std::vector<uint64_t> keep(nkeep);
    bool wait = false;
    if (ncut <= kHostCuts) {
        std::memcpy(out + *n, c->h_cuts, ncut * 8);
    } else {
        HIP_TRY(c, hipMemcpyAsync(out + *n, c->d_cuts.p, ncut * 8, hipMemcpyDeviceToHost, c->stream));
        wait = true;
    }
    if (nkeep <= kHostKeep) {
        if (nkeep) std::memcpy(keep.data(), c->h_keep, nkeep * 8);
    } else {
        HIP_TRY(c, hipMemcpyAsync(keep.data(), c->d_C.as<uint64_t>() + idx, nkeep * 8,
                                  hipMemcpyDeviceToHost, c->stream));
        wait = true;
    }
    if (wait) HIP_TRY(c, hipStreamSynchronize(c->stream));
    *n += ncut;
    return finish_resolve(c, s_open, end, keep, ncut);
}

// Single-workgroup resolve (np + nnew + 2 <= kSmallResolveMax): pending candidates are
// in d_C[0..np), the new unsorted ones in newc[0..nnew).  One host sync.
int run_resolve_small(pbs_chunker* c, const uint64_t* newc, uint32_t np, uint32_t nnew,
                      uint64_t end, uint64_t* out, size_t cap, size_t* n) {
    const Params& p = c->prm;
    const uint32_t m = np + nnew;
    HIP_TRY(c, c->d_nxt.ensure(((size_t)m + 2) * 4));
    HIP_TRY(c, c->d_nf.ensure(((size_t)m + 2) * 8));
    HIP_TRY(c, c->d_res.ensure(32));
    const uint64_t out_cap = cut_bound(c, m, end);
    HIP_TRY(c, c->d_cuts.ensure(out_cap * 8));
    int rc = ensure_small_host_bufs(c);
    if (rc) return rc;
    uint64_t *cuts_dev = nullptr, *keep_dev = nullptr, *small_dev = nullptr;
    if ((rc = mapped(c, c->h_cuts, &cuts_dev)) || (rc = mapped(c, c->h_keep, &keep_dev)) ||
        (rc = mapped(c, c->h_small, &small_dev)))
        return rc;
    HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    ResolveParams rp{p.min_eff, p.max_eff, end, c->chunk_start};
    HIP_TRY(c, launch_resolve_small(newc, nnew, c->d_C.as<uint64_t>(), np, rp,
                                    c->d_nxt.as<uint32_t>(), c->d_nf.as<uint64_t>(),
                                    c->d_cuts.as<uint64_t>(), out_cap, cuts_dev, kHostCuts,
                                    keep_dev, kHostKeep, c->d_res.as<uint64_t>(), small_dev + 8,
                                    c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return small_finish(c, m, out_cap, end, out, cap, n);
}

// Small batch (bl <= kFusedMaxBytes), stream bytes [pos, pos + bl) from host `hsrc` or
// device `dsrc`: carry | pending (| host input) are staged in pinned memory and sent with
// ONE H2D; scan_blocks_kernel + resolve_small_kernel<1> (resolve) or <2> (candidates
// only, for scan()); one host sync.  *overflow: the batch holds too many candidates for
// one workgroup -- nothing changed, the caller takes the regular path.
int fused_batch(pbs_chunker* c, const uint8_t* dsrc, const uint8_t* hsrc, uint64_t pos,
                uint64_t bl, size_t np, uint64_t rend, bool resolve, uint64_t* out, size_t cap,
                size_t* n, bool* overflow) {
    const Params& p = c->prm;
    *overflow = false;
    const size_t data_off = (64 + np * 8 + 15) & ~(size_t)15;
    const size_t stage_bytes = data_off + (hsrc ? bl : 0);
    if (stage_bytes > c->h_stage_cap) {
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        const size_t want = std::max<size_t>(stage_bytes, kFusedMaxBytes + 64 + 8 * 1024 + 16);
        HIP_TRY(c, hipHostMalloc((void**)&c->h_stage, want, hipHostMallocDefault));
        c->h_stage_cap = want;
    }
    std::memcpy(c->h_stage + 64 - c->carry_len, c->carry, c->carry_len);
    if (np) std::memcpy(c->h_stage + 64, c->pending.data() + c->pend_head, np * 8);
    // one pinned staging copy + ONE H2D beats a second H2D straight from the caller's
    // pageable buffer for pieces <= 256 KiB (34 vs 49 us per 64 KiB piece) and ties above
    if (hsrc) std::memcpy(c->h_stage + data_off, hsrc, bl);
    HIP_TRY(c, c->d_stage.ensure(stage_bytes));
    HIP_TRY(c, hipMemcpyAsync(c->d_stage.p, c->h_stage, stage_bytes, hipMemcpyHostToDevice, c->stream));
    const uint8_t* data = hsrc ? c->d_stage.as<uint8_t>() + data_off : dsrc;
    // block grid on 16-byte-aligned addresses (scan_blocks_kernel): block b starts at
    // stream offset pos - misalign + 128 b
    const uint64_t misalign = (uintptr_t)data & 15;
    const uint64_t nblk = (bl + misalign + kBlockBytes - 1) / kBlockBytes;
    HIP_TRY(c, c->d_hits.ensure(std::max<uint64_t>(nblk, 1) * 16));
    HIP_TRY(c, c->d_nxt.ensure((kSmallResolveMax + 2) * 4));
    HIP_TRY(c, c->d_nf.ensure((kSmallResolveMax + 2) * 8));
    HIP_TRY(c, c->d_C.ensure((kSmallResolveMax + 2) * 8));
    HIP_TRY(c, c->d_res.ensure(32));
    const uint64_t out_cap = cut_bound(c, kSmallResolveMax, rend);
    HIP_TRY(c, c->d_cuts.ensure(out_cap * 8));
    int rc = ensure_small_host_bufs(c);
    if (rc) return rc;
    if (!c->h_cand)
        HIP_TRY(c, hipHostMalloc((void**)&c->h_cand, kSmallResolveMax * 8, hipHostMallocMapped));
    uint64_t *cuts_dev = nullptr, *keep_dev = nullptr, *small_dev = nullptr, *cand_dev = nullptr;
    if ((rc = mapped(c, c->h_cuts, &cuts_dev)) || (rc = mapped(c, c->h_keep, &keep_dev)) ||
        (rc = mapped(c, c->h_small, &small_dev)) || (rc = mapped(c, c->h_cand, &cand_dev)))
        return rc;
    FusedScanArgs fa{data, bl, c->d_stage.as<uint8_t>() + 64 - c->carry_len, c->carry_len,
                     pos - misalign,
                     p.mask, p.minimum, c->d_hits.as<uint4>(), nblk,
                     reinterpret_cast<const uint64_t*>(c->d_stage.as<uint8_t>() + 64), cand_dev,
                     kSmallResolveMax};
    ResolveParams rp{p.min_eff, p.max_eff, rend, c->chunk_start};
    HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    HIP_TRY(c, launch_scan_resolve_small(fa, resolve ? 1 : 0, c->d_C.as<uint64_t>(), (uint32_t)np,
                                         rp, c->d_nxt.as<uint32_t>(), c->d_nf.as<uint64_t>(),
                                         c->d_cuts.as<uint64_t>(), out_cap, cuts_dev, kHostCuts,
                                         keep_dev, kHostKeep, c->d_res.as<uint64_t>(),
                                         small_dev + 8, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
    const uint64_t tl = std::min<uint64_t>(bl, kWindow - 1);
    uint8_t* tail = reinterpret_cast<uint8_t*>(c->h_small + 24);
    if (tl && !hsrc)
        HIP_TRY(c, hipMemcpyAsync(tail, dsrc + bl - tl, tl, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->h_small[20]) {
        *overflow = true;
        return PBS_OK;
    }
    c->timing.bytes += bl;
    if (resolve) {
        const uint32_t m = (uint32_t)c->h_small[21];
        c->timing.candidates += m - np;
        rc = small_finish(c, m, out_cap, rend, out, cap, n);
        if (rc) return rc;
    } else {
        const uint64_t k = c->h_small[8];
        c->timing.candidates += k;
        const size_t old = c->pending.size();
        c->pending.resize(old + k);
        std::memcpy(c->pending.data() + old, c->h_cand, k * 8);
    }
    update_carry(c, hsrc ? hsrc + bl - tl : tail, tl);
    c->scanned_end = pos + bl;
    return PBS_OK;
}

constexpr uint64_t kServerIdleTicks = 100000000ull / 1000 * 5;  // 5 ms (wall_clock64: 100 MHz)
constexpr double kServerTimeoutS = 10.0;

// Stop the scan server (quit flag, then its stream drained).  Called before any other
// device work of the handle: a hipFree elsewhere would otherwise wait for its idle exit.
void server_stop(pbs_chunker* c) {
    ScanServer& sv = c->srv;
    if (!sv.running) return;
    __atomic_store_n(&sv.req->req_len, kServerQuit, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();  // write-combined BAR stores leave now
    (void)hipStreamSynchronize(sv.stream);
    __atomic_store_n(&sv.req->req_len, 0u, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    sv.running = false;
}

int server_launch(pbs_chunker* c, uint64_t last) {
    ScanServer& sv = c->srv;
    __atomic_store_n(&sv.mb->exited, ~0ull, __ATOMIC_RELEASE);
    const uint32_t flags = sv.flags | (sv.vram ? kSrvDevReq : 0u);
    sv.epoch = (sv.epoch + 1) & 0x3FFFFFFFu;  // kSrvEpochMask (scan_server.h)
    if (!sv.epoch) sv.epoch = 1;  // 0 is the header's initial state
    HIP_TRY(c, launch_scan_server(sv.mb_dev, sv.req_dev, sv.disp_dev, sv.slot_dev, sv.hslot_dev,
                                  c->d_table.as<uint32_t>(), c->prm.thr, last, kServerIdleTicks, flags,
                                  sv.disp_dev ? sv.n_wg : 1u, sv.epoch, sv.stream));
    sv.running = true;
    return PBS_OK;
}

// Request record + slot in fine-grained VRAM that this process can store to directly (the
// GPU's BAR mapping at the allocation's own address; mb_bar.hip).  Whether the host has
// that mapping is tested without touching it: write(2) of the record into a pipe fails
// with EFAULT on an unmapped address.  Then a host store must read back through the
// runtime.  Any failure leaves sv.vram null (pinned host memory instead).
void server_map_vram(pbs_chunker* c) {  // on the handle's device (server_scan's guard)
    ScanServer& sv = c->srv;
    void* p = nullptr;
    // the request record, the dispatch record, then the slot: only requests up to vram_max
    // use it (longer ones go to the pinned host slot)
    const size_t bytes = kServerHeader + kServerHist + sv.vram_max;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) != hipSuccess || !p) return;
    bool mapped = false;
    int fds[2];
    if (pipe(fds) == 0) {
        mapped = write(fds[1], p, sizeof(ServerReq)) == (ssize_t)sizeof(ServerReq);
        close(fds[0]);
        close(fds[1]);
    }
    if (mapped) {
        ServerReq* r = static_cast<ServerReq*>(p);
        std::memset(r, 0, kServerHeader);  // ServerDispatch tag 0: no launch's epoch
        r->pad0[0] = 0x5CA17E57u;
        __builtin_ia32_sfence();
        ServerReq back{};
        mapped = hipMemcpyAsync(&back, p, sizeof back, hipMemcpyDeviceToHost, sv.stream) == hipSuccess &&
                 hipStreamSynchronize(sv.stream) == hipSuccess && back.pad0[0] == 0x5CA17E57u &&
                 back.req_seq == 0 && back.req_len == 0;
    }
    if (!mapped) {
        (void)hipFree(p);
        (void)hipGetLastError();
        return;
    }
    sv.vram = p;
    sv.req = sv.req_dev = static_cast<ServerReq*>(p);
    sv.disp_dev = reinterpret_cast<ServerDispatch*>(static_cast<uint8_t*>(p) + 128);
    sv.slot = sv.slot_dev = static_cast<uint8_t*>(p) + kServerHeader;
}

// scan() of host bytes [pos, pos + bl) through the scan server: their candidates are
// appended to the pending list.  *served = false (nothing changed) when the server is off
// or the bytes hold more than kServerCand candidates: the caller takes the batch path.
int server_scan(pbs_chunker* c, const uint8_t* hsrc, uint64_t pos, uint64_t bl, bool* served) {
    ScanServer& sv = c->srv;
    *served = false;
    if (!sv.enabled || sv.broken || bl == 0 || bl > kServerMaxBytes || !c->prm.hash_cuts) return PBS_OK;
    if (!sv.mb) {
        // the handle's device, whatever the calling thread's current one is: the stream,
        // the VRAM record and the kernel must sit with the handle's table
        DeviceGuard g(c->device);
        if (!g.ok) return fail(c, PBS_ERR_HIP);
        const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
        HIP_TRY(c, hipHostMalloc((void**)&sv.mb, sizeof(ServerMailbox), fl));
        std::memset(sv.mb, 0, sizeof(ServerMailbox));
        HIP_TRY(c, hipHostGetDevicePointer((void**)&sv.mb_dev, sv.mb, 0));
        HIP_TRY(c, hipStreamCreateWithFlags(&sv.stream, hipStreamNonBlocking));
        if (sv.dev_req) server_map_vram(c);
        HIP_TRY(c, hipHostMalloc((void**)&sv.hslot, kServerHist + kServerMaxBytes, fl));
        HIP_TRY(c, hipHostGetDevicePointer((void**)&sv.hslot_dev, sv.hslot, 0));
        if (!sv.vram) {
            sv.slot = sv.hslot;
            sv.slot_dev = sv.hslot_dev;
            sv.req = reinterpret_cast<ServerReq*>(sv.mb);
            sv.req_dev = reinterpret_cast<ServerReq*>(sv.mb_dev);
        }
    }
    // slot: the history right-aligned in its first kServerHist bytes, then the data; long
    // requests of a VRAM-mode server go to the pinned slot (kServerVramMax)
    const bool host_slot = sv.vram && bl > sv.vram_max;
    uint8_t* const slot = host_slot ? sv.hslot : sv.slot;
    std::memcpy(slot + kServerHist - c->carry_len, c->carry, c->carry_len);
    std::memcpy(slot + kServerHist, hsrc, bl);
    const uint32_t seq = (uint32_t)++sv.seq;
    sv.req->req_base = pos;
    sv.req->req_len = (uint32_t)bl | (host_slot ? kServerHostSlot : 0u);
    // write-combined BAR stores (slot, len, base) are not ordered by a release store: fence
    // them out before the seq, and the seq itself after
    __builtin_ia32_sfence();
    if (!sv.running) {
        int rc = server_launch(c, (uint32_t)(seq - 1));
        if (rc) return rc;
    }
    __atomic_store_n(&sv.req->req_seq, seq, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    const auto t0 = std::chrono::steady_clock::now();
    // the kernel's split of this request (scan_server.h: gu workgroups, each acknowledging
    // its own region of the candidates; 1: the leader alone, mb->ack_seq)
    const uint32_t npass = (uint32_t)((bl + 8191) / 8192);
    const uint32_t minp = (sv.flags >> kSrvMinPassShift) & 0xFFu;
    const uint32_t want = npass / (minp ? minp : kSrvMinPasses), nwg = sv.disp_dev ? sv.n_wg : 1u;
    const uint32_t gu = want < 1 ? 1u : std::min(want, nwg);
    uint64_t ack = 0;
    for (uint32_t spin = 0;; ++spin) {
        if (gu > 1) {
            uint32_t got = 0, cnt = 0;
            bool ovf = false;
            for (uint32_t g = 0; g < gu; ++g) {
                const uint64_t a = __atomic_load_n(&sv.mb->wg_ack[8 * g], __ATOMIC_ACQUIRE);
                if ((uint32_t)a != seq) break;
                ++got;
                cnt += (uint32_t)((a >> 32) & 0x7FFFFFFFull);
                ovf |= (a >> 63) != 0;
            }
            if (got == gu) {
                ack = (uint64_t)seq | (uint64_t)cnt << 32 | (ovf ? 1ull << 63 : 0ull);
                break;
            }
        } else {
            ack = __atomic_load_n(&sv.mb->ack_seq, __ATOMIC_ACQUIRE);
            if ((uint32_t)ack == seq) break;
        }
        const bool late = (spin & 1023) == 1023 &&
                          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kServerTimeoutS;
        if (!late && __atomic_load_n(&sv.mb->exited, __ATOMIC_ACQUIRE) == (uint32_t)(seq - 1)) {
            // it went idle just before this request: relaunch, the request is still there
            HIP_TRY(c, hipStreamSynchronize(sv.stream));
            int rc = server_launch(c, (uint32_t)(seq - 1));
            if (rc) return rc;
            continue;
        }
        if (late) {
            sv.broken = true;
            server_stop(c);
            return fail(c, PBS_ERR_HIP);
        }
        __builtin_ia32_pause();
    }
    if (sv.flags & kSrvProbe) {
        const volatile uint64_t* pr = sv.mb->probe;
        ++sv.probe_n;
        sv.probe_rtt_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        for (int i = 0; i < 3; ++i) sv.probe_ticks[i] += pr[i + 1] - pr[i];
    }
    if (ack >> 63) return PBS_OK;  // too many candidates: batch path
    const uint64_t k = (ack >> 32) & 0x7FFFFFFFull;
    const size_t old = c->pending.size();
    c->pending.resize(old + k);
    if (gu > 1) {  // the regions in workgroup order: stream order
        const uint32_t rcap = kServerCand / gu;
        uint64_t at = old;
        for (uint32_t g = 0; g < gu; ++g) {
            const uint64_t kg = (sv.mb->wg_ack[8 * g] >> 32) & 0x7FFFFFFFull;
            std::memcpy(c->pending.data() + at, sv.mb->cand + (uint64_t)g * rcap, kg * 8);
            at += kg;
        }
    } else {
        std::memcpy(c->pending.data() + old, sv.mb->cand, k * 8);
    }
    c->timing.bytes += bl;
    c->timing.candidates += k;
    update_carry(c, hsrc, bl);
    c->scanned_end = pos + bl;
    *served = true;
    return PBS_OK;
}

void reset_stream(pbs_chunker* c) {
    c->consumed = c->chunk_start = c->scanned_end = 0;
    c->carry_len = 0;
    c->pending.clear();
    c->pend_head = 0;
}

// pbs_chunker_scan path: scan new host bytes [pos, pos + bl) (uploaded to `dsrc`) and
// append their sorted candidates to the host pending list.
int scan_host_bytes(pbs_chunker* c, const uint8_t* dsrc, const uint8_t* hsrc, uint64_t pos,
                    uint64_t bl) {
    uint64_t ncand = 0;
    int rc = scan_candidates(c, dsrc, bl, pos, &ncand);
    if (rc) return rc;
    if (c->too_dense) return PBS_OK;  // nothing changed: the caller redoes a shorter batch
    if (ncand) {
        HIP_TRY(c, c->d_C.ensure(((size_t)ncand + 2) * 8));
        rc = sort_candidates(c, ncand, c->d_C.as<uint64_t>(), pos + bl);
        if (rc) return rc;
        const size_t old = c->pending.size();
        c->pending.resize(old + ncand);
        HIP_TRY(c, hipMemcpyAsync(c->pending.data() + old, c->d_C.p, (size_t)ncand * 8,
                                  hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    update_carry(c, hsrc, bl);
    c->scanned_end = pos + bl;
    return PBS_OK;
}

// One batch of the regular path with a single host sync (see find_cuts_impl).  *done:
// the batch is resolved and the state advanced.  Otherwise *have_cands tells whether
// c->d_cand holds the batch's *nnew candidates (too many for one workgroup: the caller
// sorts them and runs the multi-kernel resolve) or a list overflowed (rescan).
int spec_batch(pbs_chunker* c, const uint8_t* dsrc, const uint8_t* hsrc, uint64_t pos,
               uint64_t bl, size_t np, uint64_t rend, uint64_t* out, size_t cap, size_t* n,
               bool* done, bool* have_cands, uint64_t* nnew) {
    const Params& p = c->prm;
    *done = *have_cands = false;
    const ScanPlan sp = plan_scan(c, bl);
    const uint32_t m_max = kSmallResolveMax - 2;
    HIP_TRY(c, c->d_C.ensure((size_t)(m_max + 2) * 8));
    if (np)
        HIP_TRY(c, hipMemcpyAsync(c->d_C.p, c->pending.data() + c->pend_head, np * 8,
                                  hipMemcpyHostToDevice, c->stream));
    int rc = scan_launch(c, dsrc, bl, pos, sp, false);
    if (rc) return rc;
    const uint64_t tl = std::min<uint64_t>(bl, kWindow - 1);
    uint8_t* tail = reinterpret_cast<uint8_t*>(c->h_small + 24);  // written by resolve_small
    HIP_TRY(c, c->d_nxt.ensure(((size_t)m_max + 2) * 4));
    HIP_TRY(c, c->d_nf.ensure(((size_t)m_max + 2) * 8));
    HIP_TRY(c, c->d_res.ensure(32));
    const uint64_t out_cap = cut_bound(c, m_max, rend);
    HIP_TRY(c, c->d_cuts.ensure(out_cap * 8));
    if ((rc = ensure_small_host_bufs(c))) return rc;
    uint64_t *cuts_dev = nullptr, *keep_dev = nullptr, *small_dev = nullptr;
    if ((rc = mapped(c, c->h_cuts, &cuts_dev)) || (rc = mapped(c, c->h_keep, &keep_dev)) ||
        (rc = mapped(c, c->h_small, &small_dev)))
        return rc;
    HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    ResolveParams rp{p.min_eff, p.max_eff, rend, c->chunk_start};
    HIP_TRY(c, launch_resolve_small(c->d_cand.as<uint64_t>(), 0, c->d_C.as<uint64_t>(),
                                    (uint32_t)np, rp, c->d_nxt.as<uint32_t>(),
                                    c->d_nf.as<uint64_t>(), c->d_cuts.as<uint64_t>(), out_cap,
                                    cuts_dev, kHostCuts, keep_dev, kHostKeep,
                                    c->d_res.as<uint64_t>(), small_dev + 8, c->stream,
                                    c->d_counters.as<unsigned long long>(), c->susp_cap,
                                    c->cand_cap, small_dev,
                                    hsrc ? nullptr : dsrc + bl - tl,
                                    hsrc ? nullptr : reinterpret_cast<uint8_t*>(small_dev + 24),
                                    hsrc ? 0u : (uint32_t)tl));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    uint64_t nsusp = 0;
    bool ok = false;
    if ((rc = scan_collect(c, bl, sp, &nsusp, nnew, &ok))) return rc;
    if (!ok) return PBS_OK;  // a list overflowed (capacities grown) or too dense: rescan
    if (c->h_small[8 + 12] != 0) {  // resolve stood down: too many keys for one workgroup
        *have_cands = true;
        return PBS_OK;
    }
    rc = small_finish(c, (uint32_t)np + *nnew, out_cap, rend, out, cap, n);
    if (rc) return rc;
    update_carry(c, hsrc ? hsrc + bl - tl : tail, tl);
    c->scanned_end = pos + bl;
    *done = true;
    return PBS_OK;
}

// Static tile order of the fused pass over `nw` scanner waves: every wave gets the same
// work, and the tiles cover the batch up to less than one row of 64 blocks (8 KiB).  Tail
// items (the bytes past the tiles) are evaluated block by block, which costs far more per
// byte than the scan: with scan_main's power-of-two segments 8 GiB left 12 MiB of them
// (+0.1 ms).  Rounds of tiles of q blocks (<= kFusedStaticSeg - 128 bytes), then one short
// round (~q/8): the tiles of a round all end together, and the resolver gets the last
// round's candidates only when the scan is over -- half of them at 2 rounds, a quarter-
// second backlog at 256 KiB averages on 8 GiB.  From 8 rounds on, the short round is half
// a round drawn from a counter as 8 x nw small tiles (the pool, below).  Small batches:
// fewer tiles than waves (>= 4 KiB segments), one group.
void fused_static_plan(uint64_t len, uint64_t nw, FusedPassArgs* a) {
    const uint64_t rows = len / (64 * kBlockBytes);
    uint64_t qmax = (uint64_t)kFusedStaticSeg / kBlockBytes - 1;
    const uint64_t qmin = 32, qsmin = 8;
    if (const char* e = std::getenv("PBS_STATIC_QMAX"))  // shorter segments, more rounds (sweeps)
        qmax = std::min<uint64_t>(qmax, std::max<uint64_t>(qmin, std::strtoull(e, nullptr, 0)));
    a->ntiles = a->t_long = a->t_small = a->t_small_long = 0;
    a->seg_q = a->seg_qs = 0;
    if (rows < qmin) return;  // all tail items
    if (rows < qmin * nw * 9 / 8) {
        const uint64_t nt = std::min(rows / qmin, nw);
        a->ntiles = a->t_small = nt;
        a->seg_q = (uint32_t)(rows / nt);
        a->t_long = rows - (uint64_t)a->seg_q * nt;
        return;
    }
    const uint64_t T = (rows + nw * qmax - 1) / (nw * qmax);  // rounds of full tiles
    // the short round, in eighths of a full round, and the pool: from 8 rounds on (64 GiB:
    // 13) a half round drawn as 8 x nw tiles -- 64 GiB VM image 10.46-10.55 -> 10.36-10.39 ms,
    // random 11.19-11.25 -> 11.10-11.15; with 2 rounds (8 GiB) the pool's short tiles cost
    // more than they balance (1.42 -> 1.45 ms), scripts/gpu_r02az.sh.  PBS_POOL_ROUND /
    // PBS_POOL_DIV override (sweeps)
    uint64_t k8 = T >= 8 ? 4 : 1, d = T >= 8 ? 8 : 0;
    if (const char* e = std::getenv("PBS_POOL_ROUND")) k8 = std::max<uint64_t>(1, std::strtoull(e, nullptr, 0));
    if (const char* e = std::getenv("PBS_POOL_DIV")) d = std::strtoull(e, nullptr, 0);
    uint64_t q = std::min<uint64_t>(8 * rows / (nw * (8 * T + k8)), qmax);
    uint64_t rem = rows - T * nw * q;
    if (rem / nw < qsmin || rem / nw + 1 > qmax) {  // no short round: T rounds, the remainder spread over them
        a->ntiles = a->t_small = T * nw;
        a->seg_q = (uint32_t)(rows / a->ntiles);
        a->t_long = rows - (uint64_t)a->seg_q * a->ntiles;
        return;
    }
    a->seg_q = (uint32_t)q;
    a->t_small = T * nw;
    a->seg_qs = (uint32_t)(rem / nw);
    a->t_small_long = rem - (uint64_t)a->seg_qs * nw;
    a->ntiles = (T + 1) * nw;
    // pool (d > 1): the short round's rows as nw * d tiles of seg_qs / d blocks that the
    // waves draw from the counter, so the waves that run ahead (faster CUs) take more
    if (d > 1 && rem / (nw * d) >= qsmin) {
        const uint64_t ns = nw * d;
        a->seg_qs = (uint32_t)(rem / ns);
        a->t_small_long = rem - (uint64_t)a->seg_qs * ns;
        a->ntiles = a->t_small + ns;
        a->pool = 1;
    }
}

// Averages served by the fused pass: from 512 KiB (round 4; 256 KiB before).  Below, the scan
// pass (fused_scan_pass) is faster.  At 256 KiB, same process, alternating handles
// (scripts/ab_handles.py, profiles/r04/): 64 GiB random 11.78 fused vs 11.57 ms scan pass, 64 GiB
// VM image 10.74 vs 10.68, 16 GiB VM image 2.85 vs 2.80, 8 GiB random 1.76 vs 1.58 -- the
// fused kernel itself runs 0.2-0.3 ms longer there (its resolver's waits); at 512 KiB random
// 11.25 vs 11.26 (equal), at 4 MiB random 11.32 vs 11.55 (the scan pass's gather + resolve after
// the kernel, ~0.23 ms, then costs more than the fused kernel saves).  Round 3:
// at 128 KiB the fused resolver's main wave, ~64 candidates per us, bounds the pass
// (same process, profiles/r03/scanpass128k/: 8 GiB VM image 1.79-1.80 ms fused vs 1.53-1.57
// scan pass, 8 GiB random 2.47-2.48 vs 1.60-1.64, 16 GiB VM image 3.16-3.17 vs 2.88-2.89,
// 64 GiB random 12.7-13.2 vs 11.8-12.3, 64 GiB VM image 11.26-11.49 vs 11.18-11.42); at
// 256 KiB (config 5) both are within noise of each other on the 64 GiB VM image.  With
// PBS_FUSED=1 (tests) the fused pass serves from 128 KiB: a tile (1-2 MiB) of random data
// then holds ~12-24 candidates, far below the 64 flagged blocks one tile's exact step takes.
constexpr uint64_t kFusedMinAvg = 512 * 1024;
constexpr uint64_t kFusedForceMinAvg = 128 * 1024;
constexpr uint64_t kFusedMinBytes = 0;

// Tile order of the fused pass: static with SIMD balancing (the wave behind its SIMD partner
// takes the issue priority, scan_fused.h) and, from 8 rounds on, the pool (fused_static_plan)
// for averages >= kStaticMinAvg -- 64 GiB at 4 MiB: 10.31-10.39 ms vs 10.64-10.94 dynamic;
// at 256 KiB (config 5) 10.62-10.70 vs 11.04-11.11; at 512 KiB 10.49-10.51 vs 10.89-10.95;
// 8 GiB random 1.41-1.45 vs 1.49-1.52 -- and the dynamic order of scan_main_plan below it
// (64 GiB at 128 KiB: 11.28 dynamic vs 11.69-11.71 static; scripts/gpu_r02ba.sh and the
// logs under profiles/r02/balance/).  PBS_SCAN_DYN=0/1 forces one (A/B).
constexpr uint64_t kStaticMinAvg = 256 << 10;
bool fused_dynamic(const pbs_chunker* c, uint64_t bl) {
    if (c->scan_dyn_env >= 0) return c->scan_dyn_env == 1;
    uint64_t nt = 0, tb = 0;
    bool dyn = false;
    (void)scan_main_plan(bl, c->cu, &nt, &dyn, &tb);
    return dyn && c->prm.avg < kStaticMinAvg;
}

// The fused pass serves every batch > 1 MiB at averages >= fused_min_avg (static order:
// faster than scan_main + resolve from 128 MiB to 64 GiB, equal at 2-4 GiB; 8 GiB at
// 256 KiB 1.52-1.55 vs 1.59-1.60 ms, scripts/gpu_r02ak.sh / r02at.sh).  PBS_FUSED=1 forces it
// for every batch it can serve (its parity tests run small inputs), PBS_FUSED=0 never,
// PBS_FUSED_MIN_BYTES raises the size threshold (A/B).
bool use_fused(const pbs_chunker* c, uint64_t bl) {
    const uint64_t min_avg = c->fused_force ? std::min(kFusedForceMinAvg, c->fused_min_avg) : c->fused_min_avg;
    if (!(c->fused && c->prm.hash_cuts && c->prm.avg >= min_avg && bl > kFusedMaxBytes && c->cu >= 2))
        return false;
    return c->fused_force || bl >= c->fused_min_bytes;
}

// One batch [pos, pos + bl) of device bytes `dsrc` (hsrc: the same bytes on the host, or
// null) in ONE launch: scan_fused_kernel scans, evaluates the flagged blocks exactly and
// resolves the cuts while it runs (scan_fused.h); one host sync.  *done = false (and
// nothing changed) when the kernel stood down on dense input: the caller takes the
// multi-launch path.
int fused_pass(pbs_chunker* c, const uint8_t* dsrc, const uint8_t* hsrc, uint64_t pos,
               uint64_t bl, size_t np, uint64_t rend, uint64_t* out, size_t cap, size_t* n,
               bool* done) {
    const Params& p = c->prm;
    *done = false;
    FusedPassArgs a{};
    uint64_t ntiles = 0, t_big = 0, covered = 0;
    bool dyn = false;
    // tile order: fused_dynamic (static with SIMD balancing at averages >= 1 MiB)
    int seg = scan_main_plan(bl, c->cu, &ntiles, &dyn, &t_big);
    dyn = dyn && fused_dynamic(c, bl);
    if (dyn) {
        covered = scan_main_covered(ntiles, t_big, seg);
    } else {
        fused_static_plan(bl, (uint64_t)c->cu * kFusedWavesPerWG - kFusedResolverWaves, &a);
        ntiles = t_big = a.ntiles;
        covered = ((a.t_small * a.seg_q + a.t_long) + (ntiles - a.t_small) * a.seg_qs + a.t_small_long) *
                  64 * kBlockBytes;
    }
    const uint64_t ntail = ((bl - covered + kBlockBytes - 1) / kBlockBytes + kTailBlocks - 1) / kTailBlocks;
    const uint64_t items = ntiles + ntail;
    if (items == 0) return PBS_OK;
    const uint64_t nsteps = (items + kResolveBatch - 1) / kResolveBatch;
    // tile + step records: a fresh allocation (or an epoch wrap) is zeroed; epochs never 0
    const void* old_rec = c->d_rec.p;
    const size_t old_cap = c->d_rec.cap;
    HIP_TRY(c, c->d_rec.ensure((items + nsteps) * 8));
    if (c->d_rec.p != old_rec || c->d_rec.cap != old_cap || ((c->rec_epoch + 1) & 0xFFFFu) == 0) {
        HIP_TRY(c, hipMemsetAsync(c->d_rec.p, 0, c->d_rec.cap, c->stream));
        c->rec_epoch = 0;
    }
    c->rec_epoch = (c->rec_epoch + 1) & 0xFFFFu;
    const uint64_t expected = bl / p.avg * 3 / 2 + 1;
    const uint64_t cand_cap = std::min<uint64_t>(std::min<uint64_t>(bl + 1, expected * 2 + 8192), kMaxBatchCand);
    HIP_TRY(c, c->d_cand.ensure(cand_cap * 8));
    HIP_TRY(c, c->d_scratch.ensure(cand_cap * 32));  // c, sk, pm, nf | xl << 32 (u64 each)
    // counters: [0] flagged blocks, [1] candidates, [2] tile counter (u32), [3] scratch
    HIP_TRY(c, c->d_counters.ensure(32));
    HIP_TRY(c, hipMemsetAsync(c->d_counters.p, 0, 32, c->stream));
    HIP_TRY(c, c->d_pre.ensure(64));
    if (c->carry_len)
        HIP_TRY(c, hipMemcpyAsync(c->d_pre.p, c->carry, c->carry_len, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, c->d_C.ensure(std::max<size_t>(np, 1) * 8));
    if (np)
        HIP_TRY(c, hipMemcpyAsync(c->d_C.p, c->pending.data() + c->pend_head, np * 8,
                                  hipMemcpyHostToDevice, c->stream));
    int rc = ensure_small_host_bufs(c);
    if (rc) return rc;
    uint64_t *cuts_dev = nullptr, *keep_dev = nullptr, *small_dev = nullptr;
    if ((rc = mapped(c, c->h_cuts, &cuts_dev)) || (rc = mapped(c, c->h_keep, &keep_dev)) ||
        (rc = mapped(c, c->h_small, &small_dev)))
        return rc;
    const uint64_t tl = std::min<uint64_t>(bl, kWindow - 1);
    unsigned long long* ctr = c->d_counters.as<unsigned long long>();
    a.data = dsrc;
    a.len = bl;
    a.ntiles = ntiles;
    a.t_big = t_big;
    a.balance = (uint32_t)c->balance;
    a.resolver = 1;
    a.groups = 1;
    a.table_rot = c->d_table.as<uint32_t>();
    a.thr = p.thr;
    a.tile_ctr = reinterpret_cast<uint32_t*>(ctr + 2);
    a.pre = c->d_pre.as<uint8_t>();
    a.pre_len = c->carry_len;
    a.covered = covered;
    a.ntail = ntail;
    a.base = pos;
    a.rec = c->d_rec.as<unsigned long long>();
    a.epoch = c->rec_epoch;
    a.cand = c->d_cand.as<uint64_t>();
    a.ncand = ctr + 1;
    a.cand_cap = cand_cap;
    a.nflag = ctr;
    a.min_eff = p.min_eff;
    a.max_eff = p.max_eff;
    a.max_shift = (uint32_t)__builtin_ctzll(p.max_eff);
    a.end = rend;
    a.s0 = c->chunk_start;
    a.pend = c->d_C.as<uint64_t>();
    a.npend = (uint32_t)np;
    a.cuts_host = cuts_dev;
    a.host_cap = kHostCuts;
    uint8_t* scr = c->d_scratch.as<uint8_t>();
    a.sc_c = reinterpret_cast<uint64_t*>(scr);
    a.sc_sk = reinterpret_cast<uint64_t*>(scr + cand_cap * 8);
    a.sc_pm = reinterpret_cast<uint64_t*>(scr + cand_cap * 16);
    a.sc_nx = reinterpret_cast<uint64_t*>(scr + cand_cap * 24);
    a.sc_ctr = ctr + 3;
    a.keep_host = keep_dev;
    a.keep_cap = (uint32_t)kHostKeep;
    a.res_host = small_dev + 8;
    a.tail_src = dsrc + bl - tl;
    a.tail_host = reinterpret_cast<uint8_t*>(small_dev + 24);
    a.tail_len = (uint32_t)tl;
    a.timeout_ticks = c->fused_timeout_ticks;  // 20 s of wall_clock64 (100 MHz) by default
    volatile uint64_t* status_word = c->h_small + 8 + 3;
    volatile uint64_t* progress = c->h_small + 8 + 9;  // cuts in h_cuts so far (every 8 steps)
    *status_word = ~0ull;
    *progress = 0;
    uint64_t copied = 0;  // the host copies them while it waits
    HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(c, launch_scan_fused(a, seg, dyn, c->cu, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
    // the resolver stores its status word last (system-scope release) once every tile is
    // resolved: spin on it rather than wait for the kernel to retire; the event tells when
    // the kernel ended without one (launch failure), the wall clock when neither comes
    const auto t_launch = std::chrono::steady_clock::now();
    const double wait_s = c->host_wait_s > 0 ? c->host_wait_s : (double)c->fused_timeout_ticks * 1e-8 + 10.0;
    for (uint32_t spin = 1;; ++spin) {
        if (__atomic_load_n(status_word, __ATOMIC_ACQUIRE) != ~0ull) break;
        const uint64_t pr = std::min<uint64_t>(__atomic_load_n(progress, __ATOMIC_ACQUIRE), cap - *n);
        if (pr > copied) {
            std::memcpy(out + *n + copied, c->h_cuts + copied, (pr - copied) * 8);
            copied = pr;
        }
        if ((spin & 255) == 0) {
            const hipError_t q = hipEventQuery(c->ev[1]);
            if (q == hipSuccess) {
                if (__atomic_load_n(status_word, __ATOMIC_ACQUIRE) != ~0ull) break;
                return fail(c, PBS_ERR_HIP);
            }
            if (q != hipErrorNotReady) return fail(c, PBS_ERR_HIP);
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t_launch).count() > wait_s) {
                c->lost = true;
                return fail(c, PBS_ERR_HIP);
            }
        }
        __builtin_ia32_pause();
    }
    const uint64_t status = *status_word;
    if (c->debug_phases)
        std::fprintf(stderr, "fused pass %llu B: status %llu, resolver last record ready %.1f us, "
                     "done %.1f us, waited %.1f us (after its start)\n",
                     (unsigned long long)bl, (unsigned long long)status, c->h_small[14] / 100.0,
                     c->h_small[15] / 100.0, c->h_small[16] / 100.0);
    if (status == 1) return PBS_OK;  // stood down: dense input
    if (status != 0) return fail(c, PBS_ERR_HIP);
    const uint64_t ncut = c->h_small[8], s_open = c->h_small[9], nkeep = c->h_small[10];
    if (*n + ncut > cap || ncut > kHostCuts || nkeep > kHostKeep) return fail(c, PBS_ERR_CAPACITY);
    if (ncut > copied) std::memcpy(out + *n + copied, c->h_cuts + copied, (ncut - copied) * 8);
    *n += ncut;
    std::vector<uint64_t> keep(c->h_keep, c->h_keep + nkeep);
    c->chunk_start = s_open;
    c->pending.swap(keep);
    c->pend_head = 0;
    c->timing_pending = true;  // scan_ms: last_timing reads ev[0] -> ev[1]
    c->timing.bytes += bl;
    c->timing.fused += bl;
    c->timing.suspects += c->h_small[13];
    c->timing.candidates += c->h_small[12];
    c->timing.cuts += ncut;
    update_carry(c, hsrc ? hsrc + bl - tl : reinterpret_cast<uint8_t*>(c->h_small + 24), tl);
    c->scanned_end = pos + bl;
    *done = true;
    return PBS_OK;
}

// Averages below the fused pass's (64 KiB: ~900 k candidates in 64 GiB, more than its resolver
// walks in time): scan_fused_kernel without resolver waves -- the static tile order with SIMD
// balancing, the flagged blocks evaluated at the tile ends (up to kFusedGroups records of 64
// blocks per tile) -- then the records' candidates gathered in stream order (no sort) and the
// multi-kernel resolve.  Replaces scan_main + scan_exact + radix sort.  *done = false (nothing
// changed) when a record overflowed: the caller takes the multi-launch path.
// (from 64 KiB: a 2.5 MiB tile of random bytes holds ~120 flagged blocks, far below the
// 256 its records take; at 32 KiB ~240, and a batch with one overflowing tile is scanned twice)
constexpr uint64_t kScanPassMinAvg = 64 * 1024;
bool use_scan_pass(const pbs_chunker* c, uint64_t bl) {
    return c->fused && c->scan_pass && c->prm.hash_cuts && c->prm.avg >= kScanPassMinAvg &&
           c->prm.avg < c->fused_min_avg && bl > kFusedMaxBytes && c->cu >= 2;
}

int fused_scan_pass(pbs_chunker* c, const uint8_t* dsrc, const uint8_t* hsrc, uint64_t pos, uint64_t bl,
                    size_t np, uint64_t rend, uint64_t* out, size_t cap, size_t* n, bool* done) {
    const Params& p = c->prm;
    *done = false;
    FusedPassArgs a{};
    uint64_t ntiles = 0, t_big = 0, covered = 0;
    bool dyn = false;
    int seg = scan_main_plan(bl, c->cu, &ntiles, &dyn, &t_big);
    dyn = dyn && c->scan_dyn_env == 1;  // static order unless PBS_SCAN_DYN=1
    if (dyn) {
        covered = scan_main_covered(ntiles, t_big, seg);
    } else {
        fused_static_plan(bl, (uint64_t)c->cu * kFusedWavesPerWG, &a);
        ntiles = t_big = a.ntiles;
        covered = ((a.t_small * a.seg_q + a.t_long) + (ntiles - a.t_small) * a.seg_qs + a.t_small_long) *
                  64 * kBlockBytes;
    }
    const uint64_t ntail = ((bl - covered + kBlockBytes - 1) / kBlockBytes + kTailBlocks - 1) / kTailBlocks;
    const uint64_t items = ntiles + ntail;
    if (items == 0) return PBS_OK;
    const uint64_t nrec = items * kFusedGroups;
    const void* old_rec = c->d_rec.p;
    const size_t old_cap = c->d_rec.cap;
    HIP_TRY(c, c->d_rec.ensure(nrec * 8));
    if (c->d_rec.p != old_rec || c->d_rec.cap != old_cap || ((c->rec_epoch + 1) & 0xFFFFu) == 0) {
        HIP_TRY(c, hipMemsetAsync(c->d_rec.p, 0, c->d_rec.cap, c->stream));
        c->rec_epoch = 0;
    }
    c->rec_epoch = (c->rec_epoch + 1) & 0xFFFFu;
    const uint64_t expected = bl / p.avg * 3 / 2 + 1;
    const uint64_t cand_cap = std::min<uint64_t>(std::min<uint64_t>(bl + 1, expected * 2 + 8192), kMaxBatchCand);
    HIP_TRY(c, c->d_cand.ensure(cand_cap * 8));
    HIP_TRY(c, c->d_counters.ensure(32));
    HIP_TRY(c, hipMemsetAsync(c->d_counters.p, 0, 32, c->stream));
    HIP_TRY(c, c->d_pre.ensure(64));
    if (c->carry_len)
        HIP_TRY(c, hipMemcpyAsync(c->d_pre.p, c->carry, c->carry_len, hipMemcpyHostToDevice, c->stream));
    // d_C = [pending (np) | the batch's candidates in stream order]
    HIP_TRY(c, c->d_C.ensure((np + cand_cap + 2) * 8));
    if (np)
        HIP_TRY(c, hipMemcpyAsync(c->d_C.p, c->pending.data() + c->pend_head, np * 8, hipMemcpyHostToDevice,
                                  c->stream));
    size_t tb = 0;
    HIP_TRY(c, exclusive_sum_u64(nullptr, &tb, nullptr, nullptr, (uint32_t)(nrec + 1), c->stream));
    HIP_TRY(c, c->d_scan_tmp.ensure(tb));
    HIP_TRY(c, c->d_cnt.ensure((nrec + 1) * 8));
    HIP_TRY(c, c->d_off.ensure((nrec + 1) * 8));
    unsigned long long* ctr = c->d_counters.as<unsigned long long>();
    a.data = dsrc;
    a.len = bl;
    a.ntiles = ntiles;
    a.t_big = t_big;
    a.balance = (uint32_t)c->balance;
    a.resolver = 0;
    a.groups = kFusedGroups;
    a.table_rot = c->d_table.as<uint32_t>();
    a.thr = p.thr;
    a.tile_ctr = reinterpret_cast<uint32_t*>(ctr + 2);
    a.pre = c->d_pre.as<uint8_t>();
    a.pre_len = c->carry_len;
    a.covered = covered;
    a.ntail = ntail;
    a.base = pos;
    a.rec = c->d_rec.as<unsigned long long>();
    a.epoch = c->rec_epoch;
    a.cand = c->d_cand.as<uint64_t>();
    a.ncand = ctr + 1;
    a.cand_cap = cand_cap;
    a.nflag = ctr;
    HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(c, launch_scan_fused(a, seg, dyn, c->cu, c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
    // the gather writes its count, the overflow flag, the kernel's counters and the batch's
    // last bytes straight to mapped host memory: one sync, no copies after it
    const uint64_t tl = std::min<uint64_t>(bl, kWindow - 1);
    uint8_t* tail = reinterpret_cast<uint8_t*>(c->h_small + 24);
    int rc0 = ensure_small_host_bufs(c);
    if (rc0) return rc0;
    uint64_t* small_dev = nullptr;
    if ((rc0 = mapped(c, c->h_small, &small_dev))) return rc0;
    c->h_small[0] = c->h_small[1] = 0;
    HIP_TRY(c, c->d_res.ensure(32));
    HIP_TRY(c, launch_fused_gather(a.rec, nrec, a.epoch, a.cand, c->d_C.as<uint64_t>() + np, c->d_cnt.as<uint64_t>(),
                                   c->d_off.as<uint64_t>(), c->d_scan_tmp.p, c->d_scan_tmp.cap, small_dev,
                                   c->d_counters.as<unsigned long long>(), dsrc + bl - tl, (uint32_t)tl,
                                   reinterpret_cast<uint8_t*>(small_dev + 24), c->d_res.as<uint64_t>(), c->stream));
    HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
    // into a pinned cut array: the resolve goes right behind the gather, the candidate count
    // read on the device, and the host syncs once for the whole pass
    uint64_t* const out_dev = c->direct_out ? out_device_view(out) : nullptr;
    if (out_dev && cap > *n && np + cand_cap + 2 <= 0xFFFFFFF0ull) {
        bool overflow = false;
        const int rc = resolve_direct(c, (uint32_t)(np + cand_cap), c->d_res.as<uint64_t>(), (uint32_t)np,
                                      c->h_small, rend, out_dev, cap, n, &overflow);
        if (rc || overflow) return rc;  // overflow: nothing changed, *done stays false
        const uint64_t nnew = c->h_small[0], nflag = c->h_small[2];
        float ms = 0;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        c->timing.scan_ms += ms;
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
        c->timing.exact_ms += ms;  // the gather
        c->timing.bytes += bl;
        c->timing.fused += bl;
        c->timing.scan_pass += bl;
        c->timing.suspects += nflag;
        c->timing.candidates += nnew;
        update_carry(c, hsrc ? hsrc + bl - tl : tail, tl);
        c->scanned_end = pos + bl;
        *done = true;
        return PBS_OK;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const uint64_t nnew = c->h_small[0], overflow = c->h_small[1], nflag = c->h_small[2];
    if (overflow || nnew > cand_cap) return PBS_OK;  // dense input: the multi-launch path
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    c->timing.scan_ms += ms;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[1], c->ev[2]));
    c->timing.exact_ms += ms;  // the gather
    c->timing.bytes += bl;
    c->timing.fused += bl;
    c->timing.scan_pass += bl;
    c->timing.suspects += nflag;
    c->timing.candidates += nnew;
    const uint64_t m = (uint64_t)np + nnew;
    if (m > 0xFFFFFFF0ull) return fail(c, PBS_ERR_NOMEM);
    int rc = run_resolve(c, (uint32_t)m, rend, out, cap, n);
    if (rc) return rc;
    update_carry(c, hsrc ? hsrc + bl - tl : tail, tl);
    c->scanned_end = pos + bl;
    *done = true;
    return PBS_OK;
}

int find_cuts_impl(pbs_chunker* c, const uint8_t* data, size_t len, int is_final, uint64_t* out,
                   size_t cap, size_t* n_out, bool device) {
    if (!c) return PBS_ERR_INVALID;
    if (c->lost) return fail(c, PBS_ERR_HIP);
    if (!n_out || (len && !data) || (!out && cap)) return fail(c, PBS_ERR_INVALID);
    *n_out = 0;
    if (cap < pbs_chunker_cuts_bound(c, len)) return fail(c, PBS_ERR_CAPACITY);
    HIP_TRY(c, hipSetDevice(c->device));
    server_stop(c);
    c->timing = pbs_timing{};
    c->timing_pending = false;
    c->batch_limit = 0;  // a dense batch shortens batches for this call only
    HIP_TRY(c, hipEventRecord(c->ev[5], c->stream));
    const uint64_t end = c->consumed + len;
    uint64_t pos = std::max(c->consumed, c->scanned_end);
    size_t n = 0;
    bool first = true;
    while (pos < end || first) {
        first = false;
        const uint64_t bl = std::min<uint64_t>(end > pos ? end - pos : 0, batch_max(c));
        const uint64_t rend = bl ? pos + bl : end;  // resolve horizon of this batch
        size_t np = 0;
        while (c->pend_head + np < c->pending.size() && c->pending[c->pend_head + np] < rend) ++np;
        uint64_t nnew = 0;
        c->too_dense = false;
        const uint8_t* dsrc = nullptr;
        const uint8_t* hsrc = nullptr;
        if (bl && bl <= kFusedMaxBytes && np + 2 <= kSmallResolveMax) {
            bool overflow = false;
            int rc = fused_batch(c, device ? data + (pos - c->consumed) : nullptr,
                                 device ? nullptr : data + (pos - c->consumed), pos, bl, np, rend,
                                 true, out, cap, &n, &overflow);
            if (rc) return rc;
            if (!overflow) {
                pos += bl;
                continue;
            }
        }
        if (bl) {
            if (device) {
                dsrc = data + (pos - c->consumed);
            } else {
                hsrc = data + (pos - c->consumed);
                HIP_TRY(c, c->d_in.ensure(bl));
                HIP_TRY(c, hipMemcpyAsync(c->d_in.p, hsrc, bl, hipMemcpyHostToDevice, c->stream));
                dsrc = c->d_in.as<uint8_t>();
            }
        }
        if (bl && use_fused(c, bl)) {
            bool done = false;
            int rc = fused_pass(c, dsrc, hsrc, pos, bl, np, rend, out, cap, &n, &done);
            if (rc) return rc;
            if (done) {
                pos += bl;
                continue;
            }
        }
        if (bl && use_scan_pass(c, bl)) {
            bool done = false;
            int rc = fused_scan_pass(c, dsrc, hsrc, pos, bl, np, rend, out, cap, &n, &done);
            if (rc) return rc;
            if (done) {
                pos += bl;
                continue;
            }
        }
        bool have_cands = false;
        if (bl && c->prm.hash_cuts && np + 2 <= kSmallResolveMax) {
            // Speculative single-sync batch: scan, exact and the one-workgroup resolve are
            // enqueued back to back; the resolve reads the candidate count on the device
            // and stands down (res flag) when the lists overflowed or hold too many keys.
            bool done = false;
            int rc = spec_batch(c, dsrc, hsrc, pos, bl, np, rend, out, cap, &n, &done, &have_cands,
                                &nnew);
            if (rc) return rc;
            if (done) {
                pos += bl;
                continue;
            }
        }
        if (bl && !have_cands && !c->too_dense) {
            int rc = scan_candidates(c, dsrc, bl, pos, &nnew);  // host sync: counts
            if (rc) return rc;
        }
        if (c->too_dense) {  // more than kMaxBatchCand candidates: redo a quarter as long
            if (bl <= (1ull << 20)) return fail(c, PBS_ERR_NOMEM);
            c->batch_limit = std::max<uint64_t>(1ull << 20, bl / 4);
            continue;
        }
        const uint64_t m = (uint64_t)np + nnew;
        if (m > 0xFFFFFFF0ull) return fail(c, PBS_ERR_NOMEM);
        const bool small = m + 2 <= kSmallResolveMax;
        // d_C = [pending (np) | new (nnew)]; the small resolve sorts the new ones itself
        HIP_TRY(c, c->d_C.ensure((size_t)(m + 2) * 8));
        if (!small && nnew) {
            int rc = sort_candidates(c, nnew, c->d_C.as<uint64_t>() + np, pos + bl);
            if (rc) return rc;
        }
        if (np)
            HIP_TRY(c, hipMemcpyAsync(c->d_C.p, c->pending.data() + c->pend_head, np * 8,
                                      hipMemcpyHostToDevice, c->stream));
        // warm-up tail of this batch for the next one (lands with the resolve's sync)
        const uint64_t tl = std::min<uint64_t>(bl, kWindow - 1);
        uint8_t* tail = reinterpret_cast<uint8_t*>(c->h_small + 24);
        if (tl && device)
            HIP_TRY(c, hipMemcpyAsync(tail, dsrc + bl - tl, tl, hipMemcpyDeviceToHost, c->stream));
        int rc = small ? run_resolve_small(c, c->d_cand.as<uint64_t>(), (uint32_t)np,
                                           (uint32_t)nnew, rend, out, cap, &n)
                       : run_resolve(c, (uint32_t)m, rend, out, cap, &n);
        if (rc) return rc;
        if (bl) {
            update_carry(c, device ? tail : hsrc + bl - tl, tl);
            c->scanned_end = pos + bl;
        }
        pos += bl;
    }
    c->consumed = end;
    if (is_final) {
        if (c->chunk_start < end) {
            if (n >= cap) return fail(c, PBS_ERR_CAPACITY);
            out[n++] = end;
        }
        reset_stream(c);
    }
    if (!c->timing_pending) {
        float ms = 0;  // ev[4] = end of the last resolve (every path records it), synchronized
        HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[5], c->ev[4]));
        c->timing.total_ms = ms;
    }
    *n_out = n;
    return PBS_OK;
}

// A lost handle's stream, drained within `seconds`? (hipStreamQuery only: no call that
// could wait for a kernel that never retires)
bool drained(pbs_chunker* c, double seconds) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) return true;
        if (q != hipErrorNotReady) return false;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds) return false;
        usleep(1000);
    }
}

void destroy(pbs_chunker* c) {
    if (c->lost && !drained(c, 2.0)) {
        // a kernel of this handle still runs and may write its buffers: they are leaked
        // (freeing them would wait for it, possibly forever)
        std::fprintf(stderr, "pbs_chunker_free: a kernel of this handle did not finish; its device "
                             "buffers are not freed\n");
        delete c;
        return;
    }
    server_stop(c);
    if (c->srv.probe_n) {
        const ScanServer& sv = c->srv;
        const double n = (double)sv.probe_n;
        std::fprintf(stderr,
                     "scan server probe (request + slot in %s): %llu requests, host round trip %.2f us; kernel: "
                     "loads + chains %.2f us, hash %.2f us, compaction + ack %.2f us (request seen -> acknowledged "
                     "%.2f us)\n",
                     sv.vram ? "VRAM" : "pinned host memory", (unsigned long long)sv.probe_n,
                     sv.probe_rtt_us / n, sv.probe_ticks[0] / n / 100.0,
                     sv.probe_ticks[1] / n / 100.0, sv.probe_ticks[2] / n / 100.0,
                     (sv.probe_ticks[0] + sv.probe_ticks[1] + sv.probe_ticks[2]) / n / 100.0);
    }
    if (c->srv.stream) (void)hipStreamDestroy(c->srv.stream);
    if (c->srv.mb) (void)hipHostFree(c->srv.mb);
    if (c->srv.vram) (void)hipFree(c->srv.vram);
    if (c->srv.hslot) (void)hipHostFree(c->srv.hslot);
    DevBuf* bufs[] = {&c->d_table, &c->d_pre, &c->d_counters, &c->d_susp, &c->d_cand, &c->d_C,
                      &c->d_sort_tmp, &c->d_nxt, &c->d_jtmp, &c->d_nf, &c->d_on, &c->d_cnt,
                      &c->d_off, &c->d_scan_tmp, &c->d_cuts, &c->d_res, &c->d_in, &c->d_rec,
                      &c->d_scratch};
    for (DevBuf* b : bufs) b->release();
    c->d_stage.release();
    c->d_hits.release();
    if (c->h_cand) (void)hipHostFree(c->h_cand);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_cuts) (void)hipHostFree(c->h_cuts);
    if (c->h_keep) (void)hipHostFree(c->h_keep);
    delete c;
}

}  // namespace

// ------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------
extern "C" {

const char* pbs_strerror(int code) {
    switch (code) {
        case PBS_OK: return "ok";
        case PBS_ERR_NOT_POW2: return "got unexpected chunk size - not a power of two.";
        case PBS_ERR_NO_DEVICE: return "no HIP device available (the chunker has no CPU path)";
        case PBS_ERR_HIP: return "HIP runtime error";
        case PBS_ERR_NOMEM: return "out of memory";
        case PBS_ERR_CAPACITY: return "output array too small";
        case PBS_ERR_INVALID: return "invalid argument";
        default: return "unknown error";
    }
}

int pbs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

size_t pbs_chunker_max_cuts(size_t len) { return len / 65 + 3; }

size_t pbs_chunker_cuts_bound(const pbs_chunker* c, size_t len) {
    if (!c) return pbs_chunker_max_cuts(len);
    return len / c->prm.min_eff + 3;
}

pbs_chunker* pbs_chunker_new(size_t chunk_size_avg, int* err) {
    int dummy;
    if (!err) err = &dummy;
    Params prm;
    if (make_params(chunk_size_avg, &prm) != PBS_OK) {
        *err = PBS_ERR_NOT_POW2;
        return nullptr;
    }
    if (pbs_device_count() <= 0) {
        *err = PBS_ERR_NO_DEVICE;
        return nullptr;
    }
    pbs_chunker* c = new (std::nothrow) pbs_chunker();
    if (!c) {
        *err = PBS_ERR_NOMEM;
        return nullptr;
    }
    c->prm = prm;
    if (const char* e = std::getenv("PBS_DEBUG_PHASES")) c->debug_phases = e[0] == '1';
    if (const char* e = std::getenv("PBS_FUSED")) {
        c->fused = e[0] != '0';
        c->fused_force = e[0] == '1';
    }
    if (const char* e = std::getenv("PBS_SCAN_SERVER")) c->srv.enabled = e[0] != '0';
    if (const char* e = std::getenv("PBS_SERVER_VRAM")) c->srv.dev_req = e[0] != '0';
    if (const char* e = std::getenv("PBS_SERVER_WGS")) {
        const long v = std::atol(e);
        c->srv.n_wg = v < 1 ? 1u : (v > (long)kSrvMaxWgs ? kSrvMaxWgs : (uint32_t)v);
    }
    if (const char* e = std::getenv("PBS_SERVER_VRAM_MAX")) {
        const long long v = std::atoll(e);
        c->srv.vram_max = v < 0 ? 0 : std::min<uint64_t>((uint64_t)v, kServerMaxBytes);
    }
    if (const char* e = std::getenv("PBS_SCAN_PASS")) c->scan_pass = e[0] != '0';
    if (const char* e = std::getenv("PBS_SERVER_POLL")) c->srv.flags = e[0] == '4' ? kSrvPollAll : 0u;
    if (const char* e = std::getenv("PBS_SERVER_PROBE"))
        if (e[0] == '1') c->srv.flags |= kSrvProbe;
    if (const char* e = std::getenv("PBS_SERVER_MINPASS"))  // passes per workgroup of a split request (A/B)
        c->srv.flags |= (uint32_t)(std::min(255L, std::max(1L, std::atol(e)))) << kSrvMinPassShift;
    c->fused_min_avg = kFusedMinAvg;
    if (const char* e = std::getenv("PBS_BALANCE")) c->balance = std::atoi(e);
    if (const char* e = std::getenv("PBS_DIRECT_OUT")) c->direct_out = e[0] != '0';
    if (const char* e = std::getenv("PBS_SYNC_MODE")) c->sync_mode = std::atoi(e);
    if (const char* e = std::getenv("PBS_SCAN_DYN")) c->scan_dyn_env = e[0] == '1' ? 1 : 0;
    c->fused_min_bytes = kFusedMinBytes;
    if (const char* e = std::getenv("PBS_FUSED_MIN_BYTES")) c->fused_min_bytes = std::strtoull(e, nullptr, 0);
    if (const char* e = std::getenv("PBS_FUSED_MIN_AVG")) c->fused_min_avg = std::strtoull(e, nullptr, 0);
    if (const char* e = std::getenv("PBS_FUSED_TIMEOUT_TICKS")) c->fused_timeout_ticks = std::strtoull(e, nullptr, 0);
    if (const char* e = std::getenv("PBS_HOST_WAIT_MS")) c->host_wait_s = std::strtod(e, nullptr) * 1e-3;
    bool ok = hipGetDevice(&c->device) == hipSuccess;
    hipDeviceProp_t prop;
    if (ok && hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu = prop.multiProcessorCount;
    ok = ok && hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) == hipSuccess;
    c->stream = c->own_stream;
    for (auto& e : c->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&c->h_small, kSmallBytes, hipHostMallocMapped) == hipSuccess;
    ok = ok && c->d_table.ensure(512 * 4) == hipSuccess;
    if (ok) {
        // frame 1: T' = rotl(T, rot); frame 2: [T0 | T1], even bytes rot + 1, odd bytes rot
        uint32_t t[512];
        for (int i = 0; i < 256; ++i) {
            t[i] = rotl32(kBuzhashTable[i], kScanFrame == 1 ? prm.rot : prm.rot + 1);
            t[256 + i] = rotl32(kBuzhashTable[i], prm.rot);
        }
        // landed before any launch: copied on the handle's own non-blocking stream and waited
        // for there.  (Not the null stream: a null-stream copy waits for every blocking
        // stream's work, e.g. the pipeline's resident digest queue grid, whose drain can in
        // turn wait for this thread -- pbs_pipeline.cpp.)
        ok = hipMemcpyAsync(c->d_table.p, t, sizeof(t), hipMemcpyHostToDevice, c->own_stream) == hipSuccess &&
             hipStreamSynchronize(c->own_stream) == hipSuccess;
    }
    if (!ok) {
        destroy(c);
        *err = PBS_ERR_HIP;
        return nullptr;
    }
    *err = PBS_OK;
    return c;
}

void pbs_chunker_free(pbs_chunker* c) {
    if (c) destroy(c);
}

int pbs_chunker_reset(pbs_chunker* c) {
    if (!c) return PBS_ERR_INVALID;
    if (c->lost) {  // usable again once the kernel that outlived its bound has retired
        if (!drained(c, 0.0)) return fail(c, PBS_ERR_HIP);
        c->lost = false;
    }
    reset_stream(c);
    // the buffers this handle outgrew (DevBuf): freed now that it is idle -- its server
    // stopped, its stream drained -- so a handle whose batches grew does not keep ~2x its
    // peak scratch for its whole life (hipFree waits for the device: only when there are any)
    DevBuf* const bufs[] = {&c->d_table, &c->d_pre, &c->d_counters, &c->d_susp, &c->d_cand, &c->d_C,
                            &c->d_sort_tmp, &c->d_nxt, &c->d_jtmp, &c->d_nf, &c->d_on, &c->d_cnt, &c->d_off,
                            &c->d_scan_tmp, &c->d_cuts, &c->d_res, &c->d_in, &c->d_stage, &c->d_hits, &c->d_rec,
                            &c->d_scratch};
    bool any = false;
    for (DevBuf* b : bufs) any |= !b->retired.empty();
    if (any) {
        server_stop(c);
        if (hipStreamSynchronize(c->stream) != hipSuccess) return PBS_ERR_HIP;
        for (DevBuf* b : bufs) b->drop_retired();
    }
    return PBS_OK;
}

}  // extern "C"

int pbs::chunker_rewind(pbs_chunker* c) {
    if (!c) return PBS_ERR_INVALID;
    if (c->lost) {
        if (!drained(c, 0.0)) return fail(c, PBS_ERR_HIP);
        c->lost = false;
    }
    reset_stream(c);
    return PBS_OK;
}

extern "C" {

int pbs_chunker_set_cu_count(pbs_chunker* c, int cus) {
    if (!c || cus < 1) return PBS_ERR_INVALID;
    c->cu = cus;
    return PBS_OK;
}

int pbs_chunker_set_stream(pbs_chunker* c, void* hip_stream) {
    if (!c) return PBS_ERR_INVALID;
    c->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->own_stream;
    return PBS_OK;
}

int pbs_chunker_last_error(const pbs_chunker* c) { return c ? c->last_error : PBS_ERR_INVALID; }

uint64_t pbs_chunker_stream_offset(const pbs_chunker* c) { return c ? c->consumed : 0; }
uint64_t pbs_chunker_chunk_start(const pbs_chunker* c) { return c ? c->chunk_start : 0; }

int pbs_chunker_last_timing(const pbs_chunker* c, pbs_timing* t) {
    if (!c || !t) return PBS_ERR_INVALID;
    if (c->timing_pending) {  // a fused pass returned before its kernel retired
        pbs_chunker* m = const_cast<pbs_chunker*>(c);
        float scan = 0, total = 0;
        if (hipEventSynchronize(c->ev[4]) != hipSuccess ||
            hipEventElapsedTime(&scan, c->ev[0], c->ev[1]) != hipSuccess ||
            hipEventElapsedTime(&total, c->ev[5], c->ev[4]) != hipSuccess)
            return fail(m, PBS_ERR_HIP);
        m->timing.scan_ms += scan;
        m->timing.total_ms = total;
        m->timing_pending = false;
    }
    *t = c->timing;
    return PBS_OK;
}

size_t pbs_chunker_scan(pbs_chunker* c, const uint8_t* data, size_t len) {
    if (!c) return SIZE_MAX;
    if (c->lost) {
        fail(c, PBS_ERR_HIP);
        return SIZE_MAX;
    }
    if (len && !data) {
        fail(c, PBS_ERR_INVALID);
        return SIZE_MAX;
    }
    if (hipSetDevice(c->device) != hipSuccess) {
        fail(c, PBS_ERR_HIP);
        return SIZE_MAX;
    }
    const uint64_t end = c->consumed + len;
    if (end > c->scanned_end) {
        c->timing = pbs_timing{};
        c->batch_limit = 0;  // a dense batch shortens batches for this call only
        // No cut can fall before chunk_start + min_eff - 1, and no window of a later position
        // reaches back before that minus 63: those bytes only update the 63-byte history
        // (exact for every later chunk too, whose starts are later)
        const uint64_t lo = c->chunk_start + c->prm.min_eff - 1;
        const uint64_t skip_to = std::min<uint64_t>(end, lo >= kWindow - 1 ? lo - (kWindow - 1) : 0);
        if (c->prm.hash_cuts && skip_to > c->scanned_end) {
            update_carry(c, data + (c->scanned_end - c->consumed), skip_to - c->scanned_end);
            c->timing.bytes += skip_to - c->scanned_end;
            c->scanned_end = skip_to;
        }
        uint64_t pos = c->scanned_end;
        while (pos < end) {
            const uint64_t bl = std::min<uint64_t>(end - pos, batch_max(c));
            const uint8_t* hsrc = data + (pos - c->consumed);
            if (bl <= kServerMaxBytes) {
                bool served = false;
                if (server_scan(c, hsrc, pos, bl, &served) != PBS_OK) return SIZE_MAX;
                if (served) {
                    pos += bl;
                    continue;
                }
            }
            server_stop(c);  // the batch paths below do other device work on the handle
            if (bl <= kFusedMaxBytes) {
                bool overflow = false;
                size_t dummy = 0;
                if (fused_batch(c, nullptr, hsrc, pos, bl, 0, pos + bl, false, nullptr, 0, &dummy,
                                &overflow) != PBS_OK)
                    return SIZE_MAX;
                if (!overflow) {
                    pos += bl;
                    continue;
                }
            }
            if (c->d_in.ensure(bl) != hipSuccess ||
                hipMemcpyAsync(c->d_in.p, hsrc, bl, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
                fail(c, PBS_ERR_HIP);
                return SIZE_MAX;
            }
            c->too_dense = false;
            if (scan_host_bytes(c, c->d_in.as<uint8_t>(), hsrc, pos, bl) != PBS_OK)
                return SIZE_MAX;
            if (c->too_dense) {  // redo a quarter as long
                if (bl <= (1ull << 20)) {
                    fail(c, PBS_ERR_NOMEM);
                    return SIZE_MAX;
                }
                c->batch_limit = std::max<uint64_t>(1ull << 20, bl / 4);
                continue;
            }
            pos += bl;
        }
    }
    // shall_break (chunker.rs:172-186) over the cached candidates
    const Params& p = c->prm;
    const uint64_t lo = c->chunk_start + p.min_eff - 1;
    const uint64_t hi = c->chunk_start + p.max_eff - 1;
    while (c->pend_head < c->pending.size() && c->pending[c->pend_head] < lo) ++c->pend_head;
    if (c->pend_head > 4096) {
        c->pending.erase(c->pending.begin(), c->pending.begin() + (ptrdiff_t)c->pend_head);
        c->pend_head = 0;
    }
    uint64_t cut = UINT64_MAX;
    if (c->pend_head < c->pending.size() && c->pending[c->pend_head] <= hi &&
        c->pending[c->pend_head] < end)
        cut = c->pending[c->pend_head];
    else if (hi < end)
        cut = hi;
    if (cut == UINT64_MAX) {
        c->consumed = end;
        return 0;
    }
    const size_t ret = (size_t)(cut + 1 - c->consumed);
    c->consumed = c->chunk_start = cut + 1;
    return ret;
}

int pbs_chunker_find_cuts(pbs_chunker* c, const uint8_t* data, size_t len, int is_final,
                          uint64_t* out, size_t cap, size_t* n_out) {
    return find_cuts_impl(c, data, len, is_final, out, cap, n_out, false);
}

int pbs_chunker_find_cuts_device(pbs_chunker* c, const uint8_t* dev_data, size_t len,
                                 int is_final, uint64_t* out, size_t cap, size_t* n_out) {
    return find_cuts_impl(c, dev_data, len, is_final, out, cap, n_out, true);
}

int pbs_chunker_candidates_device(pbs_chunker* c, const uint8_t* dev, size_t len,
                                  const uint8_t* pre, size_t pre_len, uint64_t base,
                                  uint64_t* out_dev, size_t cap, size_t* n_out) {
    if (!c) return PBS_ERR_INVALID;
    if (c->lost) return fail(c, PBS_ERR_HIP);
    if (!n_out || (len && !dev) || (pre_len && !pre) || (cap && !out_dev) ||
        pre_len != std::min<uint64_t>(base, kWindow - 1))
        return fail(c, PBS_ERR_INVALID);
    *n_out = 0;
    HIP_TRY(c, hipSetDevice(c->device));
    server_stop(c);
    c->timing = pbs_timing{};
    // the handle's carry is the warm-up history of scan_candidates: swap the halo in
    uint8_t saved[64];
    const uint32_t saved_len = c->carry_len;
    std::memcpy(saved, c->carry, saved_len);
    std::memcpy(c->carry, pre, pre_len);
    c->carry_len = (uint32_t)pre_len;
    uint64_t n = 0;
    c->too_dense = false;
    int rc = scan_candidates(c, dev, len, base, &n);
    std::memcpy(c->carry, saved, saved_len);
    c->carry_len = saved_len;
    if (rc) return rc;
    if (c->too_dense) return fail(c, PBS_ERR_NOMEM);  // split the range further
    *n_out = n;
    if (n > cap) return fail(c, PBS_ERR_CAPACITY);
    rc = sort_candidates(c, n, out_dev, base + len);
    if (rc) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return PBS_OK;
}

int pbs_chunker_resolve_device(pbs_chunker* c, const uint64_t* cand_dev, size_t n, uint64_t end,
                               int is_final, uint64_t* out, size_t cap, size_t* n_out) {
    if (!c) return PBS_ERR_INVALID;
    if (c->lost) return fail(c, PBS_ERR_HIP);
    if (!n_out || (n && !cand_dev) || (!out && cap)) return fail(c, PBS_ERR_INVALID);
    *n_out = 0;
    if (n > 0xFFFFFFF0ull) return fail(c, PBS_ERR_NOMEM);
    if (cap < pbs_chunker_cuts_bound(c, end)) return fail(c, PBS_ERR_CAPACITY);
    HIP_TRY(c, hipSetDevice(c->device));
    server_stop(c);
    reset_stream(c);
    // keep the phase-A fields of a preceding candidates_device call
    c->timing.resolve_ms = c->timing.total_ms = 0;
    c->timing.cuts = 0;
    HIP_TRY(c, hipEventRecord(c->ev[5], c->stream));
    HIP_TRY(c, c->d_C.ensure((n + 2) * 8));
    size_t k = 0;
    int rc;
    if (n + 2 <= kSmallResolveMax) {
        rc = run_resolve_small(c, cand_dev, 0, (uint32_t)n, end, out, cap, &k);
    } else {
        if (n)
            HIP_TRY(c, hipMemcpyAsync(c->d_C.p, cand_dev, n * 8, hipMemcpyDeviceToDevice, c->stream));
        rc = run_resolve(c, (uint32_t)n, end, out, cap, &k);
    }
    if (rc) {
        reset_stream(c);
        return rc;
    }
    if (is_final && c->chunk_start < end) out[k++] = end;
    reset_stream(c);
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev[5], c->ev[4]));
    c->timing.total_ms = ms;
    *n_out = k;
    return PBS_OK;
}

int pbs_candidates_host(const uint8_t* data, size_t len, size_t avg, uint64_t* out, size_t cap,
                        size_t* n_out) {
    if (!n_out || (len && !data)) return PBS_ERR_INVALID;
    int err = 0;
    pbs_chunker* c = pbs_chunker_new(avg, &err);
    if (!c) return err;
    int rc = PBS_OK;
    uint64_t n = 0;
    if (len) {
        if (c->d_in.ensure(len) != hipSuccess ||
            hipMemcpyAsync(c->d_in.p, data, len, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            rc = PBS_ERR_HIP;
        if (!rc) rc = scan_candidates(c, c->d_in.as<uint8_t>(), len, 0, &n);
        if (!rc && c->too_dense) rc = PBS_ERR_NOMEM;
        if (!rc && n > cap) rc = PBS_ERR_CAPACITY;
        if (!rc && n) {
            if (c->d_C.ensure((size_t)n * 8) != hipSuccess) rc = PBS_ERR_HIP;
            if (!rc) rc = sort_candidates(c, n, c->d_C.as<uint64_t>(), len);
            if (!rc && (hipMemcpyAsync(out, c->d_C.p, (size_t)n * 8, hipMemcpyDeviceToHost,
                                       c->stream) != hipSuccess ||
                        hipStreamSynchronize(c->stream) != hipSuccess))
                rc = PBS_ERR_HIP;
        }
    }
    *n_out = n;
    pbs_chunker_free(c);
    return rc;
}

int pbs_generate_device(uint8_t* dev, size_t len, int kind, uint64_t seed, uint64_t offset,
                        void* hip_stream) {
    if ((len & 7) || (offset & 7) || (len && !dev)) return PBS_ERR_INVALID;
    if (kind < kGenCounter || kind > kGenVmImage) return PBS_ERR_INVALID;
    hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (launch_gen(reinterpret_cast<uint64_t*>(dev), len / 8, seed, offset / 8, kind, s) !=
        hipSuccess)
        return PBS_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return PBS_ERR_HIP;
    return PBS_OK;
}

#ifndef PBS_BUILD_ID
#define PBS_BUILD_ID "unknown"
#endif
const char* pbs_build_id(void) { return PBS_BUILD_ID; }

// Test hook (not part of the drop-in API, so not in include/): the static tile plan of the
// fused pass for a batch of `len` bytes over `nw` scanner waves -- out = {ntiles, seg_q,
// t_long, t_small, seg_qs, t_small_long, covered bytes, pool}.  tests/test_capi_cpu.py checks
// its invariants on the CPU.
int pbs_test_fused_static_plan(uint64_t len, uint64_t nw, uint64_t* out) {
    if (!out || nw == 0) return PBS_ERR_INVALID;
    FusedPassArgs a{};
    fused_static_plan(len, nw, &a);
    out[0] = a.ntiles;
    out[1] = a.seg_q;
    out[2] = a.t_long;
    out[3] = a.t_small;
    out[4] = a.seg_qs;
    out[5] = a.t_small_long;
    out[6] = ((a.t_small * a.seg_q + a.t_long) + (a.ntiles - a.t_small) * a.seg_qs + a.t_small_long) *
             64 * kBlockBytes;
    out[7] = a.pool;
    return PBS_OK;
}

int pbs_table_copy(uint32_t* out256) {
    if (!out256) return PBS_ERR_INVALID;
    std::memcpy(out256, kBuzhashTable, sizeof(kBuzhashTable));
    return PBS_OK;
}

}  // extern "C"
