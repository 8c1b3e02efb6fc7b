// Internal declarations shared by the kernels TU and the C-ABI/host pipeline TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef struct pbs_chunker pbs_chunker;  // include/pbs_chunker.h

namespace pbs {

// Hash frame of the product scan_main_kernel (scan_main.h): 1 =
// one rotate per byte, exact block test (measured 2-4 % faster in the full,
// power-limited kernel than the parity frame 2, and half the suspect blocks).
constexpr int kScanFrame = 1;
constexpr uint64_t kBlockBytes = 128;  // exact-evaluation granule (one lane iteration)

// generator kinds (see oracle/chunker_oracle.c; bytes must match)
constexpr int kGenCounter = 0;
constexpr int kGenRandom = 1;
constexpr int kGenVmImage = 2;
constexpr uint64_t kVmSeedPage = 0x7A65726F50414745ull;
constexpr uint64_t kVmSeedWord = 0x52414E44574F5244ull;
constexpr uint64_t kVmSeedExt = 0x4558544E54000000ull;

struct ResolveParams {
    uint64_t min_eff;  // max(avg/4, 65): first length at which a hash cut may happen
    uint64_t max_eff;  // max(avg*4, 65): forced cut length
    uint64_t end;      // absolute end of the bytes known so far (exclusive)
    uint64_t s0;       // absolute start of the open chunk
};

// Segment bytes per lane for a scan of `len` bytes (a wave tile = 64 segments) and
// the number of full wave tiles; bytes past ntiles*64*seg are the tail.
int scan_main_plan(uint64_t len, int cu, uint64_t* ntiles, bool* dyn, uint64_t* t_big);
// bytes covered by the plan's tiles (tiles >= t_big are small: 64 * seg / 4 bytes)
uint64_t scan_main_covered(uint64_t ntiles, uint64_t t_big, int seg);
hipError_t launch_scan_main(const uint8_t* data, uint64_t ntiles, int seg,
                            const uint32_t* table_rot, uint32_t thr, uint64_t* susp,
                            unsigned long long* nsusp, uint64_t cap, int grid, hipStream_t stream,
                            uint32_t* tile_ctr = nullptr, bool dynamic = false,
                            uint64_t t_big = ~0ull, bool balance = false);
// One launch for a whole batch: scan + exact positions + resolve (scan_fused.h).  `seg`
// and `dyn` from scan_main_plan; grid = one workgroup per CU.
// scan_fused_kernel geometry (checked in scan_fused.h): 8 waves per workgroup, waves 0..2
// of workgroup 0 resolve, every other wave scans tiles.
constexpr int kFusedWavesPerWG = 8;
constexpr int kFusedResolverWaves = 5;

struct FusedPassArgs {
    // phase A
    const uint8_t* data;   // batch bytes [0, len) (device)
    uint64_t len;
    uint64_t ntiles, t_big;     // dynamic order: tiles, first small tile
    // static order (fused_static_plan): tiles [0, t_small) have segments of seg_q 128-byte
    // blocks, the first t_long of them one more; tiles [t_small, ntiles) -- the last, short
    // round -- seg_qs blocks, the first t_small_long of them one more
    uint32_t seg_q, seg_qs;
    uint64_t t_long, t_small, t_small_long;
    uint32_t balance;           // SIMD partners trade issue priority by progress (PBS_BALANCE)
    uint32_t resolver;          // 1: waves 0..4 of workgroup 0 resolve (records: `groups` == 1);
                                // 0: every wave scans, the host resolves the records (scan pass)
    uint32_t groups;            // records per tile: up to 64 flagged blocks each (1 or kFusedGroups)
    uint32_t pool;              // static order: tiles [t_small, ntiles) are drawn from tile_ctr
    const uint32_t* table_rot;  // T' (256 words)
    uint32_t thr;
    uint32_t* tile_ctr;         // zeroed device counter (dynamic tile order)
    const uint8_t* pre;         // the pre_len <= 63 stream bytes before data[0] (device, 64 B)
    uint32_t pre_len;
    uint64_t covered;           // bytes covered by the tiles
    uint64_t ntail;             // tail items (kTailBlocks blocks each) after the tiles
    uint64_t base;              // absolute stream offset of data[0]
    // tile records and candidates
    unsigned long long* rec;    // ntiles + ntail records {epoch:16 | count:16 | index:32},
                                // then one record per resolver step (kResolveBatch tiles)
    uint32_t epoch;             // != 0, differs from every record left by earlier launches
    uint64_t* cand;             // candidate list (absolute positions; per tile contiguous)
    unsigned long long* ncand;  // zeroed counter
    uint64_t cand_cap;          // <= 2^32
    unsigned long long* nflag;  // zeroed counter: flagged blocks (statistics)
    // phase B
    uint64_t min_eff, max_eff;  // max_eff a power of two
    uint32_t max_shift;         // log2(max_eff)
    uint64_t end;               // bytes known: base + len
    uint64_t s0;                // open chunk start
    const uint64_t* pend;       // pending candidates of the open chunk (sorted, device)
    uint32_t npend;
    uint64_t* cuts_host;        // mapped host memory: the cut list (host_cap entries)
    uint64_t host_cap;
    // resolver scratch (cand_cap entries each): a step's candidates in stream order with
    // their in-vector successor, forced cuts and exit state (scan_fused.h fused_helper)
    uint64_t* sc_c;
    uint64_t* sc_sk;
    uint64_t* sc_pm;
    uint64_t* sc_nx;  // nf | xl << 32
    unsigned long long* sc_ctr;  // zeroed counter (scratch entries handed out)
    uint64_t* keep_host;        // mapped: candidates of the open chunk
    uint32_t keep_cap;
    uint64_t* res_host;         // mapped: [0] cuts [1] open chunk start [2] kept [3] status
                                // [4] candidates [5] flagged blocks
    const uint8_t* tail_src;    // the batch's last tail_len <= 63 bytes (device) -> tail_host
    uint8_t* tail_host;
    uint32_t tail_len;
    uint64_t timeout_ticks;     // resolver wait limit (wall_clock64 ticks, 100 MHz)
};

constexpr int kTailBlocks = 64;     // blocks per tail item of the fused pass
constexpr int kFusedGroups = 4;     // scan pass (no resolver): records per tile, so a tile may
                                    // hold 4 x 64 flagged blocks (small averages)
constexpr int kFusedStaticSeg = 40960;  // static-order fused pass: longest segment (bitmap size)
constexpr int kResolveBatch = 256;  // tile records per resolver step (4 per lane)
hipError_t launch_scan_fused(const FusedPassArgs& a, int seg, bool dyn, int grid, hipStream_t stream);
// Scan pass (FusedPassArgs::resolver == 0): the records' candidates, in record order (= stream
// order), to out[0 ..); counts/offs: nrec + 1 u64 scratch each; res (mapped host memory,
// res[1] zeroed by the caller): [0] candidates, [1] = 1 when a record overflowed (the batch
// must take another path), [2] / [3] the counters (flagged blocks, candidates listed); the
// batch's last tl <= 256 bytes to tail_dst; the candidate count also to count_dev (device).
hipError_t launch_fused_gather(const unsigned long long* rec, uint64_t nrec, uint32_t epoch,
                               const uint64_t* cand, uint64_t* out, uint64_t* counts, uint64_t* offs,
                               void* scan_tmp, size_t scan_tmp_bytes, uint64_t* res,
                               const unsigned long long* counters, const uint8_t* tail_src, uint32_t tl,
                               uint8_t* tail_dst, uint64_t* count_dev, hipStream_t stream);
// The open chunk's candidates C[res[2], m) -> keep (mapped host memory, keep_cap entries);
// res[3] = 1 when they do not fit.
hipError_t launch_resolve_keep(const uint64_t* C, uint32_t m, uint64_t* res, uint64_t* keep, uint64_t keep_cap,
                               const uint64_t* m_dev, uint32_t m_base, hipStream_t stream);
hipError_t launch_scan_exact(const uint8_t* data, uint64_t len, const uint8_t* pre,
                             uint32_t pre_len, const uint64_t* susp,
                             const unsigned long long* nsusp, uint64_t susp_cap, uint64_t ext_first,
                             uint64_t ext_count, int head, uint32_t mask, uint32_t minimum,
                             uint64_t base, uint64_t* cand, unsigned long long* ncand,
                             uint64_t cand_cap, uint64_t max_items, hipStream_t stream);
// pbs_sort.hip (in-house; hipCUB-style two-call protocol: tmp == nullptr asks for the
// temporary bytes).  radix_sort: stable LSD sort of u64 keys over [begin_bit, end_bit),
// values (u32) carried when vin != nullptr.
hipError_t radix_sort(void* tmp, size_t* tmp_bytes, const uint64_t* kin, uint64_t* kout,
                      const uint32_t* vin, uint32_t* vout, uint64_t n, int begin_bit, int end_bit,
                      hipStream_t stream);
hipError_t sort_u64(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, uint32_t n,
                    int end_bit, hipStream_t stream);
hipError_t exclusive_sum_u64(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out,
                             uint32_t n, hipStream_t stream);
// pbs_blob.hip: CRC-32 of blob payloads [bounds[i] + skip, bounds[i+1]) of `data`
hipError_t launch_crc32_skip(const uint8_t* data, const uint64_t* bounds_dev, uint64_t n, uint64_t skip,
                             uint32_t* out, hipStream_t st);
hipError_t inclusive_max_u32(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint32_t* out,
                             uint64_t n, hipStream_t stream);
// m_dev != nullptr: the node count is m_base + *m_dev, on the device only; m is then its upper
// bound (grids, the scan); the host needs no sync between the producer of m and this.
hipError_t launch_resolve(const uint64_t* C, uint32_t m, const ResolveParams& p, uint32_t* nxt,
                          uint32_t* jtmp, uint64_t* nforced, uint32_t* on, uint64_t* cnt,
                          uint64_t* off, void* scan_tmp, size_t scan_tmp_bytes, uint64_t* out,
                          uint64_t out_cap, uint64_t* res, hipStream_t stream,
                          const uint64_t* m_dev = nullptr, uint32_t m_base = 0);
// Single-workgroup sort + resolve + emit for batches with np + nnew + 2 <= kSmallResolveMax
// candidates (keys sorted in LDS).  C[0..np) holds the pending (sorted) candidates on
// entry and C[0..m) all sorted candidates on exit.  Cuts go to out[] and, while they
// fit, to the mapped pinned out_host[]; res/res_host = {ncut, s_open, idx}; the open
// chunk's candidates C[idx..m) are copied to keep_host when m - idx <= keep_cap.
constexpr uint32_t kSmallResolveMax = 16384;
hipError_t launch_resolve_small(const uint64_t* newc, uint32_t nnew, uint64_t* C, uint32_t np,
                                const ResolveParams& p, uint32_t* nxt, uint64_t* nforced,
                                uint64_t* out, uint64_t out_cap, uint64_t* out_host,
                                uint64_t host_cap, uint64_t* keep_host, uint64_t keep_cap,
                                uint64_t* res, uint64_t* res_host, hipStream_t stream,
                                const unsigned long long* counts = nullptr, uint64_t susp_cap = 0,
                                uint64_t cand_cap = 0, uint64_t* counts_host = nullptr,
                                const uint8_t* tail_src = nullptr, uint8_t* tail_host = nullptr,
                                uint32_t tail_len = 0);
// Small-input path (scan_blocks_kernel + resolve_small_kernel<1|2>, two launches, no
// host sync between): the input bytes `data[0..len)` (stream offset `base`, device
// memory) with the pre_len <= 63 bytes before them in `pre` (device), the test
// (h & mask) >= minimum, `hits` = device scratch of nblk = ceil(len/128) uint4 masks,
// the pending candidates in `pend` (device or mapped), and for scan-only calls the
// output array for the new candidates (mapped).
struct FusedScanArgs {
    const uint8_t* data;
    uint64_t len;
    const uint8_t* pre;
    uint32_t pre_len;
    uint64_t base;
    uint32_t mask, minimum;
    const uint4* hits;
    uint64_t nblk;
    const uint64_t* pend;
    uint64_t* cand_out;
    uint64_t cand_cap;
    // FUSED = 0 with counts != nullptr (speculative single-sync path): nnew is read from
    // counts[1] (scan_exact's candidate counter); counts[0] > susp_cap, counts[1] >
    // cand_cap or too many keys -> res_host[12] = 1 and nothing else is written
    const unsigned long long* counts;  // [0] suspects, [1] candidates (64-bit counters)
    uint64_t susp_cap;
    // speculative path, written before the stand-down test (saves two D2H copies): the
    // two counters to counts_host, the tail_len <= 63 bytes at tail_src (the warm-up
    // history of the next call) to tail_host; both mapped host memory, may be null
    uint64_t* counts_host;
    const uint8_t* tail_src;
    uint8_t* tail_host;
    uint32_t tail_len;
};
constexpr uint64_t kFusedMaxBytes = 1ull << 20;  // inputs up to this size take the fused path
hipError_t launch_scan_resolve_small(const FusedScanArgs& fa, int resolve, uint64_t* C,
                                     uint32_t np, const ResolveParams& p, uint32_t* nxt,
                                     uint64_t* nforced, uint64_t* out, uint64_t out_cap,
                                     uint64_t* out_host, uint64_t host_cap, uint64_t* keep_host,
                                     uint64_t keep_cap, uint64_t* res, uint64_t* res_host,
                                     hipStream_t stream);
// ---- scan server (scan_server.h): the low-latency path of pbs_chunker_scan ----------
// A persistent one-workgroup kernel polls a mailbox in fine-grained (coherent) pinned host
// memory; the host writes a request (the new bytes go to a pinned slot) and spins on the
// acknowledgement, so one scan() call costs one PCIe round trip instead of a copy, two
// launches and a stream sync.
constexpr uint32_t kServerMaxBytes = 1u << 20;  // request slot (bigger calls: batch path)
constexpr uint32_t kServerCand = 16384;         // candidates one request may return
constexpr uint32_t kServerHist = 64;            // slot bytes before the data: the history
constexpr uint32_t kServerQuit = 1u << 31;      // req_len flag
constexpr uint32_t kServerHostSlot = 1u << 30;  // req_len flag: the data are in the pinned host slot
// requests up to this size go to the VRAM slot when there is one (PBS_SERVER_VRAM_MAX for
// A/B): the host's write-combined BAR stores (~47 GB/s) beat the kernel's PCIe reads of
// pinned memory (8 KiB 7.2 -> 4.9 us round trip, mb_bar.hip).  Until round 5 it was 128 KiB:
// one workgroup hashing ~6 GB/s made the copy's speed moot for longer requests
// (profiles/r03/vram); with several workgroups per request (kSrvMaxWgs) it is not.
constexpr uint32_t kServerVramMax = kServerMaxBytes;
// Requests of at least 2 kSrvMinPasses passes are split over up to `n_wg` workgroups of the
// server (PBS_SERVER_WGS, scan_server.h): each polls the host's request record and hashes a
// contiguous range of passes.  This record, in the same fine-grained VRAM allocation (+128
// bytes), carries only the leader's exit: tag = last seq | epoch << 32 | 1 << 63 (epoch:
// the launch number mod 2^30, so a record left by an earlier launch is never taken).
struct alignas(64) ServerDispatch {
    uint64_t tag;
};
constexpr uint32_t kSrvMaxWgs = 32;
constexpr uint32_t kSrvMinPasses = 1;  // split requests: passes per workgroup at least (PBS_SERVER_MINPASS; 2 until round 6)
constexpr uint32_t kSrvDefaultWgs = 16;
constexpr uint32_t kServerHeader = 256;  // VRAM allocation: record (0), dispatch (128), then the slot
static_assert(sizeof(ServerDispatch) <= kServerHeader - 128, "dispatch record past the header");
struct alignas(64) ServerMailbox {
    // host -> device: ONE 16-byte record the kernel polls with one load (the host stores
    // len and base before seq, all in one cache line, so a record with the new seq has them)
    uint32_t req_seq;   // request number, stored last (release)
    uint32_t req_len;   // data bytes in the slot (after its kServerHist history bytes);
                        // kServerQuit set: exit now
    uint64_t req_base;  // absolute stream offset of the data; history = the min(63, base)
                        // stream bytes before it, right-aligned in the slot's first 64 bytes
    uint32_t pad0[12];
    // device -> host
    alignas(64) uint64_t ack_seq;  // once served (release): req_seq | ncand << 32 | overflow << 63,
                                   // ncand = candidates in cand[] (ascending, absolute), overflow:
                                   // more than kServerCand (nothing usable)
    uint64_t exited;               // last served request when the kernel exited; ~0 while up
    uint64_t probe[4];             // kSrvProbe: wall_clock64 at request seen, chains done, hashed, acked
    // a split request (gu > 1 workgroups, scan_server.h): workgroup g stores its candidates in
    // cand[g * (kServerCand / gu) ..] and then acknowledges alone in wg_ack[8 g] (its own cache
    // line; the same word layout as ack_seq, the count of its region) -- no device atomics,
    // and the host reads the regions in order (ascending already)
    alignas(64) uint64_t wg_ack[8 * kSrvMaxWgs];
    uint64_t cand[kServerCand];
};
// The request record alone (the layout of ServerMailbox's first 64 bytes).  With the
// request in device memory (kSrvDevReq) the host writes it and the slot through the GPU's
// BAR mapping of a fine-grained VRAM allocation, so the kernel polls and reads its own HBM
// instead of pinned host memory across PCIe; otherwise it points at the mailbox.
struct alignas(64) ServerReq {
    uint32_t req_seq;
    uint32_t req_len;
    uint64_t req_base;
    uint32_t pad0[12];
};
static_assert(sizeof(ServerReq) == 64, "ServerReq is one cache line");
constexpr uint32_t kSrvPollAll = 1;  // launch flag: every wave polls (staggered), not one lane
constexpr uint32_t kSrvProbe = 2;    // launch flag: per-request phase stamps into probe[]
constexpr uint32_t kSrvDevReq = 4;   // launch flag: request + slot in fine-grained VRAM written by the host
constexpr uint32_t kSrvMinPassShift = 8;  // launch flags bits 8-15: passes per workgroup of a split request (0: default)
hipError_t launch_scan_server(ServerMailbox* mb_dev, const ServerReq* req_dev, ServerDispatch* disp_dev,
                              const uint8_t* slot_dev, const uint8_t* hslot_dev, const uint32_t* table_rot,
                              uint32_t thr, uint64_t last_seq, uint64_t idle_ticks,
                              uint32_t flags, uint32_t n_wg, uint32_t epoch, hipStream_t stream);

// Makes `dev` the calling thread's current device for a scope (allocations and stream /
// event creation land on the current device, not on the device of the stream a call was
// handed) and restores the previous one.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            prev = -1;
            return;
        }
        ok = prev == dev || hipSetDevice(dev) == hipSuccess;
        if (prev == dev) prev = -1;  // nothing to restore
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// pbs_blob.hip: free the blob-CRC chunk counter kept for `st` (call before destroying it)
void release_stream_counter(hipStream_t st);

// ---- digest queue (pbs_digest.hip sha256_queue_kernel; used by pbs_pipeline.cpp) -------
struct DigestJob {   // in pinned host memory, written by the host before the count
    uint64_t start;  // chunk start, bytes from the device buffer's start
    uint64_t len;
    uint64_t idx;    // output slot (the chunk's index): digests + 32 * idx
    uint64_t done;   // written 1 by the GPU once the digest is in memory (system-scope release
                     // before it): the upload path's encoder waits for it (the host zeroes it)
};
struct DigestQueueDev {  // device memory, zeroed before the launch
    unsigned long long next;       // jobs claimed
    unsigned long long mirror;     // last control word seen: count | final << 63
    unsigned long long last_poll;  // wall_clock64 of the last read of the host word
    unsigned long long polls;      // reads of the host word (statistics)
    unsigned long long last_h;     // the last value read
    unsigned long long nseen;      // debug: distinct values read, and when (wall_clock64)
    unsigned long long seen[16];
    unsigned long long seen_t[16];
};
constexpr uint64_t kDigestQueueFinal = 1ull << 63;
// Persistent grid of `grid` two-wave workgroups on `st` hashing the published jobs into
// digests (device, 32 bytes per slot) until the final bit is set and every job is taken,
// or idle_ticks (100 MHz) pass without a new job (launch it again for later jobs: the
// queue state in `q` carries over).  key: <= PBS_DIGEST_MAX_KEY bytes.
hipError_t launch_sha256_queue(const uint8_t* data, const uint8_t* key, size_t key_len, const DigestJob* jobs_dev,
                               const uint64_t* ctl_dev, DigestQueueDev* q, uint8_t* digests, int grid,
                               uint64_t idle_ticks, hipStream_t st);
// frees the calling thread's counters of the shared stream handles (pbs_blob.hip)
void release_thread_counters();
hipError_t launch_gen(uint64_t* out, uint64_t nwords, uint64_t seed, uint64_t word_offset,
                      int kind, hipStream_t stream);

// pbs_chunker_reset without freeing the buffers the handle outgrew (pbs_chunker_reset's
// hipFree waits for the whole device, e.g. for a digest queue grid another thread's
// pipeline keeps resident): the pipeline's reused handle starts each stream with this;
// its outgrown buffers go when the handle is freed.
int chunker_rewind(::pbs_chunker* c);

}  // namespace pbs
