// scan_fused_kernel: the whole chunking pass of a batch in ONE launch (DESIGN.md section 2,
// "Fused pass") -- phase A (the scan_main_kernel loop), the exact candidate positions of the
// flagged 128-byte blocks, and phase B, the min/max rule of chunker.rs:172-183, resolved
// while the scan runs.
//
//   scanner waves   every wave but workgroup 0.s three resolver waves runs scan_main.s tile
//                   loop (static order: a whole number of tiles each).  A flagged block is a
//                   bit in the wave's LDS bitmap (no global atomic).  At the end of a tile
//                   (ring registers dead, the next tile's first DMA in flight) the wave
//                   evaluates its flagged blocks exactly (exact_block.h, one block per wave
//                   step, windows re-read from HBM), appends the tile's candidates -- already
//                   in stream order: lanes own ascending segments, bits ascending blocks -- to
//                   the candidate list with ONE atomic, and publishes the tile record
//                   {epoch, count, list index} (write-through stores, drained, then the
//                   record: the hand-off of MI355X_MICROARCH.md "Inter-workgroup
//                   visibility").  After the tiles, the bytes past the last tile ("tail
//                   items", 64 blocks each) are evaluated the same way.
//   resolver waves  waves 0..4 of workgroup 0 take no tiles: four helpers turn the tile
//                   records, in stream order and 256 records per step, into per-candidate
//                   chain data (below); the main wave walks the cut chain over them, with
//                   the pending candidates of the open chunk first.  Cuts go to mapped host
//                   memory (the host copies them out while the pass runs); at the end the
//                   main wave writes the open chunk's start, its candidates and the batch's
//                   last 63 bytes to the host.  It finishes a few microseconds after the
//                   last tile, so the pass costs one launch and one host sync.
//
// Scan pass (FusedPassArgs::resolver == 0, small averages): no resolver waves -- every wave
// scans, and a tile publishes up to `groups` records of 64 flagged blocks each; the host
// gathers the records' candidates in record (= stream) order and resolves them
// (pbs_chunker_capi.cpp fused_scan_pass).
//
// Stand-down: a tile with more than 64 flagged blocks, a full candidate list or more than
// kFusedKeep open-chunk candidates (dense input) sets status 1 -- the host then runs the
// batch through the multi-launch path (scan_main + scan_exact + resolve), which has no
// such limits.  A resolver that waits longer than timeout_ticks sets status 2 (error).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_block.h"
#include "pbs_chunker_internal.h"  // FusedPassArgs
#include "scan_main.h"

namespace pbs {

constexpr int kFusedKeep = 512;     // open-chunk candidates the resolver keeps in LDS
constexpr int kCutBuf = kStagePerWave / 8 - kFusedKeep;  // cuts the main wave buffers in LDS
constexpr int kLaneProbes = 3;      // linear probes before the binary lane search
constexpr int kMainAhead = 8;       // resolver vectors the main wave has in flight
constexpr int kStageCand = 512;     // candidates of one resolver step staged in LDS
constexpr int kFusedHelpers = 4;    // resolver helper waves (workgroup 0, waves 1..4)
constexpr int kPubDepth = 16;       // exact windows in flight per wave (fused_publish)

constexpr uint32_t kRecOverflow = 0xFFFFu;
static_assert(kFusedWavesPerWG == kWavesPerWG && kFusedResolverWaves == 1 + kFusedHelpers,
              "pbs_chunker_internal.h describes this kernel's wave roles");

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

__device__ __forceinline__ uint64_t uni64(uint64_t v) {  // wave-uniform value into SGPRs
    // (readfirstlane returns int: through uint32_t, or the low word sign-extends)
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

__device__ __forceinline__ void store_wt(uint64_t* p, uint64_t v) {  // write-through (sc1)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Evaluate the blocks lane j names (B_j relative to data, j < nb <= 64) exactly, append
// their candidates to the list in lane order and publish record `item`.  `over`: more than
// 64 flagged blocks (the record says overflow).  Wave-uniform control flow.
__device__ __forceinline__ void fused_publish(const FusedPassArgs& a, const uint32_t* tab,
                                              uint64_t item, int64_t myB, int nb, bool over,
                                              int lane) {
    uint4 mh = make_uint4(0, 0, 0, 0);
    if (nb > 0 && !over) {
        // groups of kPubDepth blocks: the windows of group g+1 load while group g is hashed
        // (one block at a time waited a memory latency per block: a 64-block tail item,
        // never streamed before, cost ~64 HBM round trips -- 8 GiB static order: +0.1 ms)
        uint32_t cur[kPubDepth], nxt[kPubDepth];
        auto load_group = [&](int g, uint32_t (&w)[kPubDepth]) {
#pragma unroll
            for (int k = 0; k < kPubDepth; ++k)
                w[k] = g + k < nb ? exact_load(a.data, a.len, a.pre, a.pre_len,
                                               (int64_t)readlane64((uint64_t)myB, g + k), lane)
                                  : 0u;
        };
        load_group(0, cur);
        for (int g = 0; g < nb; g += kPubDepth) {
            if (g + kPubDepth < nb) load_group(g + kPubDepth, nxt);
#pragma unroll
            for (int k = 0; k < kPubDepth; ++k) {
                if (g + k < nb) {
                    const int64_t B = (int64_t)readlane64((uint64_t)myB, g + k);
                    const uint4 h = exact_hits<true>(cur[k], a.len, a.pre_len, B, tab, a.thr, 0u, lane);
                    if (lane == g + k) mh = h;
                }
            }
#pragma unroll
            for (int k = 0; k < kPubDepth; ++k) cur[k] = nxt[k];
        }
    }
    const uint32_t cnt = __builtin_popcount(mh.x) + __builtin_popcount(mh.y) +
                         __builtin_popcount(mh.z) + __builtin_popcount(mh.w);
    const uint32_t incl = wave_incl_sum(cnt);  // inclusive prefix over lanes
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    uint64_t idx = 0;
    bool ovf = over || total >= kRecOverflow;
    if (!ovf && total) {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(a.ncand, (unsigned long long)total);
        idx = readlane64(b, 0);
        if (idx + total > a.cand_cap) {
            ovf = true;
        } else {
            uint64_t o = idx + (incl - cnt);
            const uint64_t p0 = a.base + (uint64_t)myB;
            const uint32_t w4[4] = {mh.x, mh.y, mh.z, mh.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t m = w4[q];
                while (m) {
                    const int bit = __builtin_ctz(m);
                    m &= m - 1;
                    store_wt(a.cand + o, p0 + (uint64_t)(q * 32 + bit));
                    ++o;
                }
            }
            // the candidates are written through to memory before the record says so
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    if (lane == 0) {
        const uint64_t r = ((uint64_t)a.epoch << 48) |
                           ((uint64_t)(ovf ? kRecOverflow : total) << 32) | (idx & 0xFFFFFFFFull);
        __hip_atomic_store(a.rec + item, (unsigned long long)r, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {  // divergent source lane
    return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, src, 64) |
           ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64) << 32);
}

// first lane in [from, nv) whose candidate is >= x (nv if none); lanes [0, nv) hold
// ascending candidates.  The next few lanes are probed first (a chunk usually ends at one
// of the next candidates); the rest is a binary search that runs only as long as some lane needs it.
// All 64 lanes take part (the shuffles read every lane).
__device__ __forceinline__ int lanes_lower_bound(uint64_t c, int from, int nv, uint64_t x) {
    int lo = from < nv ? from : nv, hi = nv;
    // kLaneProbes linear probes first: with one, ~1 lane in 5 still needed the search at
    // 64 KiB averages (the next candidate within the minimum size), so nearly every
    // vector paid its 6 shuffle rounds
#pragma unroll
    for (int p = 0; p < kLaneProbes; ++p) {
        if (!__any(lo < hi)) break;
        const uint64_t v = shfl64(c, lo < 64 ? lo : 63);
        if (lo < hi) {
            if (v >= x)
                hi = lo;
            else
                ++lo;
        }
    }
    while (__any(lo < hi)) {
        const int mid = (lo + hi) >> 1;
        const uint64_t v = shfl64(c, mid < 64 ? mid : 63);
        const bool go_right = lo < hi && v < x;
        const bool go_left = lo < hi && !(v < x);
        lo = go_right ? mid + 1 : lo;
        hi = go_left ? mid : hi;
    }
    return lo;
}

// Phase B (chunker.rs:172-183) is split over five waves of workgroup 0 (four helpers: with
// two, the static tile order at 256 KiB averages waited for them -- 8 GiB 1.62 -> 1.50-1.53 ms):
//
//   helpers (4)  take the record steps (kResolveBatch records) round-robin: wait for the
//                step's tiles, gather its candidates in stream order and, for every 64-
//                candidate vector, compute per candidate lane-parallel (independent of
//                everything before the vector): the next cut inside the vector if a cut
//                were taken there (or "leaves the vector"), the forced cuts in between (nf)
//                and the state after them (sk); then by pointer doubling (6 rounds of
//                shuffles) the chain mask pm = the lanes cut on the chain from this lane
//                until it leaves the vector, and xl = the lane where it leaves.  The step's
//                {c, sk, pm, nf, xl} go to a scratch area, then the step record is
//                published (workgroup scope: helpers and main share the CU).
//   main (1)     takes the steps in order: per vector, the first cut from the incoming
//                state (one ballot; forced cuts in closed form), then the whole chain from
//                pm / xl of that lane in O(1) -- the cuts (and each cut's nf forced cuts)
//                written with vector stores, the candidates past the chain kept for the
//                open chunk.  Pending candidates of earlier calls come first (walked cut by
//                cut).
//
// One wave's serial walk cost ~35 instructions per cut at the ~4-cycle issue cadence of a
// wave; with the chain masks it is a few instructions per 64 candidates, so the main wave
// keeps up with 128 KiB averages and finishes a few microseconds after the last tile.
struct FusedStep {  // one resolver step, in scratch (stream order)
    uint64_t* c;   // candidate
    uint64_t* sk;  // state after a cut here and its forced cuts, if the chain leaves here
    uint64_t* pm;  // lanes on the chain from here to where it leaves the vector
    uint64_t* nx;  // forced cuts after a cut here | the lane where the chain from here
                   // leaves the vector << 32 (one load: both are read where the walk needs them)
};

__device__ void fused_helper(const FusedPassArgs& a, uint64_t* stc, int h, int nh, int lane) {
    const uint64_t total = a.ntiles + a.ntail;
    const uint64_t nsteps = (total + kResolveBatch - 1) / kResolveBatch;
    const uint64_t min1 = a.min_eff - 1, max_eff = a.max_eff, max1 = a.max_eff - 1;
    const uint32_t sh = a.max_shift, epoch = a.epoch;
    const unsigned long long* const rec = a.rec;
    const uint64_t* const cand = a.cand;
    unsigned long long* const sinfo = a.rec + total;  // step records after the tile records
    const FusedStep sc{a.sc_c, a.sc_sk, a.sc_pm, a.sc_nx};
    const uint64_t t_start = wall_clock64();
    for (uint64_t st = (uint64_t)h; st < nsteps; st += (uint64_t)nh) {
        const uint64_t t0 = st * kResolveBatch;
        uint64_t rv[4];
        bool done = true;
        for (;;) {
            done = true;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t t = t0 + 4 * (uint64_t)lane + q;
                rv[q] = t < total ? __hip_atomic_load(rec + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : ((uint64_t)epoch << 48);
                done = done && (uint32_t)(rv[q] >> 48) == epoch;
            }
            if (__all(done)) break;
            if (wall_clock64() - t_start > a.timeout_ticks) return;  // the main wave times out too
            __builtin_amdgcn_s_sleep(2);
        }
        uint32_t cq[4], iq[4];
        bool ovf = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            cq[q] = (uint32_t)(rv[q] >> 32) & 0xFFFFu;
            iq[q] = (uint32_t)rv[q];
            ovf = ovf || cq[q] == kRecOverflow;
        }
        const uint32_t p1 = cq[0], p2 = p1 + cq[1], p3 = p2 + cq[2], sum = p3 + cq[3];
        const uint32_t incl = wave_incl_sum(sum);
        const uint32_t base = incl - sum;
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        uint64_t o = 0;
        if (!__any(ovf) && T) {
            unsigned long long b = 0;
            if (lane == 0) b = atomicAdd(a.sc_ctr, (unsigned long long)T);
            o = readlane64(b, 0);
            ovf = o + T > a.cand_cap || T >= (1u << 20);
        }
        if (!__any(ovf)) {
            for (uint32_t k0 = 0; k0 < T; k0 += kStageCand) {
                // stage this chunk's candidates in stream order, 8 loads in flight per lane
                for (uint32_t i0 = 0; __any(i0 < sum); i0 += 8) {
                    uint64_t v[8];
                    uint32_t at[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t i = i0 + (uint32_t)u, kk = base + i;
                        const bool ok = i < sum && kk >= k0 && kk < k0 + kStageCand;
                        const uint32_t q = (i >= p1 ? 1u : 0u) + (i >= p2 ? 1u : 0u) + (i >= p3 ? 1u : 0u);
                        const uint32_t ix = q == 0 ? iq[0] + i : q == 1 ? iq[1] + (i - p1)
                                          : q == 2 ? iq[2] + (i - p2) : iq[3] + (i - p3);
                        v[u] = ok ? __hip_atomic_load(cand + ix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                        at[u] = ok ? kk - k0 : ~0u;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (at[u] != ~0u) stc[at[u]] = v[u];
                }
                const uint32_t nhere = T - k0 < (uint32_t)kStageCand ? T - k0 : (uint32_t)kStageCand;
                for (uint32_t v0 = 0; v0 < nhere; v0 += 64) {
                    const int nv = (int)(nhere - v0 < 64 ? nhere - v0 : 64);
                    const uint64_t c = lane < nv ? stc[v0 + lane] : ~0ull;
                    // successor of a cut at this lane's candidate, inside the vector
                    uint64_t sk = c + 1;
                    uint32_t nf = 0;
                    int nx = lane, from = lane + 1;
                    bool active = lane < nv;
                    for (int guard = 0; guard < 64 && __any(active); ++guard) {  // j moves on each round
                        const int j = lanes_lower_bound(c, from, nv, sk + min1);
                        const uint64_t cj = shfl64(c, j < 64 ? j : 63);
                        if (active) {
                            if (j >= nv) {
                                active = false;
                            } else if (cj <= sk + max1) {
                                nx = j;
                                active = false;
                            } else {
                                const uint64_t K = (cj - (sk + max1) + max_eff - 1) >> sh;
                                nf += (uint32_t)K;
                                sk += K * max_eff;
                                from = j;
                            }
                        }
                    }
                    // the chain from every lane: path masks and exit lanes by pointer
                    // doubling (6 rounds: pm covers 2^t nodes, J = the 2^t-th successor)
                    uint64_t pm = (1ull << lane) | (1ull << nx);
                    int xl = nx;
#pragma unroll
                    for (int t = 0; t < 6; ++t) {
                        pm |= shfl64(pm, xl);
                        xl = __shfl(xl, xl, 64);
                    }
                    if (lane < nv) {
                        const uint64_t w = o + k0 + v0 + (uint64_t)lane;
                        sc.c[w] = c;
                        sc.sk[w] = sk;
                        sc.pm[w] = pm;
                        sc.nx[w] = (uint64_t)nf | ((uint64_t)(uint32_t)xl << 32);
                    }
                }
            }
            // helper and main share a CU (workgroup 0): workgroup scope is the hand-off,
            // so the main wave reads the step from L1/L2, not HBM
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        }
        const bool any_ovf = __any(ovf);  // (a ballot inside `lane == 0` would see lane 0 only)
        if (lane == 0) {
            const uint64_t r = ((uint64_t)epoch << 48) | (any_ovf ? (1ull << 47) : 0ull) |
                               ((uint64_t)(T & 0xFFFFFu) << 27) | (o & 0x7FFFFFFull);
            __hip_atomic_store(sinfo + st, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

__device__ void fused_main(const FusedPassArgs& a, uint64_t* keep, int lane) {
    // every field in a register: the struct lives in kernarg memory behind a generic
    // reference and would be re-read after each store
    const uint64_t total = a.ntiles + a.ntail;
    const uint64_t nsteps = (total + kResolveBatch - 1) / kResolveBatch;
    const uint64_t min1 = a.min_eff - 1, max_eff = a.max_eff, max1 = a.max_eff - 1;
    const uint32_t sh = a.max_shift, epoch = a.epoch;
    uint64_t* const cuts_host = a.cuts_host;
    const uint64_t host_cap = a.host_cap;
    const unsigned long long* const sinfo = a.rec + total;
    const FusedStep sc{a.sc_c, a.sc_sk, a.sc_pm, a.sc_nx};
    const uint64_t timeout = a.timeout_ticks, end = a.end;
    uint64_t s = a.s0, ncut = 0;
    // timeout_ticks 0 (PBS_FUSED_TIMEOUT_TICKS=0): fail at once -- the error path's test
    uint32_t nkeep = 0, status = timeout == 0 ? 2u : 0u;
    const uint64_t t_start = wall_clock64();
    uint64_t t_wait = 0, t_ready = t_start;
    const unsigned long long below = (1ull << lane) - 1;

    // cuts go to mapped host memory (a list longer than host_cap stands down) through an
    // LDS buffer: cuts [fl, ncut) wait in cbuf[0, ncut - fl) and go out kCutBuf at a time.
    // Stored one vector at a time, every wait for the next vector's loads also waited for
    // the PCIe acknowledgement of the previous stores (vmcnt counts both): ~1 us per
    // vector, which made the main wave the bottleneck at 64 KiB averages (17.7 ms pass).
    uint64_t* const cbuf = keep + kFusedKeep;  // the second half of the wave's stage
    uint64_t fl = 0;
    auto flush = [&]() {
        const uint64_t nb = ncut - fl;
        for (uint64_t j = (uint64_t)lane; j < nb; j += 64)
            if (fl + j < host_cap) cuts_host[fl + j] = cbuf[j];
        fl = ncut;
    };
    // room for k more cuts: true = put them in cbuf, false = straight to host memory
    auto reserve = [&](uint64_t k) -> bool {
        if (ncut - fl + k <= (uint64_t)kCutBuf) return true;
        flush();
        if (k <= (uint64_t)kCutBuf) return true;
        fl = ncut + k;  // a long run of forced cuts: written directly
        return false;
    };
    auto put = [&](bool lds, uint64_t i, uint64_t x) {
        if (lds)
            cbuf[i - fl] = x;
        else if (i < host_cap)
            cuts_host[i] = x;
    };
    auto forced = [&](uint64_t k) {  // k forced (max-size) cuts from s, lane-parallel
        const bool lds = reserve(k);
        for (uint64_t j = (uint64_t)lane; j < k; j += 64) put(lds, ncut + j, s + (j + 1) * max_eff);
        ncut += k;
        s += k * max_eff;
    };
    // the vector's first cut from state s: ballot over the candidates >= s + min - 1;
    // forced cuts while that candidate lies past s + max - 1.  Returns its lane or -1;
    // `rem` loses the lanes that can no longer cut.
    auto entry = [&](uint64_t c, unsigned long long& rem, bool& reset) -> int {
        for (;;) {
            const unsigned long long m = __ballot(c >= s + min1) & rem;
            if (!m) return -1;
            const int k = __ffsll(m) - 1;
            const uint64_t ck = readlane64(c, k);
            reset = true;
            if (ck > s + max1) {  // the candidates before k stay below every later minimum
                forced((ck - (s + max1) + max_eff - 1) >> sh);
                rem &= ~((1ull << k) - 1);
                continue;
            }
            return k;
        }
    };
    auto keep_rest = [&](uint64_t c, unsigned long long rem, bool reset) {
        if (reset) nkeep = 0;
        const unsigned long long km = __ballot(c >= s) & rem;
        if ((km >> lane) & 1ull) {
            const uint32_t pos = nkeep + (uint32_t)__popcll(km & below);
            if (pos < kFusedKeep) keep[pos] = c;
        }
        nkeep += (uint32_t)__popcll(km);
    };
    // emit the chain `mask` (lanes, ascending), each cut followed by its nf forced cuts
    auto emit_chain = [&](uint64_t c, unsigned long long mask, uint32_t nf) {
        const bool on = (mask >> lane) & 1ull;
        const uint32_t cnt = on ? 1u + nf : 0u;
        uint64_t off;
        uint32_t tot;
        if (__any(on && nf != 0)) {
            const uint32_t incl = wave_incl_sum(cnt);
            off = incl - cnt;
            tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        } else {
            off = (uint64_t)__popcll(mask & below);
            tot = (uint32_t)__popcll(mask);
        }
        const bool lds = reserve(tot);
        if (on) {
            const uint64_t o = ncut + off;
            put(lds, o, c + 1);
            for (uint32_t i = 1; i <= nf; ++i) put(lds, o + i, c + 1 + (uint64_t)i * max_eff);
        }
        ncut += tot;
    };

    // pending candidates of the open chunk (earlier calls): walked cut by cut
    for (uint32_t i = 0; i < a.npend; i += 64) {
        const bool v = i + lane < a.npend;
        const uint64_t c = v ? a.pend[i + lane] : ~0ull;
        unsigned long long rem = __ballot(v);
        bool reset = false;
        for (;;) {
            const int k = entry(c, rem, reset);
            if (k < 0) break;
            emit_chain(c, 1ull << k, 0u);
            s = readlane64(c, k) + 1;
            rem = k == 63 ? 0ull : rem & ~((2ull << k) - 1);
        }
        keep_rest(c, rem, reset);
    }
    // the next step's record and the next vector's data are in flight while the current
    // vector is walked
    auto load_info = [&](uint64_t st) -> uint64_t {
        return st < nsteps ? __hip_atomic_load(sinfo + st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0ull;
    };
    struct Vec {
        uint64_t c, sk, pm, nx;
    };
    // lane i of a vector at v0 (clamped to the step's last candidate: the loads are
    // unconditional, so the compiler can count them in vmcnt)
    auto load_vec = [&](uint64_t o, uint32_t T, uint32_t v0) -> Vec {
        const uint32_t i = v0 + (uint32_t)lane < T ? v0 + (uint32_t)lane : T - 1;
        const uint64_t w = o + i;
        return Vec{sc.c[w], sc.sk[w], sc.pm[w], sc.nx[w]};
    };
    // one vector: the first cut from the incoming state, then the chain the helper
    // precomputed from that lane
    auto walk = [&](const Vec& q, uint32_t v0, uint32_t T) {
        const bool v = v0 + (uint32_t)lane < T;
        const uint64_t c = v ? q.c : ~0ull;
        unsigned long long rem = __ballot(v);
        bool reset = false;
        const int e = entry(c, rem, reset);
        // read unconditionally (lane 0 when no cut): used only under the branch, the loads
        // were sunk into it and issued one vector ahead instead of kMainAhead
        const int ee = e < 0 ? 0 : e;
        const unsigned long long mask = readlane64(q.pm, ee);
        const int x = __builtin_amdgcn_readlane((int)(uint32_t)(q.nx >> 32), ee);
        const uint64_t sx = readlane64(q.sk, x);
        if (e >= 0) {
            emit_chain(c, mask, (uint32_t)q.nx);
            s = sx;
            rem = x == 63 ? 0ull : rem & ~((2ull << x) - 1);
        }
        keep_rest(c, rem, reset);
    };
    uint64_t r_next = load_info(0);
    for (uint64_t st = 0; st < nsteps && status == 0; ++st) {
        uint64_t r = r_next;
        if ((uint32_t)(r >> 48) != epoch) {
            const uint64_t w0 = wall_clock64();
            while ((uint32_t)(r >> 48) != epoch) {
                if (wall_clock64() - t_start > timeout) {
                    status = 2;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
                r = load_info(st);
            }
            t_ready = wall_clock64();
            t_wait += t_ready - w0;
            if (status) break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the step's scratch is visible
        r_next = load_info(st + 1);
        if ((r >> 47) & 1ull) {
            status = 1;
            break;
        }
        const uint32_t T = (uint32_t)(r >> 27) & 0xFFFFFu;
        const uint64_t o = r & 0x7FFFFFFull;
        // kMainAhead vectors in flight, in a ring walked in place: rotating them through
        // copies (cur = next) made every vector wait for the loads issued with it
        if (T) {
            Vec q[kMainAhead];
#pragma unroll
            for (int i = 0; i < kMainAhead; ++i) q[i] = load_vec(o, T, 64u * i);
            for (uint32_t v0 = 0; v0 < T; v0 += 64u * kMainAhead) {
#pragma unroll
                for (int i = 0; i < kMainAhead; ++i) {
                    const uint32_t vi = v0 + 64u * i;
                    if (vi < T) {
                        walk(q[i], vi, T);
                        q[i] = load_vec(o, T, vi + 64u * kMainAhead);
                    }
                }
            }
        }
        if ((st & 7) == 7 && lane == 0) {  // progress: the host copies the cuts stored so far
            const uint64_t done = fl < ncut ? fl : ncut;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(a.res_host + 9, done < host_cap ? done : host_cap, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (status == 0) {
        if (s + max_eff <= end) {  // no candidate left: forced cuts up to the end
            forced((end - s) >> sh);
            nkeep = 0;
        }
        if (nkeep > kFusedKeep || ncut > host_cap) status = 1;
    }
    if (fl < ncut) flush();
    if (status == 0 && nkeep <= a.keep_cap)
        for (uint32_t i = lane; i < nkeep; i += 64) a.keep_host[i] = keep[i];
    if ((uint32_t)lane < a.tail_len) a.tail_host[lane] = a.tail_src[lane];
    if (lane == 0) {
        const uint64_t t_end = wall_clock64();
        a.res_host[0] = ncut;
        a.res_host[1] = s;
        a.res_host[2] = nkeep;
        a.res_host[4] = __hip_atomic_load(a.ncand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.res_host[5] = __hip_atomic_load(a.nflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.res_host[6] = t_ready - t_start;  // diagnostics (100 MHz ticks): last step ready,
        a.res_host[7] = t_end - t_start;    // resolver done, time spent waiting for steps
        a.res_host[8] = t_wait;
        // last, after every other result (and the cuts) is in host memory: the host
        // returns as soon as it sees this word
        __hip_atomic_store(a.res_host + 3, (uint64_t)status, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#ifdef PBS_SCAN_PROBE  // scripts/microbench/fused_probe.py: per-wave start / tiles done / done
__device__ uint64_t g_fused_probe[4 * kScanProbeMax];  // start, tiles done, done, SIMD
#define PBS_FUSED_STAMP(k)                                                               \
    if (lane == 0 && blockIdx.x * NW + wave < kScanProbeMax)                             \
        g_fused_probe[(k) * kScanProbeMax + blockIdx.x * NW + wave] = wall_clock64();
#else
#define PBS_FUSED_STAMP(k)
#endif

// SEG: segment bytes per lane (16/32 KiB: the fused pass serves batches of >= 1 MiB);
// DYN: tile order as scan_main_kernel.  8 waves per workgroup, one workgroup per CU.
template <int SEG, int DYN>
__global__ __launch_bounds__(kWavesPerWG * 64) void scan_fused_kernel(FusedPassArgs a) {
    static_assert(SEG % 4096 == 0, "bitmap words per lane");
    constexpr int SEG2 = SEG / 4;
    constexpr int NW = kWavesPerWG;
    constexpr int NBW = SEG / kIter / 32;  // bitmap words per lane (one bit per block)
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords + NW * kStagePerWave / 4];
    __shared__ uint32_t s_bm[NW * 64 * NBW];
    __shared__ uint32_t s_simd[NW], s_prog[NW];  // SIMD of each wave; blocks scanned so far

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTableDwords; i += NW * 64) s_lds[i] = a.table_rot[i >> 6];
    for (int i = tid; i < NW * 64 * NBW; i += NW * 64) s_bm[i] = 0;
    if (lane == 0) {
        s_simd[wave] = (__builtin_amdgcn_s_getreg(kHwRegHwId) >> 4) & 3u;  // HW_ID.SIMD_ID
        s_prog[wave] = 0;
    }
    __syncthreads();
    // SIMD partner: the other wave of this workgroup on the same SIMD (the issue arbiter
    // favours the older one by ~30 %: probe, scripts/microbench/fused_probe.py), or none
    int partner = wave;
    for (int w = 0; w < NW; ++w)
        if (w != wave && s_simd[w] == s_simd[wave]) partner = w;
    partner = __builtin_amdgcn_readfirstlane(partner);
    const bool balance = a.balance != 0 && partner != wave;  // equal progress of SIMD partners
    const bool bal_sleep = a.balance == 2;
    uint8_t* stage = (uint8_t*)(s_lds + kTableDwords) + wave * kStagePerWave;
    PBS_FUSED_STAMP(0)
    const bool resolver = __builtin_amdgcn_readfirstlane(a.resolver) != 0;
    const uint32_t nres = resolver ? 1u + kFusedHelpers : 0u;  // resolver waves (workgroup 0)
    const uint32_t G = __builtin_amdgcn_readfirstlane(a.groups);  // records per tile
    if (resolver && blockIdx.x == 0 && wave == 0) {
        fused_main(a, reinterpret_cast<uint64_t*>(stage), lane);
        return;
    }
    if (resolver && blockIdx.x == 0 && wave <= kFusedHelpers) {
        fused_helper(a, reinterpret_cast<uint64_t*>(stage), wave - 1, kFusedHelpers, lane);
        return;
    }
    uint32_t* bm = s_bm + wave * 64 * NBW + lane * NBW;

    const uint32_t lanebase = (uint32_t)lane * 4u;
    // LDS-DMA lane offsets of a tile with segments of `seg` bytes: instruction j stages
    // lines of segments 8j..8j+7, chunk k of lane l's line at the XOR-swizzled slot
    uint32_t voff[8], voff2[8];
    auto set_voff = [&](uint32_t (&v)[8], uint32_t seg) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t l = 8u * j + ((uint32_t)lane >> 3);
            const uint32_t k = ((uint32_t)lane & 7u) ^ ((l >> 1) & 7u);
            v[j] = l * seg + k * 16u;
        }
    };
    if constexpr (DYN != 0) {
        set_voff(voff, (uint32_t)SEG);
        set_voff(voff2, (uint32_t)SEG2);
    }
    const uint32_t rd_base = (uint32_t)lane * 128u;
    const uint32_t rsw = ((uint32_t)lane >> 1) & 7u;
    // scanner waves: all but workgroup 0's resolver waves
    const uint64_t nw = (uint64_t)gridDim.x * NW - nres;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave - nres;
    const uint64_t ntiles = a.ntiles, t_big = a.t_big;
    const uint8_t* data = a.data;

    // tile geometry.  DYN: SEG-byte segments, SEG2 from tile t_big on.  Static: two groups
    // of runtime segment lengths (FusedPassArgs; the host sizes them so the tiles cover the
    // batch up to < 8 KiB, every scanner wave gets the same work, and the last round is short)
    // (wave-uniform copies: selecting between two fields of `a` made the compiler load the
    // chosen one through a computed address in VGPRs, and the static kernel spill)
    const uint32_t g_q = __builtin_amdgcn_readfirstlane(a.seg_q);
    const uint32_t g_qs = __builtin_amdgcn_readfirstlane(a.seg_qs);
    const uint64_t g_tl = uni64(a.t_long), g_ts = uni64(a.t_small), g_tsl = uni64(a.t_small_long);
    auto tile_nit = [&](uint64_t t) -> uint32_t {  // blocks per segment
        if constexpr (DYN != 0)
            return (uint32_t)((t >= t_big ? SEG2 : SEG) / kIter);
        else
            return t < g_ts ? g_q + (t < g_tl ? 1u : 0u) : g_qs + (t - g_ts < g_tsl ? 1u : 0u);
    };
    auto tile_off = [&](uint64_t t) -> uint64_t {
        if constexpr (DYN != 0) {
            if (t >= t_big) return t_big * (64ull * SEG) + (t - t_big) * (64ull * SEG2);
            return t * (64ull * SEG);
        } else {
            if (t < g_ts) return (t * g_q + (t < g_tl ? t : g_tl)) * (64ull * kIter);
            const uint64_t u = t - g_ts;
            return (g_ts * g_q + g_tl + u * g_qs + (u < g_tsl ? u : g_tsl)) * (64ull * kIter);
        }
    };
    auto issue = [&](uint64_t t, int it) {  // scan_main_kernel's LDS-DMA of one iteration
        const bool sm = DYN != 0 && t >= t_big;
        const uint8_t* tb = data + tile_off(t);
        const bool first = (t == 0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(first ? tb : tb - kIter), 0, (int)(64u * tile_nit(t) * kIter + kIter), 0x00020000);
        const bool warm0 = first && it == 0;
        const uint32_t soff = warm0 ? 0u : (uint32_t)it * kIter - (first ? (uint32_t)kIter : 0u);
        if (sm) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, voff2[j], soff, 0, 2);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t vo = warm0 ? (voff[j] >= (uint32_t)kIter ? voff[j] - kIter : 0u) : voff[j];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, vo, soff, 0, 2);
            }
        }
    };
    // the wave's flagged blocks of tile t (bitmap, lane order = stream order) -> publish,
    // 64 blocks per record (records t * G .. t * G + G - 1; more blocks: overflow)
    auto tile_end = [&](uint64_t t, uint64_t toff, uint32_t seg_cur) {
        uint32_t w[NBW];
#pragma unroll
        for (int q = 0; q < NBW; ++q) {
            w[q] = bm[q];
            bm[q] = 0;
        }
        if (t == 0 && lane == 0) w[0] |= 1u;  // the stream's first block: carry bytes
        for (uint32_t g = 0;; ++g) {
            int nb = 0;
            bool over = false, more = false;
            int64_t myB = 0;
            for (;;) {
                bool has = false;
#pragma unroll
                for (int q = 0; q < NBW; ++q) has |= w[q] != 0u;
                const unsigned long long m = __ballot(has);
                if (!m) break;
                if (nb == 64) {
                    more = true;
                    over = g + 1 == G;
                    break;
                }
                const int L = __ffsll(m) - 1;
                int bitpos = 0;
                bool found = false;
#pragma unroll
                for (int q = 0; q < NBW; ++q) {
                    if (!found && w[q]) {
                        bitpos = q * 32 + __builtin_ctz(w[q]);
                        found = true;
                    }
                }
                bitpos = __builtin_amdgcn_readlane(bitpos, L);  // L is wave-uniform
                if (lane == L) {
#pragma unroll
                    for (int q = 0; q < NBW; ++q)
                        if (q == (bitpos >> 5)) w[q] &= w[q] - 1;
                }
                if (lane == nb) myB = (int64_t)(toff + (uint64_t)L * seg_cur + (uint64_t)bitpos * kIter);
                ++nb;
            }
            if (nb && lane == 0) atomicAdd(a.nflag, (unsigned long long)nb);
            fused_publish(a, s_lds, t * G + g, myB, nb, over, lane);
            if (!more || over) break;
        }
    };

    const bool pool = DYN == 0 && __builtin_amdgcn_readfirstlane(a.pool) != 0;
    if (pool && tile >= g_ts) {  // no static tile: the counter hands out the rest
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(a.tile_ctr, 1u);
        tile = g_ts + (uint64_t)__builtin_amdgcn_readfirstlane(v);
    }
    if (tile < ntiles) {
        uint32_t ring[128];
#pragma unroll
        for (int r = 0; r < 128; ++r) ring[r] = 0;
        uint32_t h = 0;
        uint32_t dyn_v = 0;
        uint32_t prog = 0;  // blocks scanned (wave-uniform)
        // static order with a pool (a.pool): tiles [0, t_small) round-robin, then the pool's
        // short tiles from the counter (drawn at the start of a wave's last static tile)
        auto next_tile = [&]() -> uint64_t {
            if constexpr (DYN != 0)
                return nw + (uint64_t)__builtin_amdgcn_readfirstlane(dyn_v);
            else
                return (pool && tile + nw >= g_ts)
                           ? g_ts + (uint64_t)__builtin_amdgcn_readfirstlane(dyn_v)
                           : tile + nw;
        };
        if constexpr (DYN == 0) set_voff(voff, tile_nit(tile) * kIter);
        issue(tile, 0);
        for (;;) {
            if (DYN != 0 || (pool && tile + nw >= g_ts)) {
                if (lane == 0) dyn_v = atomicAdd(a.tile_ctr, 1u);
            }
            const int nit_cur = (int)tile_nit(tile) + 1;  // + the warm-up block
            const uint64_t toff = tile_off(tile);
            const uint32_t seg_cur = tile_nit(tile) * kIter;
            for (int it = 0; it < nit_cur; ++it) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                uint32_t d[32];
                if (balance) {
                    if (lane == 0) s_prog[wave] = prog;
                }
                const uint32_t pprog = balance ? s_prog[partner] : 0u;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint4 v = *(const uint4*)(stage + rd_base + (((uint32_t)k ^ rsw) << 4));
                    d[4 * k] = v.x;
                    d[4 * k + 1] = v.y;
                    d[4 * k + 2] = v.z;
                    d[4 * k + 3] = v.w;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (balance) {
                    // the wave behind its SIMD partner takes the issue priority until it
                    // has caught up, so both finish together
                    const uint32_t pp = __builtin_amdgcn_readfirstlane(pprog);
                    if (pp > prog)
                        __builtin_amdgcn_s_setprio(2);
                    else
                        __builtin_amdgcn_s_setprio(0);
                    if (bal_sleep && prog > pp + 2) __builtin_amdgcn_s_sleep(1);  // ahead: yield
                    ++prog;
                }
                {
                    uint64_t nt = tile;
                    int nit = it + 1;
                    if (nit == nit_cur) {
                        nt = next_tile();
                        nit = 0;
                        // static order: the next tile's segment length (this tile issues no more)
                        if constexpr (DYN == 0)
                            if (nt < ntiles) set_voff(voff, tile_nit(nt) * kIter);
                    }
                    if (nt < ntiles) issue(nt, nit);
                }
                if (it == 0) {
                    h = 0;
#pragma unroll
                    for (int r = 64; r < 128; ++r) ring[r] = 0;
                }
                const uint32_t acc = roll128_asm_g4(d, ring, h, lanebase);
                if (it == 0) {
                    if (tile == 0 && lane == 0) {  // no bytes before the stream: no warm-up
                        h = 0;
#pragma unroll
                        for (int r = 64; r < 128; ++r) ring[r] = 0;
                    }
                } else if (acc >= a.thr) {
                    const uint32_t bit = (uint32_t)(it - 1);
                    atomicOr(&bm[bit >> 5], 1u << (bit & 31u));
                }
            }
            tile_end(tile, toff, seg_cur);
            tile = next_tile();
            if (tile >= ntiles) break;
        }
    }
    PBS_FUSED_STAMP(1)
    // the bytes past the last tile: items of kTailBlocks consecutive blocks
    const uint64_t nblk = (a.len + kIter - 1) / kIter;
    while (tile < ntiles + a.ntail) {
        const uint64_t b0 = a.covered / kIter + (tile - ntiles) * kTailBlocks;
        const int nb = (int)(nblk - b0 < (uint64_t)kTailBlocks ? nblk - b0 : (uint64_t)kTailBlocks);
        fused_publish(a, s_lds, tile * G, (int64_t)((b0 + (uint64_t)lane) * kIter), nb, false, lane);
        if (DYN != 0 || pool) {
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(a.tile_ctr, 1u);
            tile = (DYN != 0 ? nw : g_ts) + (uint64_t)__builtin_amdgcn_readfirstlane(v);
        } else {
            tile += nw;
        }
    }
    PBS_FUSED_STAMP(2)
#ifdef PBS_SCAN_PROBE  // SIMD and partner, stored last (stored at the start, it made the probe
                       // build of the static kernel spill: probe timings of such a build are void)
    if (lane == 0 && blockIdx.x * NW + wave < kScanProbeMax)
        g_fused_probe[3 * kScanProbeMax + blockIdx.x * NW + wave] = s_simd[wave] | ((uint64_t)partner << 8);
#endif
}

}  // namespace pbs
