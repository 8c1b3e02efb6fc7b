// scan_server_kernel: the low-latency path of pbs_chunker_scan (Chunker::scan,
// chunker.rs:112-168, called by ChunkStream on every read, chunk_stream.rs:40-77).
//
// ONE persistent workgroup polls the mailbox (pbs_chunker_internal.h) in fine-grained
// pinned host memory with 16-byte loads {seq, len | quit, base} (kSrvPollAll: lane 0 of
// every wave, staggered -- measured no faster, off by default).  A request
// then costs one more PCIe round trip: the slot's history and data (host memory) are
// staged in LDS, 32 KiB per pass, all loads in flight at once.  The cut test runs at
// every position, each of the 256 threads over S = 32, 64 or 128 bytes (the shortest
// that covers the pass: an 8 KiB read is 64 + 32 steps per lane; the reference's
// recurrence, chunker.rs:118-165, test :185).
// The hits are compacted in stream order into the mailbox, and after every wave drained
// its stores the acknowledgement -- seq, candidate count and overflow flag in one 8-byte
// word -- is stored (system-scope release).  The host applies
// shall_break's min/max rule to the returned candidates.  Exit: the quit flag, or
// idle_ticks (wall_clock64, 100 MHz) without a request -- the host relaunches it on the
// next call (pbs_chunker_capi.cpp server_scan), so a process that stops calling leaves
// no kernel running.  kSrvProbe: per-request phase stamps (PBS_SERVER_PROBE=1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_block.h"
#include "pbs_chunker_internal.h"

namespace pbs {

constexpr int kSrvThreads = 256;  // 4 waves, one per SIMD
constexpr int kSrvPass = 32 * 1024;  // bytes staged per pass
static_assert(kSrvPass == 128 * kSrvThreads, "a pass is at most 128 bytes per thread");

typedef uint32_t srv_u32x4 __attribute__((ext_vector_type(4)));

// hits of the S bytes at sd[B .. B+S) (LDS; sd[B-64 .. B) readable): bit i of word i / 32
// = the window ending at byte B + i passes the test -- 64 fill steps over the bytes before
// the segment (the window hash of chunker.rs:118-136), S roll steps (:141-165), the test
// (:185); one lane per segment, every lane of the workgroup busy
template <int S>
__device__ __forceinline__ uint4 lane_hits(const uint8_t* sd, int B, const uint32_t* tab, uint32_t mask,
                                           uint32_t minimum) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(sd + B - 64);
    uint32_t d[(64 + S) / 4];
#pragma unroll
    for (int k = 0; k < (64 + S) / 4; ++k) d[k] = w[k];
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i)
        h = __builtin_amdgcn_alignbit(h, h, 31) ^ tab[(d[i >> 2] >> (8 * (i & 3))) & 0xffu];
    uint32_t hw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const uint32_t out = (d[i >> 2] >> (8 * (i & 3))) & 0xffu;
        const uint32_t in = (d[(i + 64) >> 2] >> (8 * (i & 3))) & 0xffu;
        h = __builtin_amdgcn_alignbit(h, h, 31) ^ tab[out] ^ tab[in];
        hw[i >> 5] |= ((h & mask) >= minimum ? 1u : 0u) << (i & 31);
    }
    return make_uint4(hw[0], hw[1], hw[2], hw[3]);
}

__global__ __launch_bounds__(kSrvThreads) void scan_server_kernel(ServerMailbox* mb,
                                                                  const uint8_t* __restrict__ slot,
                                                                  uint32_t mask, uint32_t minimum,
                                                                  uint64_t last_seq,
                                                                  uint64_t idle_ticks, uint32_t flags) {
    __shared__ uint32_t tab[256];
    __shared__ __attribute__((aligned(16))) uint8_t st[kServerHist + kSrvPass + 128];
    __shared__ uint32_t wsum[kSrvThreads / 64];
    __shared__ uint32_t s_go;    // 0 polling, 1 serve, 2 exit
    __shared__ uint64_t ctl[2];  // [0] seq | len << 32 [1] base
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool poll_all = (flags & kSrvPollAll) != 0, probe = (flags & kSrvProbe) != 0;
    for (int i = tid; i < 256; i += kSrvThreads) tab[i] = kBuzhashTable[i];
    if (tid == 0) s_go = 0;
    __syncthreads();
    uint32_t last = (uint32_t)last_seq;
    uint64_t t_idle = wall_clock64();
    for (;;) {
        // poll the request record (one 16-byte load {seq, len | quit, base}); with
        // kSrvPollAll lane 0 of every wave polls, the waves staggered so that several
        // PCIe reads are in flight and a new request is seen sooner
        if (lane == 0 && (poll_all || wave == 0)) {
            if (poll_all)
                for (int d = 0; d < wave; ++d) __builtin_amdgcn_s_sleep(8);
            for (;;) {
                if (__hip_atomic_load(&s_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                const srv_u32x4 r = *reinterpret_cast<volatile srv_u32x4*>(&mb->req_seq);  // {seq, len, base}
                uint32_t go = 0;
                if (r.y & kServerQuit) {
                    go = 2;
                } else if (r.x != last) {
                    ctl[0] = (uint64_t)r.x | ((uint64_t)r.y << 32);
                    ctl[1] = (uint64_t)r.z | ((uint64_t)r.w << 32);
                    go = 1;
                } else if (wall_clock64() - t_idle > idle_ticks) {
                    go = 2;
                }
                if (go) {
                    __hip_atomic_store(&s_go, go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (!poll_all) __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the slot is read after the record
        if (s_go != 1) {
            if (tid == 0)
                __hip_atomic_store(&mb->exited, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;  // uniform
        }
        const uint64_t t_seen = probe ? wall_clock64() : 0;
        uint64_t t_staged = 0, t_hashed = 0;
        const uint32_t seq = (uint32_t)ctl[0], len = (uint32_t)(ctl[0] >> 32);
        const uint64_t base = ctl[1];
        uint32_t total = 0;
        for (uint32_t off = 0; off < len; off += kSrvPass) {
            const uint32_t plen = len - off < (uint32_t)kSrvPass ? len - off : (uint32_t)kSrvPass;
            // stream positions < 63 have no full window (chunker.rs:118-136): never reported
            const uint64_t pos0 = base + off;
            const uint32_t lo_ok = pos0 >= 63 ? 0u : (uint32_t)(63 - pos0);
            // pass 0 stages the slot's history with the data; later passes keep the
            // previous pass's last 64 bytes as theirs
            const uint32_t src0 = off == 0 ? 0u : kServerHist + off;
            const uint32_t dst0 = off == 0 ? 0u : kServerHist;
            if (off > 0) {
                uint8_t v = 0;
                if (tid < 64) v = st[kSrvPass + tid];
                __syncthreads();
                if (tid < 64) st[tid] = v;
            }
            const uint32_t nbytes = off == 0 ? kServerHist + plen : plen;
            const uint32_t n16 = nbytes / 16;
            const srv_u32x4* src = reinterpret_cast<const srv_u32x4*>(slot + src0);
            for (uint32_t i0 = tid; i0 < n16; i0 += 8 * kSrvThreads) {  // 8 loads in flight
                srv_u32x4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t i = i0 + (uint32_t)u * kSrvThreads;
                    if (i < n16) v[u] = __builtin_nontemporal_load(src + i);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t i = i0 + (uint32_t)u * kSrvThreads;
                    if (i < n16) *reinterpret_cast<srv_u32x4*>(st + dst0 + 16 * i) = v[u];
                }
            }
            for (uint32_t i = n16 * 16 + tid; i < nbytes; i += kSrvThreads) st[dst0 + i] = slot[src0 + i];
            __syncthreads();
            if (probe && off == 0) t_staged = wall_clock64();
            // the cut test at every position: thread t takes the S bytes at t * S (S = 32,
            // 64 or 128: the shortest that covers the pass with the 256 threads)
            const uint32_t S = plen <= 32 * kSrvThreads ? 32u : plen <= 64 * kSrvThreads ? 64u : 128u;
            uint4 h = make_uint4(0, 0, 0, 0);
            if (tid * S < plen) {
                const uint8_t* const sd = st + kServerHist;
                h = S == 32 ? lane_hits<32>(sd, (int)(tid * S), tab, mask, minimum)
                    : S == 64 ? lane_hits<64>(sd, (int)(tid * S), tab, mask, minimum)
                              : lane_hits<128>(sd, (int)(tid * S), tab, mask, minimum);
                uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {  // reportable positions [lo_ok, plen)
                    const int p0 = (int)(tid * S) + 32 * q;
                    const int lo = (int)lo_ok - p0, up = (int)plen - p0;
                    const uint32_t keep_lo = lo <= 0 ? 0xFFFFFFFFu : (lo >= 32 ? 0u : (0xFFFFFFFFu << lo));
                    const uint32_t keep_hi = up >= 32 ? 0xFFFFFFFFu : (up <= 0 ? 0u : (0xFFFFFFFFu >> (32 - up)));
                    hw[q] &= q < (int)(S / 32) ? keep_lo & keep_hi : 0u;
                }
                h = make_uint4(hw[0], hw[1], hw[2], hw[3]);
            }
            if (probe && off == 0) t_hashed = wall_clock64();
            // stream-order compaction: thread t owns positions [t S, t S + S)
            const uint32_t c = __builtin_popcount(h.x) + __builtin_popcount(h.y) +
                               __builtin_popcount(h.z) + __builtin_popcount(h.w);
            uint32_t x = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (lane >= d) x += y;
            }
            if (lane == 63) wsum[wave] = x;
            __syncthreads();
            uint32_t before = total, all = total;
#pragma unroll
            for (int w2 = 0; w2 < kSrvThreads / 64; ++w2) {
                before += w2 < wave ? wsum[w2] : 0u;
                all += wsum[w2];
            }
            uint32_t o = before + x - c;
            const uint32_t w4[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t m = w4[q];
                while (m) {
                    const int bit = __builtin_ctz(m);
                    m &= m - 1;
                    if (o < kServerCand) mb->cand[o] = pos0 + (uint64_t)(tid * S + q * 32 + bit);
                    ++o;
                }
            }
            total = all;
            __syncthreads();  // st, hv, wsum reused by the next pass
        }
        // every wave's stores drained, then the acknowledgement (system scope)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            if (probe) {
                mb->probe[0] = t_seen;
                mb->probe[1] = t_staged;
                mb->probe[2] = t_hashed;
                mb->probe[3] = wall_clock64();
            }
            s_go = 0;
            // ONE 8-byte store: seq, candidate count, overflow flag (the host reads them together)
            const uint64_t ack = (uint64_t)seq | (uint64_t)(total < kServerCand ? total : kServerCand) << 32 |
                                 (total > kServerCand ? 1ull << 63 : 0ull);
            __hip_atomic_store(&mb->ack_seq, ack, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        last = seq;
        t_idle = wall_clock64();
    }
}

}  // namespace pbs
