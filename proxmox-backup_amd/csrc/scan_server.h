// scan_server_kernel: the low-latency path of pbs_chunker_scan (Chunker::scan,
// chunker.rs:112-168, called by ChunkStream on every read, chunk_stream.rs:40-77).
//
// ONE persistent workgroup polls the mailbox (pbs_chunker_internal.h) in fine-grained
// pinned host memory with one 16-byte load {seq, len | quit, base}.  A request then costs one
// more PCIe round trip: the slot's history and data (host memory) are staged in LDS,
// 32 KiB per pass, all loads in flight at once.  The cut test runs at every position --
// one 128-byte block per lane, the blocks spread over the four SIMDs: 64 fill steps over
// the bytes before the block (the window hash of chunker.rs:118-136), 128 roll steps
// (:141-165) and the test (h & mask) >= mask - 2 (:185).  The hits are compacted in stream
// order into the mailbox, and after every wave drained its stores the acknowledgement is
// stored (system-scope release).  The host applies shall_break's min/max rule to the
// returned candidates.  Exit: the quit flag, or idle_ticks (wall_clock64, 100 MHz) without
// a request -- the host relaunches it on the next call (pbs_chunker_capi.cpp server_scan),
// so a process that stops calling leaves no kernel running.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbs_chunker_internal.h"

namespace pbs {

constexpr int kSrvThreads = 256;  // 4 waves, one per SIMD
constexpr int kSrvPass = 32 * 1024;  // bytes staged per pass
constexpr int kSrvBlocks = kSrvPass / 128;
static_assert(kSrvBlocks == kSrvThreads, "one block per thread");

// hits of the 128-byte block at sd[B .. B+128) (LDS; sd[B-64 .. B) readable): bit i = the
// window ending at byte B + i passes the test
__device__ __forceinline__ uint4 lane_block_hits(const uint8_t* sd, int B, const uint32_t* tab,
                                                 uint32_t mask, uint32_t minimum) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(sd + B - 64);
    uint32_t d[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) d[k] = w[k];
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i)
        h = __builtin_amdgcn_alignbit(h, h, 31) ^ tab[(d[i >> 2] >> (8 * (i & 3))) & 0xffu];
    uint32_t hw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 128; ++i) {
        const uint32_t out = (d[i >> 2] >> (8 * (i & 3))) & 0xffu;
        const uint32_t in = (d[(i + 64) >> 2] >> (8 * (i & 3))) & 0xffu;
        h = __builtin_amdgcn_alignbit(h, h, 31) ^ tab[out] ^ tab[in];
        hw[i >> 5] |= ((h & mask) >= minimum ? 1u : 0u) << (i & 31);
    }
    return make_uint4(hw[0], hw[1], hw[2], hw[3]);
}

typedef uint32_t srv_u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kSrvThreads) void scan_server_kernel(ServerMailbox* mb,
                                                                  const uint8_t* __restrict__ slot,
                                                                  uint32_t mask, uint32_t minimum,
                                                                  uint64_t last_seq,
                                                                  uint64_t idle_ticks) {
    __shared__ uint32_t tab[256];
    __shared__ __attribute__((aligned(16))) uint8_t st[kServerHist + kSrvPass + 128];
    __shared__ uint4 hv[kSrvBlocks];
    __shared__ uint32_t wsum[kSrvThreads / 64];
    __shared__ uint64_t ctl[3];  // [0] command (1 serve, 2 exit) [1] seq | len << 32 [2] base
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 256; i += kSrvThreads) tab[i] = kBuzhashTable[i];
    uint32_t last = (uint32_t)last_seq;
    uint64_t t_idle = wall_clock64();
    for (;;) {
        if (tid == 0) {
            uint64_t cmd = 2;
            srv_u32x4 r = {last, 0u, 0u, 0u};
            for (;;) {
                r = *reinterpret_cast<volatile srv_u32x4*>(&mb->req_seq);  // {seq, len, base}
                if (r.y & kServerQuit) break;
                if (r.x != last) {
                    cmd = 1;
                    break;
                }
                if (wall_clock64() - t_idle > idle_ticks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the slot is read after the record
            ctl[0] = cmd;
            ctl[1] = (uint64_t)r.x | ((uint64_t)r.y << 32);
            ctl[2] = (uint64_t)r.z | ((uint64_t)r.w << 32);
        }
        __syncthreads();
        if (ctl[0] != 1) {
            if (tid == 0)
                __hip_atomic_store(&mb->exited, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;  // uniform
        }
        const uint32_t seq = (uint32_t)ctl[1], len = (uint32_t)(ctl[1] >> 32);
        const uint64_t base = ctl[2];
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
            const int nblk = (int)((plen + 127) / 128);
            {
                // block b runs on lane b/4 of wave b%4: small requests use all four SIMDs
                const int b = (tid & 63) * 4 + (tid >> 6);
                if (b < nblk) {
                    uint4 h = lane_block_hits(st + kServerHist, b * 128, tab, mask, minimum);
                    uint32_t hw[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {  // reportable positions [lo_ok, plen)
                        const int p0 = b * 128 + 32 * q;
                        const int lo = (int)lo_ok - p0, up = (int)plen - p0;
                        const uint32_t keep_lo = lo <= 0 ? 0xFFFFFFFFu : (lo >= 32 ? 0u : (0xFFFFFFFFu << lo));
                        const uint32_t keep_hi = up >= 32 ? 0xFFFFFFFFu : (up <= 0 ? 0u : (0xFFFFFFFFu >> (32 - up)));
                        hw[q] &= keep_lo & keep_hi;
                    }
                    hv[b] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
                }
            }
            __syncthreads();
            // stream-order compaction: thread t owns block t
            const uint4 h = tid < nblk ? hv[tid] : make_uint4(0, 0, 0, 0);
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
                    if (o < kServerCand) mb->cand[o] = pos0 + (uint64_t)(tid * 128 + q * 32 + bit);
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
            mb->ncand = total < kServerCand ? total : kServerCand;
            mb->status = total > kServerCand ? 1u : 0u;
            __hip_atomic_store(&mb->ack_seq, (uint64_t)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = seq;
        t_idle = wall_clock64();
    }
}

}  // namespace pbs
