// scan_server_kernel: the low-latency path of pbs_chunker_scan (Chunker::scan,
// chunker.rs:112-168, called by ChunkStream on every read, chunk_stream.rs:40-77).
//
// Persistent workgroups: workgroup 0 (the leader) polls the request record (pbs_chunker_internal.h ServerReq)
// with 16-byte loads {seq, len | quit, base} (kSrvPollAll: lane 0 of every wave,
// staggered), then every lane loads its 32 bytes of the slot straight into registers (8 KiB
// per pass over 256 lanes; the next kSrvAhead passes' bytes in flight while one is hashed).
// kSrvDevReq (the default since round 3): record and slot live in fine-grained VRAM that the
// host writes through the BAR (posted write-combined stores), so polling and the slot
// reads stay in this GPU's HBM -- 8 KiB round trip 7.2 -> 4.9 us in
// scripts/microbench/mb_bar.hip.  Otherwise both sit in the mailbox's pinned host memory
// and cost PCIe round trips (a dependent load of host memory ~1.2 us, 8 KiB ~1.6 us,
// mb_poll.hip).  Acknowledgement and candidates always go to pinned host memory.
//
// The hash at every position without the 64-step warm-up per lane: with the chain
// Q(j) = rotl(Q(j-1), 1) ^ T[b_j] over the whole slot, h(j) = Q(j) ^ Q(j-64) (rotations are
// mod 32, so the terms 64 back cancel; the reference's recurrence, chunker.rs:118-165).
// Lane t owns the 32 bytes at 32 t and runs the chain from its first byte (Q_t); with
// A_u = Q_u(31) and E_u = Q(32 u - 1) (so E_{u+1} = rotl(E_u, 32) ^ A_u = E_u ^ A_u),
//     h(32 t + i) = Q_t(i) ^ Q_{t-2}(i) ^ rotl(E_t ^ E_{t-2}, i + 1),
//     E_t ^ E_{t-2} = A_{t-2} ^ A_{t-1},
// so a lane needs the chain of the lane two back (LDS rows) and one more total.  The 64
// bytes before a pass are "lanes" -2 and -1: the slot's history (first pass; their chains
// by a rotating prefix over 32-lane halves of one wave) or the previous pass's last two
// rows.  Per byte: one address op, one table read (64 replicas, conflict-free), the
// chain's two ops, then two for h and half a max -- against ~3x that for a warm-up of 64
// steps per 32 bytes (the previous kernel: 8 KiB reads 1.22 GiB/s).  16 bytes per lane
// over 512 lanes measured slower for 8 KiB reads (1.25 vs 1.43 GiB/s: eight waves to
// synchronize; 256 KiB reads gain, 3.6 vs 2.7 GB/s, from the prefetch kept here).  The
// table is pre-rotated by the handle (T' = rotl(T, rot)), so h' = rotl(h, rot) and the
// test (h & mask) >= mask - 2 (:185) is h' >= thr; a max over the lane's positions
// screens (32 positions per lane), and only lanes with a hit build their bit masks.
//
// The hits are compacted in stream order into the mailbox, and after every wave drained
// its stores the acknowledgement -- seq, candidate count and overflow flag in one 8-byte
// word -- is stored (system-scope release).  The host applies shall_break's min/max rule
// to the returned candidates.  Exit: the quit flag, or idle_ticks (wall_clock64, 100 MHz)
// without a request -- the host relaunches it on the next call (pbs_chunker_capi.cpp
// server_scan), so a process that stops calling leaves no kernel running.  kSrvProbe:
// per-request phase stamps (PBS_SERVER_PROBE=1).
//
// Split requests (round 5): one workgroup hashes ~6 GB/s (1.3 us per 8 KiB pass), so a
// 256 KiB read cost 42 us of kernel time and the unchanged caller reached 3.8 GB/s against
// 5.4 GB/s gathering 4 MiB per scan().  A request of >= 2 kSrvMinPasses passes is split
// over gu = min(n_wg, passes / kSrvMinPasses) workgroups (one pass each since round 6):
// every workgroup polls the host's request record and computes the split from its length
// (round 5: the leader re-published each request for the others, one more detection hop),
// hashes a contiguous range of passes (rows 0 and 1 from the 64 slot bytes before its first
// pass, the slot's history for pass 0), writes its candidates into its own region of the
// array and acknowledges that region on its own line after a system-scope release (round 5
// reserved slots with device atomics and counted the workgroups done, the last one
// acknowledging); the host waits for the gu acknowledgements and reads the regions in order,
// which is stream order.  One-pass requests stay with the leader alone; the leader's exit
// (quit or idle) is published in the ServerDispatch record, tagged with the launch's epoch.
// 256 KiB reads 3.85 -> 6.97 GB/s, 1 MiB 3.18 -> 5.50, 64 KiB 3.39 -> 4.42, 8 KiB
// 1.48 -> 1.49 (profiles/r05/scan_server); round 6: profiles/r06/server/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbs_chunker_internal.h"

namespace pbs {

constexpr int kSrvThreads = 256;  // 4 waves, one per SIMD
constexpr int kSrvLaneBytes = 32;
constexpr int kSrvPass = kSrvLaneBytes * kSrvThreads;  // bytes per pass (8 KiB)
constexpr int kSrvRows = kSrvThreads + 2;              // chain rows: the two before the pass, then one per lane
constexpr int kSrvAhead = 4;                           // passes whose bytes are in flight
constexpr uint32_t kSrvEpochMask = 0x3FFFFFFFu;         // ServerDispatch tag bits 32..61: the launch's epoch

typedef uint32_t srv_u32x4 __attribute__((ext_vector_type(4)));

// chain row r (32 dwords), dwords [4k, 4k+4) at a swizzled 16-byte slot (ds_*_b128 of
// lanes 128 bytes apart would hit the same banks)
__device__ __forceinline__ uint32_t srv_row_off(uint32_t r, uint32_t k) {
    return r * 128u + ((k ^ (r & 7u)) << 4);
}
__device__ __forceinline__ uint32_t srv_row_dw(uint32_t r, uint32_t i) {  // dword i of row r
    return srv_row_off(r, i >> 2) + 4u * (i & 3u);
}

__global__ __launch_bounds__(kSrvThreads) void scan_server_kernel(ServerMailbox* mb,
                                                                  const ServerReq* req,
                                                                  ServerDispatch* disp,
                                                                  const uint8_t* __restrict__ slot_main,
                                                                  const uint8_t* __restrict__ slot_host,
                                                                  const uint32_t* __restrict__ table_rot,
                                                                  uint32_t thr, uint64_t last_seq,
                                                                  uint64_t idle_ticks, uint32_t flags,
                                                                  uint32_t n_wg, uint32_t epoch) {
    // T'[b] replicated 64x at byte b * 256 + lane * 4: one v_perm forms the address
    __shared__ __attribute__((aligned(16))) uint32_t tab[256 * 64];
    __shared__ __attribute__((aligned(16))) uint8_t rows[kSrvRows * 128];
    __shared__ uint32_t wsum[kSrvThreads / 64];
    __shared__ uint32_t s_go;    // 0 polling, 1 serve, 2 exit
    __shared__ uint64_t ctl[2];  // [0] seq | len << 32 [1] base
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t g = blockIdx.x;
    const bool leader = g == 0;
    const bool poll_all = (flags & kSrvPollAll) != 0, probe = (flags & kSrvProbe) != 0;
    for (int i = tid; i < 256 * 64; i += kSrvThreads) tab[i] = table_rot[i >> 6];
    if (tid == 0) s_go = 0;
    __syncthreads();
    const uint32_t lane4 = (uint32_t)lane * 4u;
    auto lookup = [&](uint32_t word, int k) -> uint32_t {  // T'[byte k of word] (this lane's replica)
        const uint32_t addr = __builtin_amdgcn_perm(word, lane4, 0x0C0C0000u | ((uint32_t)(4 + k) << 8));
        return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(tab) + addr);
    };
    auto rd = [&](uint32_t off) -> uint32_t { return *reinterpret_cast<const uint32_t*>(rows + off); };
    uint32_t last = (uint32_t)last_seq;
    uint64_t t_idle = wall_clock64();
    for (;;) {
        if (leader) {
            // poll the request record (one 16-byte load {seq, len, base}); with kSrvPollAll
            // lane 0 of every wave polls, the waves staggered
            if (lane == 0 && (poll_all || wave == 0)) {
                if (poll_all)
                    for (int d = 0; d < wave; ++d) __builtin_amdgcn_s_sleep(8);
                for (;;) {
                    if (__hip_atomic_load(&s_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                    const srv_u32x4 r = *reinterpret_cast<const volatile srv_u32x4*>(&req->req_seq);
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
        } else if (tid == 0) {
            // a follower polls the host's request record itself (one 16-byte load, consistent
            // by construction: the host stores len and base before seq) and, for the exit, the
            // leader's dispatch record.  (Until round 6 the leader re-published each request
            // there for the followers: one more detection hop, ~1 us per split request, and
            // the reason the record needed a seqlock.)
            for (;;) {
                const srv_u32x4 r = *reinterpret_cast<const volatile srv_u32x4*>(&req->req_seq);
                if (r.y & kServerQuit) {
                    s_go = 2;
                    break;
                }
                if (r.x != last) {
                    ctl[0] = (uint64_t)r.x | ((uint64_t)r.y << 32);
                    ctl[1] = (uint64_t)r.z | ((uint64_t)r.w << 32);
                    s_go = 1;
                    break;
                }
                const uint64_t t = __hip_atomic_load(&disp->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (((uint32_t)(t >> 32) & kSrvEpochMask) == epoch && (t >> 63)) {
                    s_go = 2;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        // the slot is read after the record; a slot in VRAM written over the BAR is reused by
        // every request, so no stale line of it may survive in the caches (system scope)
        if (flags & kSrvDevReq)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        else
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (s_go != 1) {
            if (leader && tid == 0) {
                if (n_wg > 1)  // the followers exit on this record
                    __hip_atomic_store(&disp->tag, (uint64_t)last | (uint64_t)epoch << 32 | 1ull << 63,
                                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&mb->exited, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;  // uniform
        }
        const uint64_t t_seen = probe ? wall_clock64() : 0;
        uint64_t t_loaded = 0, t_hashed = 0;
        const uint32_t seq = (uint32_t)ctl[0], len = (uint32_t)(ctl[0] >> 32) & ~kServerHostSlot;
        const uint32_t npass = (len + kSrvPass - 1) / kSrvPass;
        // the request's split over gu workgroups: every workgroup computes it from the length
        // (the host does too, to know whose acknowledgements to wait for)
        const uint32_t minp = (flags >> kSrvMinPassShift) & 0xFFu;  // 0: kSrvMinPasses
        const uint32_t want = npass / (minp ? minp : kSrvMinPasses);
        const uint32_t gu = want < 1 ? 1 : (want < n_wg ? want : n_wg);
        const bool split = gu > 1;
        // this workgroup's passes [p_lo, p_hi) (a follower beyond gu has none)
        const uint32_t p_lo = g < gu ? (uint32_t)((uint64_t)g * npass / gu) : npass;
        const uint32_t p_hi = g < gu ? (uint32_t)((uint64_t)(g + 1) * npass / gu) : npass;
        // long requests of a VRAM-mode server come in the pinned host slot (kServerHostSlot)
        const uint8_t* const slot = (ctl[0] >> 32) & kServerHostSlot ? slot_host : slot_main;
        const uint64_t base = ctl[1];
        const srv_u32x4* const src = reinterpret_cast<const srv_u32x4*>(slot + kServerHist);
        // this lane's 32 bytes of pass p (lanes wholly past the data load nothing)
        auto load = [&](uint32_t p, srv_u32x4 (&x)[2]) {
            const uint32_t b = p * (uint32_t)kSrvPass + (uint32_t)tid * kSrvLaneBytes;
            if (p < p_hi && b < len) {
                x[0] = __builtin_nontemporal_load(src + b / 16);
                x[1] = __builtin_nontemporal_load(src + b / 16 + 1);
            }
        };
        uint32_t total = 0;
        bool stored = false;  // some pass stored candidates (block-uniform)
        // a split request's workgroup writes its own region of the candidate array
        const uint32_t rcap = split ? kServerCand / gu : kServerCand;
        const uint32_t rbase = split ? (g < gu ? g : 0u) * rcap : 0u;
        if (p_lo < p_hi) {
            srv_u32x4 ring[kSrvAhead][2];
#pragma unroll
            for (int k = 0; k < kSrvAhead; ++k) {
                ring[k][0] = ring[k][1] = srv_u32x4{0u, 0u, 0u, 0u};
                load(p_lo + (uint32_t)k, ring[k]);
            }
            // rows 0 and 1: the chains of the 64 bytes before the first pass (the slot's
            // history for pass 0; one byte per lane of wave 0; a rotating prefix over each
            // 32-lane half: x = rotl(x_{l-d}, d) ^ x_l)
            if (wave == 0) {
                uint32_t x = lookup((uint32_t)slot[p_lo * (uint32_t)kSrvPass + (uint32_t)lane], 0);
#pragma unroll
                for (int d = 1; d < 32; d <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)x, d, 32);
                    if ((lane & 31) >= d) x ^= __builtin_amdgcn_alignbit(y, y, 32 - d);
                }
                *reinterpret_cast<uint32_t*>(rows + srv_row_dw((uint32_t)lane >> 5, (uint32_t)lane & 31u)) = x;
            }
            auto pass = [&](uint32_t p, srv_u32x4 (&cur)[2]) {
                const uint32_t off = p * (uint32_t)kSrvPass;
                const uint32_t plen = len - off < (uint32_t)kSrvPass ? len - off : (uint32_t)kSrvPass;
                // stream positions < 63 have no full window (chunker.rs:118-136): never reported
                const uint64_t pos0 = base + off;
                const uint32_t lo_ok = pos0 >= 63 ? 0u : (uint32_t)(63 - pos0);
                const uint32_t d[8] = {cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y, cur[1].z, cur[1].w};
                uint32_t q[32];
                uint32_t h = 0;
#pragma unroll
                for (int i = 0; i < 32; ++i) {
                    h = __builtin_amdgcn_alignbit(h, h, 31) ^ lookup(d[i >> 2], i & 3);
                    q[i] = h;
                }
                load(p + kSrvAhead, cur);  // the slot's registers are free again
                if (probe && p == p_lo) t_loaded = wall_clock64();
                // this lane's chain is row tid + 2 (the previous pass's readers are done: the
                // barrier before the row copy below)
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    *reinterpret_cast<srv_u32x4*>(rows + srv_row_off((uint32_t)tid + 2u, (uint32_t)k)) =
                        srv_u32x4{q[4 * k], q[4 * k + 1], q[4 * k + 2], q[4 * k + 3]};
                __syncthreads();
                uint32_t p2[32];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const srv_u32x4 v = *reinterpret_cast<const srv_u32x4*>(rows + srv_row_off((uint32_t)tid, (uint32_t)k));
                    p2[4 * k] = v.x;
                    p2[4 * k + 1] = v.y;
                    p2[4 * k + 2] = v.z;
                    p2[4 * k + 3] = v.w;
                }
                const uint32_t X = p2[31] ^ rd(srv_row_dw((uint32_t)tid + 1u, 31u));
                uint32_t hp[32];
                uint32_t mx = 0;
#pragma unroll
                for (int i = 0; i < 32; ++i) {
                    hp[i] = q[i] ^ p2[i] ^ __builtin_amdgcn_alignbit(X, X, 31 - i);
                    mx = mx > hp[i] ? mx : hp[i];
                }
                // bit i = position off + 32 tid + i passes, within [lo_ok, plen)
                uint32_t bits = 0;
                if (mx >= thr) {
                    const int p0 = tid * kSrvLaneBytes;
#pragma unroll
                    for (int i = 0; i < 32; ++i) bits |= (hp[i] >= thr ? 1u : 0u) << i;
                    const int lo = (int)lo_ok - p0, up = (int)plen - p0;
                    const uint32_t keep_lo = lo <= 0 ? 0xFFFFFFFFu : (lo >= 32 ? 0u : (0xFFFFFFFFu << lo));
                    const uint32_t keep_hi = up >= 32 ? 0xFFFFFFFFu : (up <= 0 ? 0u : (0xFFFFFFFFu >> (32 - up)));
                    bits &= keep_lo & keep_hi;
                }
                if (probe && p == p_lo) t_hashed = wall_clock64();
                // stream-order compaction (hits are rare: one barrier tells whether any); a
                // split request reserves the pass's slots with one device atomic (the host
                // sorts the workgroups' runs)
                const uint32_t c = __builtin_popcount(bits);
                if (__syncthreads_or(c != 0)) {
                    stored = true;
                    uint32_t x = c;
#pragma unroll
                    for (int dd = 1; dd < 64; dd <<= 1) {
                        const uint32_t z = __shfl_up(x, dd, 64);
                        if (lane >= dd) x += z;
                    }
                    if (lane == 63) wsum[wave] = x;
                    __syncthreads();
                    uint32_t before = 0, all = 0;
#pragma unroll
                    for (int w2 = 0; w2 < kSrvThreads / 64; ++w2) {
                        before += w2 < wave ? wsum[w2] : 0u;
                        all += wsum[w2];
                    }
                    uint32_t o = total + before + x - c;
                    uint32_t m = bits;
                    while (m) {
                        const int bit = __builtin_ctz(m);
                        m &= m - 1;
                        if (o < rcap) mb->cand[rbase + o] = pos0 + (uint64_t)(tid * kSrvLaneBytes + bit);
                        ++o;
                    }
                    total += all;
                    __syncthreads();  // wsum reused
                }
                // the next pass's rows 0 and 1 = this pass's last two rows (every reader of them
                // is past the barrier above)
                if (p + 1 < p_hi) {
                    if (tid < 64) {
                        const uint32_t r = (uint32_t)tid >> 5, i = (uint32_t)tid & 31u;
                        *reinterpret_cast<uint32_t*>(rows + srv_row_dw(r, i)) = rd(srv_row_dw(kSrvThreads + r, i));
                    }
                    __syncthreads();
                }
            };
            for (uint32_t p0 = p_lo; p0 < p_hi; p0 += kSrvAhead) {
#pragma unroll
                for (int k = 0; k < kSrvAhead; ++k)
                    if (p0 + k < p_hi) pass(p0 + k, ring[k]);
            }
        }
        // every wave's stores drained, then the acknowledgement (system scope); without
        // candidates every wave is past the last pass's barrier already
        if (stored || split) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (tid == 0) {
            if (probe && leader) {
                mb->probe[0] = t_seen;
                mb->probe[1] = t_loaded;
                mb->probe[2] = t_hashed;
            }
            s_go = 0;
            if (split && g < gu) {
                // this workgroup's acknowledgement of its region, on its own line (release: its
                // candidates -- and the leader's probe stamps -- before it); the host waits for
                // all gu of them.  (Round 5 counted the workgroups done with a device atomic and
                // the last one acknowledged: a serial atomic and a second release per request.)
                if (probe && leader) mb->probe[3] = wall_clock64();
                const uint64_t ack = (uint64_t)seq | (uint64_t)(total < rcap ? total : rcap) << 32 |
                                     (total > rcap ? 1ull << 63 : 0ull);
                __hip_atomic_store(&mb->wg_ack[8 * g], ack, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (!split && leader) {  // (the followers see every request now, the unsplit ones too)
                if (probe) mb->probe[3] = wall_clock64();
                // ONE 8-byte store: seq, candidate count, overflow flag (the host reads them
                // together); a release (an L2 write-back first) only when candidates -- or the
                // probe stamps -- were stored before it
                const uint64_t ack = (uint64_t)seq | (uint64_t)(total < kServerCand ? total : kServerCand) << 32 |
                                     (total > kServerCand ? 1ull << 63 : 0ull);
                if (stored || probe)
                    __hip_atomic_store(&mb->ack_seq, ack, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                else
                    __hip_atomic_store(&mb->ack_seq, ack, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
        last = seq;
        t_idle = wall_clock64();
    }
}

}  // namespace pbs
