// Per-chunk SHA-256 on the GPU: the digest every chunk gets
// right after the chunker, `DataChunkBuilder::digest` (pbs-datastore/src/data_blob.rs:
// 516-536) = SHA-256(chunk), or SHA-256(chunk || id_key) with a crypt config
// (pbs-tools/src/crypt_config.rs:79-84).  C ABI: include/pbs_digest.h.
//
// SHA-256 is a serial chain of 64-byte compressions per message, so the parallelism is
// the chunks: ONE LANE PER CHUNK.  A lane streams its chunk 64 bytes at a time from
// HBM (the dword-aligned 68-byte window, loaded one block ahead of its use), builds the
// big-endian message words with one v_perm_b32 each (byte alignment and byte swap in
// one op, selector from the chunk's start & 3), and runs the 64 rounds in registers
// (v_alignbit rotations, v_bitop3 for Ch/Maj/3-way XOR, v_add3).  The product kernel
// (sha256_chunks_split_kernel) gives the schedule and the rounds of each block to two
// waves of one workgroup; the single-wave form (sha256_chunks_kernel, 1422
// instructions per block) is kept for A/B runs.  Either way the kernel is
// VALU-issue-bound along one chunk's chain, not HBM-bound: a workgroup takes as long as
// its longest chunk, and the host orders the chunks by length (longest first) so the
// 64 lanes finish together.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "dev_arena.h"
#include <numeric>
#include <thread>
#include <vector>

#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"
#include "pbs_digest.h"
#include "sha_host.h"

namespace pbs {
namespace {

__constant__ uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// 3-input XOR in one v_bitop3_b32 (gfx950 has no v_xor3_b32)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One SHA-256 compression (FIPS 180-4 6.2.2) of the 16 big-endian words w into st.
__device__ __forceinline__ void compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const uint32_t x = w[(t - 15) & 15], y = w[(t - 2) & 15];
            const uint32_t s0 = xor3(rotr(x, 7), rotr(x, 18), x >> 3);
            const uint32_t s1 = xor3(rotr(y, 17), rotr(y, 19), y >> 10);
            wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
            w[t & 15] = wt;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // e ? f : g
        const uint32_t t1 = h + S1 + ch + kK[t] + wt;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t maj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + S0 + maj;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
}

// 68 readable bytes in global memory: the window a producer lane loads when it has no
// block two ahead (a select between two global pointers keeps the loads global; a
// constant-memory dummy made them flat loads, which also count on the LDS counter)
__device__ uint32_t g_dummy_window[17];

struct DigestKey {
    uint32_t len;
    uint8_t bytes[PBS_DIGEST_MAX_KEY];
};

__device__ __forceinline__ void load_window(const uint32_t* __restrict__ pa, bool tail_dw,
                                            uint32_t (&d)[17]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = __builtin_nontemporal_load(pa + q);
    d[16] = tail_dw ? __builtin_nontemporal_load(pa + 16) : 0u;
}

// Branch-free form: dword 16 is read from pa + 16 when the chunk start is misaligned
// (it then holds a byte of the block) and from pa + 15 otherwise (inside the window;
// the perms of an aligned block never select it).
__device__ __forceinline__ void load_window_nb(const uint32_t* __restrict__ pa, uint32_t dw16,
                                               uint32_t (&d)[17]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = __builtin_nontemporal_load(pa + q);
    d[16] = __builtin_nontemporal_load(pa + dw16);
}

// Lane k hashes chunk order[k] (identity if order == nullptr): [bounds[i], bounds[i+1])
// relative to `data` after subtracting `base`.
__global__ __launch_bounds__(64) void sha256_chunks_kernel(const uint8_t* __restrict__ data,
                                                           uint64_t base,
                                                           const uint64_t* __restrict__ bounds,
                                                           const uint32_t* __restrict__ order,
                                                           uint64_t n, DigestKey key,
                                                           uint8_t* __restrict__ digests) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t i = order ? order[k] : k;
    const uint64_t s = bounds[i] - base, e = bounds[i + 1] - base, len = e - s;
    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    const uint8_t* p = data + s;
    const uint32_t r = (uint32_t)((uintptr_t)p & 3u);
    // the dword-aligned window of block b is pa[16b .. 16b+16]; its last dword is needed
    // only when r != 0 and always holds a byte of the block, so it never leaves the
    // page of a valid byte
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(p - r);
    const uint32_t sel = (r << 24) | ((r + 1) << 16) | ((r + 2) << 8) | (r + 3);
    const uint64_t nfull = len >> 6;
    uint32_t cur[17], nxt[17];
    if (nfull) load_window(pa, r != 0, cur);
    for (uint64_t b = 0; b < nfull; ++b) {
        if (b + 1 < nfull) load_window(pa + 16 * (b + 1), r != 0, nxt);
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) w[q] = __builtin_amdgcn_perm(cur[q + 1], cur[q], sel);
        compress(st, w);
#pragma unroll
        for (int q = 0; q < 17; ++q) cur[q] = nxt[q];
    }
    // tail: remaining bytes, key, 0x80, zeros, 64-bit big-endian bit length
    const uint32_t rem = (uint32_t)(len & 63);
    const uint32_t kl = key.len;
    const uint64_t bits = (len + kl) * 8ull;
    const uint32_t nb = (rem + kl + 1 + 8 + 63) / 64;  // 1..3 blocks
    const uint8_t* tp = p + (nfull << 6);
    for (uint32_t blk = 0; blk < nb; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t t = blk * 64 + 4 * q + j;
                uint32_t byte;
                if (t < rem)
                    byte = tp[t];
                else if (t < rem + kl)
                    byte = key.bytes[t - rem];
                else if (t == rem + kl)
                    byte = 0x80u;
                else if (t >= nb * 64 - 8)
                    byte = (uint32_t)(bits >> (8 * (nb * 64 - 1 - t))) & 0xffu;
                else
                    byte = 0;
                v = (v << 8) | byte;
            }
            w[q] = v;
        }
        compress(st, w);
    }
    uint32_t* out = reinterpret_cast<uint32_t*>(digests + 32 * i);
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = __builtin_bswap32(st[q]);
}


// Two-wave form: the message schedule (48 sigma steps + K[t] per block, the data loads,
// the tail/padding blocks) runs in wave 1 one block ahead of the 64 rounds in wave 0,
// handed over through a double-buffered LDS array W[2][16][64 lanes] of 4-word groups
// (one ds_write_b128 / ds_read_b128 per 4 rounds, lane-minor: conflict-free); one
// s_barrier per block.  The producer loads block b + 1's data while it schedules
// block b, so no HBM latency sits on the per-block critical path.  The rounds' wave is the critical path:
// ~960 instructions per block instead of ~1420 for one wave doing both.
constexpr int kShaWaves = 2;
#ifdef PBS_SHA_PROBE
__device__ uint64_t g_sha_probe[5];
#endif
// The two waves of one workgroup hash 64 chunks, lane l's chunk [s, e) of `data` (live
// lanes only) into dig (32 bytes; wave 0 writes).  sw / s_blocks: the workgroup's LDS.
__device__ __forceinline__ void sha_batch(const uint8_t* __restrict__ data, uint64_t s, uint64_t e, bool live,
                                          const DigestKey& key, uint8_t* __restrict__ dig, uint4 (&sw)[3][16][64],
                                          uint32_t& s_blocks) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t len = e - s;
    const uint64_t nfull = len >> 6;
    const uint32_t rem = (uint32_t)(len & 63);
    const uint32_t kl = key.len;
    const uint32_t nb = (rem + kl + 1 + 8 + 63) / 64;  // tail blocks
    const uint64_t total = live ? nfull + nb : 0;      // blocks of this lane
    // the wave pair runs to the longest lane's block count
    if (threadIdx.x == 0) s_blocks = 0;
    __syncthreads();
    if (wave == 0) atomicMax(&s_blocks, (uint32_t)total);
    __syncthreads();
    const uint32_t nblocks = s_blocks;

    const uint8_t* p = data + s;
    const uint32_t r = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(p - r);
    const uint32_t sel = (r << 24) | ((r + 1) << 16) | ((r + 2) << 8) | (r + 3);
    const uint64_t bits = (len + kl) * 8ull;
    const uint8_t* tp = p + (nfull << 6);

    // wave 1: message block b -> W + K into slot b % 3.  Its 68-byte data window sits in
    // register window R[b % 3], loaded two blocks earlier: produce(b) issues the loads of
    // block b + 2 into the window block b - 1 has freed, so HBM latency hides behind two
    // block periods.  (A single `pre` window copied out before its reload made the
    // compiler wait for the new loads right after issuing them: the phi copy at the loop
    // latch needs their data.)
    uint32_t R0[17], R1[17], R2[17];
    const uint32_t dw16 = r ? 16u : 15u;
    if (wave == 1) {
        if (nfull) load_window_nb(pa, dw16, R0);
        if (nfull > 1) load_window_nb(pa + 16, dw16, R1);
    }
    auto produce = [&](uint32_t b, uint32_t slot, uint32_t (&cur)[17], uint32_t (&nx2)[17]) {
        // straight-line perms then loads (no branch between them, so nothing can sink the
        // perms below the loads and make their wait cover the new loads); a lane without a
        // window two blocks ahead loads the 68-byte dummy instead
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) w[q] = __builtin_amdgcn_perm(cur[q + 1], cur[q], sel);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t* src = (uint64_t)b + 2 < nfull ? pa + 16 * ((uint64_t)b + 2) : g_dummy_window;
        load_window_nb(src, dw16, nx2);
        if ((uint64_t)b >= nfull) {
            if ((uint64_t)b < total) {
                const uint32_t blk = (uint32_t)(b - nfull);
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t t = blk * 64 + 4 * q + j;
                        uint32_t byte;
                        if (t < rem)
                            byte = tp[t];
                        else if (t < rem + kl)
                            byte = key.bytes[t - rem];
                        else if (t == rem + kl)
                            byte = 0x80u;
                        else if (t >= nb * 64 - 8)
                            byte = (uint32_t)(bits >> (8 * (nb * 64 - 1 - t))) & 0xffu;
                        else
                            byte = 0;
                        v = (v << 8) | byte;
                    }
                    w[q] = v;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) w[q] = 0;
            }
        }
        uint4 (*out)[64] = sw[slot];
        uint32_t o[4];
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {
                const uint32_t x = w[(t - 15) & 15], y = w[(t - 2) & 15];
                const uint32_t s0 = xor3(rotr(x, 7), rotr(x, 18), x >> 3);
                const uint32_t s1 = xor3(rotr(y, 17), rotr(y, 19), y >> 10);
                wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
                w[t & 15] = wt;
            }
            o[t & 3] = wt + kK[t];
            if ((t & 3) == 3) out[t >> 2][lane] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    };

    uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    // Three slots, the producer two blocks ahead (its data loads two blocks ahead too).
    // The loop is unrolled by three so that slot and register window are constants in
    // each step: rotating them through one loop body put register copies between the
    // loads and their use, and the compiler then waited for the loads at once.
    if (wave == 1) {
        if (nblocks) produce(0, 0, R0, R2);
        if (nblocks > 1) produce(1, 1, R1, R0);
    }
    __syncthreads();
#ifdef PBS_SHA_PROBE  // scripts/microbench/mb_sha.hip: cycles of each wave's work vs the barrier
    uint64_t pr_work = 0, pr_wait = 0;
#endif
    // block b: the rounds wave hashes slot b % 3, the producer fills slot (b + 2) % 3
    // The rounds wave holds W + K in kwv[16]: groups 12..15 of block b are read at the top
    // of block b (needed from round 48), and group q < 12 of block b + 1 (complete since
    // the last barrier) right after round 4q + 3 consumed group q of block b, so no LDS
    // read latency lands on the chain and the barrier finds no read in flight.
    uint4 kwv[16];
    if (wave == 0) {
#pragma unroll
        for (int q = 0; q < 12; ++q) kwv[q] = sw[0][q][lane];
    }
    auto step = [&](uint32_t b, const uint4 (*in)[64], const uint4 (*nx)[64], uint32_t pslot,
                    uint32_t (&cur)[17], uint32_t (&nx2)[17]) {
#ifdef PBS_SHA_PROBE
        const uint64_t c0 = clock64();
#endif
        if (wave == 1) {
            if (b + 2 < nblocks) produce(b + 2, pslot, cur, nx2);
        } else if ((uint64_t)b < total) {
            uint32_t a = st[0], bb = st[1], c = st[2], d = st[3], ee = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
            for (int q = 12; q < 16; ++q) kwv[q] = in[q][lane];
#pragma unroll
            for (int t = 0; t < 64; ++t) {
                const uint4 kw4 = kwv[t >> 2];
                const uint32_t kw = (t & 3) == 0 ? kw4.x : (t & 3) == 1 ? kw4.y : (t & 3) == 2 ? kw4.z : kw4.w;
                if ((t & 3) == 3 && t < 48) {
                    kwv[t >> 2] = nx[t >> 2][lane];
                    __builtin_amdgcn_sched_barrier(0);  // keep the read here (hoisted, it needs copies)
                }
                const uint32_t S1 = xor3(rotr(ee, 6), rotr(ee, 11), rotr(ee, 25));
                const uint32_t ch = __builtin_amdgcn_bitop3_b32(ee, f, g, 0xCA);
                const uint32_t t1 = h + S1 + ch + kw;
                const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
                const uint32_t maj = __builtin_amdgcn_bitop3_b32(a, bb, c, 0xE8);
                h = g;
                g = f;
                f = ee;
                ee = d + t1;
                d = c;
                c = bb;
                bb = a;
                a = t1 + S0 + maj;
            }
            st[0] += a;
            st[1] += bb;
            st[2] += c;
            st[3] += d;
            st[4] += ee;
            st[5] += f;
            st[6] += g;
            st[7] += h;
        }
#ifdef PBS_SHA_PROBE
        const uint64_t c1 = clock64();
        __syncthreads();
        pr_work += c1 - c0;
        pr_wait += clock64() - c1;
#else
        __syncthreads();
#endif
    };
    for (uint32_t b = 0; b < nblocks; b += 3) {
        step(b, sw[0], sw[1], 2, R2, R1);
        if (b + 1 < nblocks) step(b + 1, sw[1], sw[2], 0, R0, R2);
        if (b + 2 < nblocks) step(b + 2, sw[2], sw[0], 1, R1, R0);
    }
#ifdef PBS_SHA_PROBE
    if (blockIdx.x == 0 && lane == 0) {
        g_sha_probe[wave * 2] = pr_work;
        g_sha_probe[wave * 2 + 1] = pr_wait;
        g_sha_probe[4] = nblocks;
    }
#endif
    if (wave == 0 && live) {
        uint32_t* out = reinterpret_cast<uint32_t*>(dig);
#pragma unroll
        for (int q = 0; q < 8; ++q) out[q] = __builtin_bswap32(st[q]);
    }
}

__global__ __launch_bounds__(64 * kShaWaves) void sha256_chunks_split_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint32_t* __restrict__ order, uint64_t n, DigestKey key, uint8_t* __restrict__ digests) {
    __shared__ uint4 sw[3][16][64];  // [slot][t / 4][lane]: W[t] + K[t] for 4 t (b128 per lane)
    __shared__ uint32_t s_blocks;
    const int lane = threadIdx.x & 63;
    const uint64_t k = (uint64_t)blockIdx.x * 64 + lane;
    const bool live = k < n;
    const uint64_t i = live ? (order ? order[k] : k) : 0;
    const uint64_t s = live ? bounds[i] - base : 0, e = live ? bounds[i + 1] - base : 0;
    sha_batch(data, s, e, live, key, digests + 32 * i, sw, s_blocks);
}

// ---------------------------------------------------------------------------------
// Digest queue (the host-stream pipeline, pbs_pipeline.cpp): a persistent grid of the
// two-wave workgroups above takes chunk jobs as the host publishes them, so a chunk's
// serial SHA-256 chain starts as soon as its end is known instead of at the next
// launch.  The host appends jobs {start, len, out index} to a pinned (coherent, mapped)
// array and then stores the count (bit 63: no more jobs) into the pinned control word.
// An idle workgroup claims up to 64 published jobs with one CAS on the device counter
// `next`; the control word is read over PCIe by at most one workgroup every ~2 us
// (`last_poll`) and mirrored in device memory, where the others see it.  A workgroup
// exits when every job is claimed and the final bit is set, or after idle_ticks (wall
// clock, 100 MHz) in which no new job was PUBLISHED (the count it sees moved: claimed by
// another workgroup or not, the stream is alive; round 5's first 50 ms idle exit counted
// only this workgroup's own claims, so most of the grid left while the host was still
// publishing and the 64 GiB pipeline's digests took 4 s instead of 1.25) -- the host
// relaunches the grid when it publishes jobs after that.  Exiting when idle matters: a resident grid holds up whatever waits
// for the whole device or for its stream (hipFree, null-stream copies).
__global__ __launch_bounds__(64 * kShaWaves) void sha256_queue_kernel(
    const uint8_t* __restrict__ data, DigestKey key, volatile DigestJob* __restrict__ jobs,
    const volatile uint64_t* __restrict__ ctl_host, DigestQueueDev* __restrict__ q, uint8_t* __restrict__ digests,
    uint64_t idle_ticks) {
    __shared__ uint4 sw[3][16][64];
    __shared__ uint32_t s_blocks;
    __shared__ uint64_t s_j0, s_k;
    const int lane = threadIdx.x & 63;
    uint64_t t_job = wall_clock64(), seen_avail = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint64_t j0 = 0, k = 0;
            for (;;) {
                const uint64_t m = __hip_atomic_load(&q->mirror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t avail = m & 0xFFFFFFFFull, nx = __hip_atomic_load(&q->next, __ATOMIC_RELAXED,
                                                                                 __HIP_MEMORY_SCOPE_AGENT);
                if (avail != seen_avail) {  // new jobs were published: not idle
                    seen_avail = avail;
                    t_job = wall_clock64();
                }
                if (avail > nx) {
                    const uint64_t want = avail - nx < 64 ? avail - nx : 64;
                    unsigned long long exp = nx;
                    if (__hip_atomic_compare_exchange_strong(&q->next, &exp, nx + want, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        j0 = nx;
                        k = want;
                        break;
                    }
                    continue;
                }
                if (m >> 63) break;  // every job claimed, no more coming
                const uint64_t now = wall_clock64();
                if (now - t_job > idle_ticks) break;  // nothing new for a while: exit (relaunched on demand)
                unsigned long long lp = __hip_atomic_load(&q->last_poll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (now - lp > 200 && __hip_atomic_compare_exchange_strong(&q->last_poll, &lp, now, __ATOMIC_RELAXED,
                                                                           __ATOMIC_RELAXED,
                                                                           __HIP_MEMORY_SCOPE_AGENT)) {
                    const uint64_t h = __hip_atomic_load(ctl_host, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_fetch_max(&q->mirror, (unsigned long long)h, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_fetch_add(&q->polls, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long prev =
                        __hip_atomic_exchange(&q->last_h, (unsigned long long)h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (prev != h) {
                        const unsigned long long ix =
                            __hip_atomic_fetch_add(&q->nseen, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (ix < 16) {
                            q->seen[ix] = h;
                            q->seen_t[ix] = now;
                        }
                    }
                } else {
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            s_j0 = j0;
            s_k = k;
        }
        __syncthreads();
        const uint64_t j0 = s_j0, k = s_k;
        if (k == 0) return;  // uniform
        t_job = wall_clock64();
        const bool live = (uint64_t)lane < k;
        uint64_t st0 = 0, len = 0, idx = 0;
        if (live) {
            st0 = jobs[j0 + lane].start;
            len = jobs[j0 + lane].len;
            idx = jobs[j0 + lane].idx;
        }
        sha_batch(data, st0, st0 + len, live, key, digests + 32 * idx, sw, s_blocks);
        // every wave's digest stores out to memory, then the jobs say done (pinned host
        // memory: the upload path's encoder reads the digests as soon as it sees the flags)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x < 64 && live)
            __hip_atomic_store(const_cast<uint64_t*>(&jobs[j0 + lane].done), (uint64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        t_job = wall_clock64();  // idle from here: look for new jobs for idle_ticks
        __syncthreads();         // s_j0 / s_k and the LDS are reused
    }
}

// ---------------------------------------------------------------------------------
// Known-chunk test (backup_writer.rs:677-697), see pbs_digest.h.  The digests are
// radix-sorted by their first 8 bytes (big-endian, i.e. byte-string order) with the
// chunk index as value; the sort is stable, so each run of equal prefixes lists its
// chunks in stream order.  A chunk is a repeat iff an earlier chunk of its run has the
// same full digest: compared with the run's first element (the usual case: all equal),
// else (a 64-bit prefix shared by different digests) against every earlier run member.
// Membership in the previous index: binary search over the sorted known digests.
__device__ __forceinline__ int cmp32(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b) {
    const uint4* x = reinterpret_cast<const uint4*>(a);
    const uint4* y = reinterpret_cast<const uint4*>(b);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint4 u = x[q], v = y[q];
        const uint32_t uu[4] = {u.x, u.y, u.z, u.w}, vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (uu[w] != vv[w]) {
                const uint32_t bu = __builtin_bswap32(uu[w]), bv = __builtin_bswap32(vv[w]);
                return bu < bv ? -1 : 1;
            }
    }
    return 0;
}

__global__ void digest_prefix_kernel(const uint8_t* __restrict__ dig, uint64_t n,
                                     uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(dig + 32 * i);
    key[i] = ((uint64_t)__builtin_bswap32(d[0]) << 32) | __builtin_bswap32(d[1]);
    idx[i] = (uint32_t)i;
}

__global__ void run_head_kernel(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ head) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    head[p] = (p == 0 || key[p] != key[p - 1]) ? (uint32_t)p : 0u;
}

__global__ void known_kernel(const uint8_t* __restrict__ dig, uint64_t n,
                             const uint32_t* __restrict__ sidx, const uint32_t* __restrict__ rstart,
                             const uint8_t* __restrict__ known, uint64_t k,
                             uint8_t* __restrict__ is_known, unsigned int* __restrict__ count) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t i = sidx[p];
    const uint8_t* di = dig + 32ull * i;
    bool rep = false;
    const uint32_t r0 = rstart[p];
    if (r0 != p) {
        if (cmp32(dig + 32ull * sidx[r0], di) == 0) {
            rep = true;
        } else {
            for (uint32_t q = r0 + 1; q < p && !rep; ++q) rep = cmp32(dig + 32ull * sidx[q], di) == 0;
        }
    }
    bool in_known = false;
    if (!rep && k) {
        uint64_t lo = 0, hi = k;  // first known >= di
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (cmp32(known + 32 * mid, di) < 0)
                lo = mid + 1;
            else
                hi = mid;
        }
        in_known = lo < k && cmp32(known + 32 * lo, di) == 0;
    }
    const bool kn = rep || in_known;
    is_known[i] = kn ? 1 : 0;
    if (kn) atomicAdd(count, 1u);
}


// Zero test of the hybrid digest's long chunks: flags[k] = 1 iff chunk order[k] is all
// zero bytes.  One workgroup per chunk, 256 lanes x 16 bytes = 4 KiB rows; a group of 16
// rows ends with a workgroup OR, so a chunk with data stops after its first 64 KiB and
// only all-zero chunks are read whole.
__global__ __launch_bounds__(256) void zero_flags_kernel(const uint8_t* __restrict__ data, uint64_t base,
                                                         const uint64_t* __restrict__ bounds,
                                                         const uint32_t* __restrict__ order, uint64_t m,
                                                         uint8_t* __restrict__ flags) {
    const uint64_t k = blockIdx.x;
    if (k >= m) return;
    const uint64_t i = order[k];
    const uint8_t* p = data + (bounds[i] - base);
    const uint8_t* e = data + (bounds[i + 1] - base);
    const uint8_t* a0 = reinterpret_cast<const uint8_t*>(((uintptr_t)p + 15) & ~(uintptr_t)15);
    const uint8_t* a1 = reinterpret_cast<const uint8_t*>((uintptr_t)e & ~(uintptr_t)15);
    int nz = 0;
    if (a0 >= a1) {  // under 32 bytes: bytewise
        for (const uint8_t* q = p + threadIdx.x; q < e; q += 256) nz |= *q;
    } else {
        if (threadIdx.x < (unsigned)(a0 - p)) nz |= p[threadIdx.x];
        if (threadIdx.x < (unsigned)(e - a1)) nz |= a1[threadIdx.x];
        const uint4* w = reinterpret_cast<const uint4*>(a0);
        const uint64_t nw = (uint64_t)(a1 - a0) / 16;
        for (uint64_t r = 0; r < nw; r += 256 * 16) {
#pragma unroll 4
            for (int j = 0; j < 16; ++j) {
                const uint64_t x = r + (uint64_t)j * 256 + threadIdx.x;
                if (x < nw) {
                    const uint4 v = w[x];
                    nz |= (int)((v.x | v.y | v.z | v.w) != 0);
                }
            }
            if (__syncthreads_or(nz)) break;
        }
    }
    nz = __syncthreads_or(nz);
    if (threadIdx.x == 0) flags[k] = nz ? 0 : 1;
}

}  // namespace

hipError_t launch_sha256_queue(const uint8_t* data, const uint8_t* key, size_t key_len, const DigestJob* jobs_dev,
                               const uint64_t* ctl_dev, DigestQueueDev* q, uint8_t* digests, int grid,
                               uint64_t idle_ticks, hipStream_t st) {
    if (key_len > PBS_DIGEST_MAX_KEY || grid <= 0) return hipErrorInvalidValue;
    DigestKey k{};
    k.len = (uint32_t)key_len;
    if (key_len) std::memcpy(k.bytes, key, key_len);
    hipLaunchKernelGGL(sha256_queue_kernel, dim3((unsigned)grid), dim3(64 * kShaWaves), 0, st, data, k,
                       (volatile DigestJob*)const_cast<DigestJob*>(jobs_dev), (const volatile uint64_t*)ctl_dev, q, digests,
                       idle_ticks);
    return hipGetLastError();
}

}  // namespace pbs

using namespace pbs;

namespace {
// work areas of the synchronous digest / known-chunk entry points (dev_arena.h)
pbs::ArenaPool& digest_pool() {
    static pbs::ArenaPool* p = new pbs::ArenaPool;  // never destroyed (HIP may be torn down first)
    return *p;
}
pbs::ArenaPool& known_pool() {
    static pbs::ArenaPool* p = new pbs::ArenaPool;
    return *p;
}
}  // namespace

extern "C" int pbs_digest_chunks_async(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                       const uint64_t* bounds_dev, const uint32_t* order_dev,
                                       size_t n, const uint8_t* key, size_t key_len,
                                       uint8_t* digests_dev, void* hip_stream) {
    if (n == 0) return PBS_OK;
    if (!bounds_dev || !digests_dev || (data_len && !dev_data) || key_len > PBS_DIGEST_MAX_KEY ||
        (key_len && !key))
        return PBS_ERR_INVALID;
    DigestKey k{};
    k.len = (uint32_t)key_len;
    if (key_len) std::memcpy(k.bytes, key, key_len);
    (void)hipGetLastError();
    const unsigned grid = (unsigned)((n + 63) / 64);
    static const bool one_wave = [] {  // PBS_SHA_ONE_WAVE=1: the single-wave kernel (A/B runs)
        const char* e = std::getenv("PBS_SHA_ONE_WAVE");
        return e && e[0] == '1';
    }();
    if (one_wave)
        hipLaunchKernelGGL(sha256_chunks_kernel, dim3(grid), dim3(64), 0, (hipStream_t)hip_stream,
                           dev_data, base, bounds_dev, order_dev, (uint64_t)n, k, digests_dev);
    else
        hipLaunchKernelGGL(sha256_chunks_split_kernel, dim3(grid), dim3(64 * kShaWaves), 0,
                           (hipStream_t)hip_stream, dev_data, base, bounds_dev, order_dev,
                           (uint64_t)n, k, digests_dev);
    return hipGetLastError() == hipSuccess ? PBS_OK : PBS_ERR_HIP;
}

extern "C" int pbs_digest_chunks_device(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                        const uint64_t* bounds, size_t n, const uint8_t* key,
                                        size_t key_len, uint8_t* digests, void* hip_stream) {
    if (n == 0) return PBS_OK;
    if (!bounds || !digests) return PBS_ERR_INVALID;
    for (size_t i = 0; i < n; ++i)  // every chunk inside the device range, ascending
        if (bounds[i] > bounds[i + 1] || bounds[i] < base || bounds[i + 1] - base > data_len)
            return PBS_ERR_INVALID;
    // longest chunks first: the lanes of a wave then hold similar lengths
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return bounds[a + 1] - bounds[a] > bounds[b + 1] - bounds[b];
    });
    hipStream_t st = (hipStream_t)hip_stream;
    int sdev = 0;
    if (hipStreamGetDevice(st, &sdev) != hipSuccess) return PBS_ERR_NO_DEVICE;
    pbs::DeviceGuard dg(sdev);  // the work area belongs on the stream's device
    if (!dg.ok) return PBS_ERR_NO_DEVICE;
    pbs::ArenaLease ar(digest_pool(), sdev);
    uint64_t* d_bounds = ar->get<uint64_t>(0, (n + 1) * 8);
    uint32_t* d_order = ar->get<uint32_t>(1, n * 4);
    uint8_t* d_dig = ar->get<uint8_t>(2, n * 32);
    int rc = PBS_OK;
    if (!d_bounds || !d_order || !d_dig) {
        rc = PBS_ERR_NOMEM;
    } else if (hipMemcpyAsync(d_bounds, bounds, (n + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
               hipMemcpyAsync(d_order, order.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = PBS_ERR_HIP;
    } else {
        rc = pbs_digest_chunks_async(dev_data, data_len, base, d_bounds, d_order, n, key, key_len,
                                     d_dig, hip_stream);
        if (rc == PBS_OK &&
            (hipMemcpyAsync(digests, d_dig, n * 32, hipMemcpyDeviceToHost, st) != hipSuccess))
            rc = PBS_ERR_HIP;
    }
    if (hipStreamSynchronize(st) != hipSuccess && rc == PBS_OK) rc = PBS_ERR_HIP;  // (before the arena goes back)
    return rc;
}

extern "C" int pbs_known_chunks_device(const uint8_t* digests_dev, size_t n, const uint8_t* known_dev,
                                       size_t k, uint8_t* is_known_dev, size_t* n_known,
                                       void* hip_stream) {
    if (n_known) *n_known = 0;
    if (n == 0) return PBS_OK;
    if (!digests_dev || !is_known_dev || (k && !known_dev) || n > 0xFFFFFFF0u) return PBS_ERR_INVALID;
    hipStream_t st = (hipStream_t)hip_stream;
    int sdev = 0;
    if (hipStreamGetDevice(st, &sdev) != hipSuccess) return PBS_ERR_NO_DEVICE;
    pbs::DeviceGuard dg(sdev);
    if (!dg.ok) return PBS_ERR_NO_DEVICE;
    pbs::ArenaLease ar(known_pool(), sdev);
    uint64_t* key = ar->get<uint64_t>(0, n * 8);
    uint64_t* skey = ar->get<uint64_t>(1, n * 8);
    uint32_t* idx = ar->get<uint32_t>(2, n * 4);
    uint32_t* sidx = ar->get<uint32_t>(3, n * 4);
    uint32_t* head = ar->get<uint32_t>(4, n * 4);
    uint32_t* rstart = ar->get<uint32_t>(5, n * 4);
    unsigned int* cnt = ar->get<unsigned int>(6, 4);
    void* tmp = nullptr;
    int rc = PBS_OK;
    size_t tb_sort = 0, tb_scan = 0;
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (!key || !skey || !idx || !sidx || !head || !rstart || !cnt) {
        rc = PBS_ERR_NOMEM;
        goto done;
    }
    if (radix_sort(nullptr, &tb_sort, key, skey, idx, sidx, n, 0, 64, st) != hipSuccess ||
        inclusive_max_u32(nullptr, &tb_scan, head, rstart, n, st) != hipSuccess ||
        !(tmp = ar->get<void>(7, std::max(tb_sort, tb_scan)))) {
        rc = PBS_ERR_NOMEM;
        goto done;
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(digest_prefix_kernel, dim3(grid), dim3(256), 0, st, digests_dev, (uint64_t)n, key, idx);
    tb_sort = std::max(tb_sort, tb_scan);
    tb_scan = tb_sort;
    if (radix_sort(tmp, &tb_sort, key, skey, idx, sidx, n, 0, 64, st) != hipSuccess) {
        rc = PBS_ERR_HIP;
        goto done;
    }
    hipLaunchKernelGGL(run_head_kernel, dim3(grid), dim3(256), 0, st, skey, (uint64_t)n, head);
    if (inclusive_max_u32(tmp, &tb_scan, head, rstart, n, st) != hipSuccess ||
        hipMemsetAsync(cnt, 0, 4, st) != hipSuccess) {
        rc = PBS_ERR_HIP;
        goto done;
    }
    hipLaunchKernelGGL(known_kernel, dim3(grid), dim3(256), 0, st, digests_dev, (uint64_t)n, sidx, rstart,
                       known_dev, (uint64_t)k, is_known_dev, cnt);
    if (hipGetLastError() != hipSuccess) {
        rc = PBS_ERR_HIP;
        goto done;
    }
    {
        unsigned int h = 0;
        if (hipMemcpyAsync(&h, cnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            rc = PBS_ERR_HIP;
            goto done;
        }
        if (n_known) *n_known = h;
    }
done:
    if (rc != PBS_OK) (void)hipStreamSynchronize(st);  // (before the arena goes back)
    return rc;
}

// ---------------------------------------------------------------------------------------
// Hybrid digest: the longest chunks on host threads (SHA extensions, pbs_sha_host.cpp),
// the rest on the GPU, all-zero long chunks hashed once per distinct length.
namespace {

using HClock = std::chrono::steady_clock;
double hms(HClock::time_point a, HClock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
}

constexpr size_t kSlice = 4u << 20;         // D2H slice of a host-hashed chunk (chunks over the ring's slot)
constexpr uint64_t kZeroMin = 1u << 20;      // chunks tested for all-zero content
constexpr uint64_t kRingMax = 1ull << 30;    // pinned ring of whole-chunk slots, at most 1 GiB
// D2H rate of whole chunks copied back to back on two streams into pinned slots (the cost
// model's cap on the host share's rate when its bytes come from HBM): 16 GB of the 64 GiB
// VM image's longest chunks in 310-316 ms on two streams, 327-337 on one
// (profiles/r04/digest_ring/)
constexpr double kD2HRate = 50e9;

// Pinned host memory and copy streams for the host share, kept for the process (pinning
// on every call would cost more than it hides): a ring of whole-chunk slots filled by one
// copy stream, and per-thread double buffers for chunks longer than a slot.
struct HostStage {
    std::mutex mu;
    int dev = -1;
    uint8_t* ring = nullptr;
    size_t ring_bytes = 0;
    hipStream_t cst[2] = {nullptr, nullptr};  // the ring's copy streams
    std::vector<hipEvent_t> rev; // one per slot
    std::vector<uint8_t*> buf;  // 2 * kSlice each
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;  // 2 per thread
    // a ring of `slots` slots of `sb` bytes (on device dv, like the streams below)
    bool ring_grow(int dv, size_t slots, size_t sb) {
        if (dev != dv) {
            release();
            dev = dv;
        }
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) return false;
        if (cur != dv && hipSetDevice(dv) != hipSuccess) return false;
        bool ok = true;
        for (auto& c : cst)
            if (ok && !c) ok = hipStreamCreateWithFlags(&c, hipStreamNonBlocking) == hipSuccess;
        if (ok && ring_bytes < slots * sb) {
            if (ring) (void)hipHostFree(ring);
            ring = nullptr;
            ring_bytes = 0;
            ok = hipHostMalloc((void**)&ring, slots * sb, hipHostMallocDefault) == hipSuccess;
            if (ok) ring_bytes = slots * sb;
        }
        while (ok && rev.size() < slots) {
            hipEvent_t e = nullptr;
            ok = hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
            if (ok) rev.push_back(e);
        }
        if (cur != dv) (void)hipSetDevice(cur);
        return ok;
    }
    // streams and events are created on device dv (the caller's stream's device), not
    // on whatever device the calling thread has current
    bool grow(int dv, int t) {
        if (dev != dv) {
            release();
            dev = dv;
        }
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess) return false;
        if (cur != dv && hipSetDevice(dv) != hipSuccess) return false;
        bool ok = true;
        while (ok && (int)buf.size() < t) {
            uint8_t* b = nullptr;
            hipStream_t s = nullptr;
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (hipHostMalloc(&b, 2 * kSlice, hipHostMallocDefault) != hipSuccess) {
                ok = false;
                break;
            }
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&e0, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess) {
                (void)hipHostFree(b);
                ok = false;
                break;
            }
            buf.push_back(b);
            st.push_back(s);
            ev.push_back(e0);
            ev.push_back(e1);
        }
        if (cur != dv) (void)hipSetDevice(cur);
        return ok;
    }
    void release() {
        if (ring) (void)hipHostFree(ring);
        for (auto& c : cst) {
            if (c) (void)hipStreamDestroy(c);
            c = nullptr;
        }
        for (auto e : rev) (void)hipEventDestroy(e);
        ring = nullptr;
        ring_bytes = 0;
        rev.clear();
        for (auto b : buf) (void)hipHostFree(b);
        for (auto s : st) (void)hipStreamDestroy(s);
        for (auto e : ev) (void)hipEventDestroy(e);
        buf.clear();
        st.clear();
        ev.clear();
    }
};
// One stage per device (its streams and events belong to that device; calls on different
// devices neither share a lock nor re-create each other's ring), created on first use and
// never destroyed: HIP may be torn down first at exit.
constexpr int kMaxStageDevices = 64;
std::mutex g_stage_mu;
HostStage* g_stages[kMaxStageDevices] = {};
HostStage* host_stage(int dev) {
    if (dev < 0 || dev >= kMaxStageDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_stage_mu);
    if (!g_stages[dev]) g_stages[dev] = new HostStage;
    return g_stages[dev];
}

// SHA-256 of one device-resident chunk on this host thread: 4 MiB slices copied into the
// thread's pinned double buffer one slice ahead of the hashing.
bool hash_from_device(const uint8_t* src, uint64_t len, const uint8_t* key, size_t key_len, uint8_t* out,
                      uint8_t* buf, hipStream_t st, hipEvent_t* ev) {
    pbs::HostSha h;
    pbs::sha256_host_init(h);
    const uint64_t ns = len ? (len + kSlice - 1) / kSlice : 0;
    if (ns && (hipMemcpyAsync(buf, src, std::min<uint64_t>(len, kSlice), hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipEventRecord(ev[0], st) != hipSuccess))
        return false;
    for (uint64_t j = 0; j < ns; ++j) {
        const uint64_t off = j * kSlice, n = std::min<uint64_t>(len - off, kSlice);
        uint8_t* cur = buf + (j & 1) * kSlice;
        if (j + 1 < ns) {
            const uint64_t n2 = std::min<uint64_t>(len - off - kSlice, kSlice);
            if (hipMemcpyAsync(buf + ((j + 1) & 1) * kSlice, src + off + kSlice, n2, hipMemcpyDeviceToHost, st) !=
                    hipSuccess ||
                hipEventRecord(ev[(j + 1) & 1], st) != hipSuccess)
                return false;
        }
        if (hipEventSynchronize(ev[j & 1]) != hipSuccess) return false;
        if (j + 1 < ns) {
            pbs::sha256_host_blocks(h, cur, n);
        } else {
            pbs::sha256_host_blocks(h, cur, n / 64 * 64);
            pbs::sha256_host_final(h, cur + n / 64 * 64, n % 64, key, key_len, out);
        }
    }
    if (!ns) pbs::sha256_host_final(h, nullptr, 0, key, key_len, out);
    return true;
}

// The host share items[0..h) from HBM through the ring: one copier (this thread) copies
// whole chunks into free slots back to back on `ncs` (1-2) copy streams in turn; `t`
// threads hash them as they land, up to four in step each (pbs::sha256_host_lanes), and
// free their slots.  Every chunk must fit a slot (sb bytes).  `bad` changes under qm, so no
// wait misses it.  False on a HIP error (no copy in flight on return).
bool hash_ring(HostStage& hs, size_t slots, size_t sb, const uint8_t* dev_data, uint64_t base,
               const uint64_t* bounds, const uint32_t* items, size_t h, const uint8_t* key, size_t key_len,
               uint8_t* digests, int t, int ncs) {
    std::mutex qm;
    std::condition_variable qcv;
    std::deque<size_t> freeq;
    std::deque<std::pair<uint32_t, size_t>> landed;  // (chunk, slot) in copy order
    bool copies_done = false;
    std::atomic<bool> bad{false};
    for (size_t j = 0; j < slots; ++j) freeq.push_back(j);
    auto next = [&](pbs::ShaJob& job, bool block) {
        std::unique_lock<std::mutex> g(qm);
        for (;;) {
            if (bad) return false;
            if (!landed.empty()) {
                const auto [i, slot] = landed.front();
                const hipError_t q = hipEventQuery(hs.rev[slot]);
                if (q == hipSuccess) {
                    landed.pop_front();
                    job = pbs::ShaJob{hs.ring + slot * sb, bounds[i + 1] - bounds[i], digests + 32 * (size_t)i, slot};
                    return true;
                }
                if (q != hipErrorNotReady) {
                    bad = true;
                    qcv.notify_all();
                    return false;
                }
                if (!block) return false;
                g.unlock();
                const bool ok = hipEventSynchronize(hs.rev[slot]) == hipSuccess;
                g.lock();
                if (!ok) {
                    bad = true;  // (under the lock, then a wake-up: the copier may wait for a slot)
                    qcv.notify_all();
                    return false;
                }
                continue;
            }
            if (copies_done || !block) return false;
            qcv.wait(g);
        }
    };
    auto done = [&](const pbs::ShaJob& job) {
        {
            std::lock_guard<std::mutex> g(qm);
            freeq.push_back((size_t)job.tag);
        }
        qcv.notify_all();
    };
    std::vector<std::thread> pool;
    for (int j = 0; j < t; ++j) pool.emplace_back([&] { pbs::sha256_host_lanes(next, done, key, key_len); });
    for (size_t k = 0; k < h && !bad; ++k) {
        size_t slot;
        {
            std::unique_lock<std::mutex> g(qm);
            qcv.wait(g, [&] { return !freeq.empty() || bad; });
            if (bad) break;
            slot = freeq.front();
            freeq.pop_front();
        }
        const uint32_t i = items[k];
        if (hipMemcpyAsync(hs.ring + slot * sb, dev_data + (bounds[i] - base), bounds[i + 1] - bounds[i],
                           hipMemcpyDeviceToHost, hs.cst[k % ncs]) != hipSuccess ||
            hipEventRecord(hs.rev[slot], hs.cst[k % ncs]) != hipSuccess) {
            std::lock_guard<std::mutex> g(qm);
            bad = true;
            break;
        }
        {
            std::lock_guard<std::mutex> g(qm);
            landed.emplace_back(i, slot);
        }
        qcv.notify_all();
    }
    {
        std::lock_guard<std::mutex> g(qm);
        copies_done = true;
    }
    qcv.notify_all();
    for (auto& th : pool) th.join();
    for (int j = 0; j < ncs; ++j)
        if (hipStreamSynchronize(hs.cst[j]) != hipSuccess) bad = true;
    return !bad;
}

}  // namespace

// Frees the hybrid digest's pinned host slices and their streams.
extern "C" void pbs_digest_hybrid_release(void) {
    for (int d = 0; d < kMaxStageDevices; ++d) {
        HostStage* hs;
        {
            std::lock_guard<std::mutex> lk(g_stage_mu);
            hs = g_stages[d];
        }
        if (!hs) continue;
        std::lock_guard<std::mutex> lk(hs->mu);
        hs->release();
        hs->dev = -1;
    }
    digest_pool().clear();
    known_pool().clear();
}

extern "C" int pbs_digest_chunks_hybrid(const uint8_t* dev_data, const uint8_t* host_data, size_t data_len,
                                        uint64_t base, const uint64_t* bounds, size_t n, const uint8_t* key,
                                        size_t key_len, uint8_t* digests, const pbs_digest_hybrid_opts* opts,
                                        pbs_digest_hybrid_timing* timing, void* hip_stream) {
    const HClock::time_point t0 = HClock::now();
    if (timing) std::memset(timing, 0, sizeof(*timing));
    if (n == 0) return PBS_OK;
    if (!bounds || !digests || (data_len && !dev_data) || key_len > PBS_DIGEST_MAX_KEY || (key_len && !key) ||
        n > 0xFFFFFFFFull)
        return PBS_ERR_INVALID;
    for (size_t i = 0; i < n; ++i)
        if (bounds[i] > bounds[i + 1] || bounds[i] < base || bounds[i + 1] - base > data_len)
            return PBS_ERR_INVALID;
    pbs_digest_hybrid_opts o{};
    if (opts) o = *opts;
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int threads = o.host_threads < 0 ? 0 : o.host_threads == 0 ? std::min(hw, 16) : o.host_threads;
    // per thread: ~4.3 GB/s with the SHA extensions and four chunks in step (EPYC 9575F,
    // profiles/r04/sha_lanes/), far less with the portable rounds
    const double host_rate = (o.host_mb_s > 0 ? o.host_mb_s : pbs::sha256_host_has_ni() ? 4000.0 : 250.0) * 1e6;
    const double gpu_rate = (o.gpu_mb_s > 0 ? o.gpu_mb_s : 35.0) * 1e6;        // bytes/s per chain
    // from HBM the host share is copied whole chunk by whole chunk into a pinned ring
    // (round 2's per-thread 4 MiB slices moved only ~14 GB/s over 16 threads)
    const double agg = std::min(threads * host_rate, host_data ? 1e12 : kD2HRate);
    hipStream_t st = (hipStream_t)hip_stream;
    auto clen = [&](uint32_t i) { return bounds[i + 1] - bounds[i]; };
    int sdev = 0;
    if (hipStreamGetDevice(st, &sdev) != hipSuccess) return PBS_ERR_NO_DEVICE;
    pbs::DeviceGuard dg(sdev);  // the scratch below belongs on the stream's device
    if (!dg.ok) return PBS_ERR_NO_DEVICE;

    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return clen(a) > clen(b); });
    size_t m = 0;  // the long chunks (order prefix) get the zero test
    if (threads > 0)
        while (m < n && clen(order[m]) >= kZeroMin) ++m;

    pbs::ArenaLease ar(digest_pool(), sdev);
    uint64_t* d_bounds = ar->get<uint64_t>(0, (n + 1) * 8);
    uint32_t* d_order = ar->get<uint32_t>(1, n * 4);
    uint8_t* d_dig = ar->get<uint8_t>(2, n * 32);
    uint8_t* d_flags = m ? ar->get<uint8_t>(3, m) : nullptr;
    int rc = PBS_OK;
    auto fail = [&](int r) {
        if (rc == PBS_OK) rc = r;
    };
    if (!d_bounds || !d_order || !d_dig || (m && !d_flags)) fail(PBS_ERR_NOMEM);
    std::vector<uint8_t> zf(m, 0);
    // the host share's D2H copies run on the HostStage streams, which do not wait for the
    // caller's stream: this event marks the point on `st` after the caller's producer
    // work (recorded before anything of ours, so the copies do not also wait for the GPU
    // digest launch)
    hipEvent_t ready = nullptr;
    if (rc == PBS_OK && !host_data && threads > 0 && (!(ready = ar->event(2)) || hipEventRecord(ready, st) != hipSuccess))
        fail(PBS_ERR_HIP);
    if (rc == PBS_OK && (hipMemcpyAsync(d_bounds, bounds, (n + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
                         hipMemcpyAsync(d_order, order.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess))
        fail(PBS_ERR_HIP);
    if (rc == PBS_OK && m) {
        hipLaunchKernelGGL(zero_flags_kernel, dim3((unsigned)m), dim3(256), 0, st, dev_data, base, d_bounds,
                           d_order, (uint64_t)m, d_flags);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(zf.data(), d_flags, m, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            fail(PBS_ERR_HIP);
    }
    const HClock::time_point t_zero = HClock::now();

    // work list: every chunk except the repeats of an all-zero length (longest first)
    std::vector<uint32_t> work;
    work.reserve(n);
    std::vector<std::pair<uint32_t, uint32_t>> dup;  // (zero chunk, its length's representative)
    uint64_t zero_chunks = 0, zero_lengths = 0;
    for (size_t k = 0; k < n; ++k) {
        const uint32_t i = order[k];
        if (k < m && zf[k]) {
            ++zero_chunks;
            // order is sorted by length, so one length's zero chunks are adjacent in dup
            if (!dup.empty() && clen(dup.back().second) == clen(i)) {
                dup.emplace_back(i, dup.back().second);
            } else {
                ++zero_lengths;
                dup.emplace_back(i, i);  // i is its own length's representative
                work.push_back(i);
            }
        } else {
            work.push_back(i);
        }
    }
    // split: the first h work items go to the host; minimise max(host time, GPU time)
    size_t h = 0;
    if (threads > 0 && rc == PBS_OK) {
        if (o.host_min_len) {
            while (h < work.size() && clen(work[h]) >= o.host_min_len) ++h;
        } else {
            double best = (double)clen(work[0]) / gpu_rate, acc = 0;
            for (size_t k = 1; k <= work.size(); ++k) {
                acc += (double)clen(work[k - 1]);
                const double c = std::max(acc / agg, k < work.size() ? (double)clen(work[k]) / gpu_rate : 0.0);
                if (c < best) {
                    best = c;
                    h = k;
                }
            }
        }
    }
    const size_t g = work.size() - h;
    hipEvent_t ev[2] = {nullptr, nullptr};
    if (rc == PBS_OK && g) {
        if (!(ev[0] = ar->event(0)) || !(ev[1] = ar->event(1)) ||
            hipMemcpyAsync(d_order, work.data() + h, g * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipEventRecord(ev[0], st) != hipSuccess)
            fail(PBS_ERR_HIP);
        else {
            const int r = pbs_digest_chunks_async(dev_data, data_len, base, d_bounds, d_order, g, key, key_len,
                                                  d_dig, hip_stream);
            if (r != PBS_OK)
                fail(r);
            else if (hipEventRecord(ev[1], st) != hipSuccess)
                fail(PBS_ERR_HIP);
        }
    }
    // host share, overlapping the GPU launch
    const HClock::time_point t_host0 = HClock::now();
    uint64_t host_bytes = 0;
    for (size_t k = 0; k < h; ++k) host_bytes += clen(work[k]);
    if (rc == PBS_OK && h) {
        if (host_data) {
            pbs::sha256_host_items(host_data, base, bounds, work.data(), h, key, key_len, digests, threads);
        } else if (HostStage* const hsp = host_stage(sdev)) {
            HostStage& hs = *hsp;
            std::lock_guard<std::mutex> lk(hs.mu);
            const int dv = sdev;
            const int t = (int)std::min<size_t>((size_t)threads, h);
            // whole chunks through the ring when a slot can hold the longest (always for the
            // reference's chunk sizes, <= 16 MiB); slots for four open chunks per thread + 8
            // in flight, within kRingMax
            const uint64_t sb = (clen(work[0]) + 4095) / 4096 * 4096;
            const size_t slots = std::min<size_t>(std::min<size_t>(h, 4 * (size_t)t + 8),
                                                  sb ? (size_t)(kRingMax / sb) : 0);
            const char* re = std::getenv("PBS_DIGEST_RING");  // 0: per-thread slices (tests, A/B)
            const bool use_ring = sb && slots >= 2 && !(re && re[0] == '0');
            bool waits = true;
            if (use_ring ? !hs.ring_grow(dv, slots, sb) : !hs.grow(dv, t)) {
                fail(PBS_ERR_NOMEM);
            } else if (use_ring) {
                waits = hipStreamWaitEvent(hs.cst[0], ready, 0) == hipSuccess &&
                        hipStreamWaitEvent(hs.cst[1], ready, 0) == hipSuccess;
                if (!waits) fail(PBS_ERR_HIP);
            } else {
                for (int j = 0; j < t; ++j)
                    waits = waits && hipStreamWaitEvent(hs.st[j], ready, 0) == hipSuccess;
                if (!waits) fail(PBS_ERR_HIP);
            }
            if (rc == PBS_OK && use_ring) {
                const char* ce = std::getenv("PBS_DIGEST_RING_STREAMS");  // copy streams, 1-2 (A/B)
                const int ncs = ce && ce[0] == '1' ? 1 : 2;
                if (!hash_ring(hs, slots, sb, dev_data, base, bounds, work.data(), h, key, key_len, digests, t, ncs))
                    fail(PBS_ERR_HIP);
            } else if (rc == PBS_OK) {
                std::atomic<size_t> next{0};
                std::atomic<bool> bad{false};
                auto run = [&](int j) {
                    for (size_t k; !bad && (k = next.fetch_add(1)) < h;) {
                        const uint32_t i = work[k];
                        if (!hash_from_device(dev_data + (bounds[i] - base), clen(i), key, key_len,
                                              digests + 32 * (size_t)i, hs.buf[j], hs.st[j], &hs.ev[2 * j]))
                            bad = true;
                    }
                };
                std::vector<std::thread> pool;
                for (int j = 1; j < t; ++j) pool.emplace_back(run, j);
                run(0);
                for (auto& th : pool) th.join();
                if (bad) fail(PBS_ERR_HIP);
            }
        } else {
            fail(PBS_ERR_NO_DEVICE);
        }
    }
    const HClock::time_point t_host1 = HClock::now();
    float gpu_ms = 0;
    std::vector<uint8_t> gd;
    if (rc == PBS_OK && g) {
        gd.resize(n * 32);
        if (hipMemcpyAsync(gd.data(), d_dig, n * 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess || hipEventElapsedTime(&gpu_ms, ev[0], ev[1]) != hipSuccess)
            fail(PBS_ERR_HIP);
        else
            for (size_t k = h; k < work.size(); ++k)
                std::memcpy(digests + 32 * (size_t)work[k], gd.data() + 32 * (size_t)work[k], 32);
    }
    if (rc == PBS_OK)
        for (const auto& d : dup)
            if (d.first != d.second) std::memcpy(digests + 32 * (size_t)d.first, digests + 32 * (size_t)d.second, 32);
    (void)hipStreamSynchronize(st);  // nothing of ours in flight when the arena goes back
    if (timing) {
        const HClock::time_point t1 = HClock::now();
        timing->total_ms = hms(t0, t1);
        timing->zero_ms = hms(t0, t_zero);
        timing->gpu_ms = gpu_ms;
        timing->host_ms = hms(t_host0, t_host1);
        timing->gpu_chunks = g;
        timing->host_chunks = h;
        timing->host_bytes = host_bytes;
        timing->zero_chunks = zero_chunks;
        timing->zero_lengths = zero_lengths;
        timing->threshold = h ? clen(work[h - 1]) : 0;
        timing->threads = threads;
    }
    return rc;
}
