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
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"
#include "pbs_digest.h"

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
__global__ __launch_bounds__(64 * kShaWaves) void sha256_chunks_split_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint32_t* __restrict__ order, uint64_t n, DigestKey key, uint8_t* __restrict__ digests) {
    __shared__ uint4 sw[2][16][64];  // [buffer][t / 4][lane]: W[t] + K[t] for 4 t (b128 per lane)
    __shared__ uint32_t s_blocks;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t k = (uint64_t)blockIdx.x * 64 + lane;
    const bool live = k < n;
    const uint64_t i = live ? (order ? order[k] : k) : 0;
    const uint64_t s = live ? bounds[i] - base : 0, e = live ? bounds[i + 1] - base : 0;
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

    // wave 1: message block b -> W + K into buffer b & 1.  The data window of block b
    // was loaded during the previous block's period (`pre`); the loads of block b + 1
    // are issued here, before the schedule, so HBM latency hides behind a block period.
    uint32_t pre[17];
    if (wave == 1 && nfull) load_window(pa, r != 0, pre);
    auto produce = [&](uint32_t b) {
        uint32_t w[16];
        if ((uint64_t)b < nfull) {
            uint32_t d[17];
#pragma unroll
            for (int q = 0; q < 17; ++q) d[q] = pre[q];
            if ((uint64_t)b + 1 < nfull) load_window(pa + 16 * ((uint64_t)b + 1), r != 0, pre);
#pragma unroll
            for (int q = 0; q < 16; ++q) w[q] = __builtin_amdgcn_perm(d[q + 1], d[q], sel);
        } else if ((uint64_t)b < total) {
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
        uint4 (*out)[64] = sw[b & 1];
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
    if (wave == 1 && nblocks) produce(0);
    __syncthreads();
#ifdef PBS_SHA_PROBE  // scripts/microbench/mb_sha.hip: cycles of each wave's work vs the barrier
    uint64_t pr_work = 0, pr_wait = 0;
#endif
    for (uint32_t b = 0; b < nblocks; ++b) {
#ifdef PBS_SHA_PROBE
        const uint64_t c0 = clock64();
#endif
        if (wave == 1) {
            if (b + 1 < nblocks) produce(b + 1);
        } else if ((uint64_t)b < total) {
            const uint4 (*in)[64] = sw[b & 1];
            uint32_t a = st[0], bb = st[1], c = st[2], d = st[3], ee = st[4], f = st[5], g = st[6], h = st[7];
            uint4 kw4 = in[0][lane];
#pragma unroll
            for (int t = 0; t < 64; ++t) {
                const uint32_t kw = (t & 3) == 0 ? kw4.x : (t & 3) == 1 ? kw4.y : (t & 3) == 2 ? kw4.z : kw4.w;
                if ((t & 3) == 3 && t < 63) kw4 = in[(t >> 2) + 1][lane];
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
    }
#ifdef PBS_SHA_PROBE
    if (blockIdx.x == 0 && lane == 0) {
        g_sha_probe[wave * 2] = pr_work;
        g_sha_probe[wave * 2 + 1] = pr_wait;
        g_sha_probe[4] = nblocks;
    }
#endif
    if (wave == 0 && live) {
        uint32_t* out = reinterpret_cast<uint32_t*>(digests + 32 * i);
#pragma unroll
        for (int q = 0; q < 8; ++q) out[q] = __builtin_bswap32(st[q]);
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

}  // namespace
}  // namespace pbs

using namespace pbs;

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
    uint64_t* d_bounds = nullptr;
    uint32_t* d_order = nullptr;
    uint8_t* d_dig = nullptr;
    int rc = PBS_OK;
    if (hipMalloc(&d_bounds, (n + 1) * 8) != hipSuccess || hipMalloc(&d_order, n * 4) != hipSuccess ||
        hipMalloc(&d_dig, n * 32) != hipSuccess) {
        rc = PBS_ERR_NOMEM;
    } else if (hipMemcpyAsync(d_bounds, bounds, (n + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
               hipMemcpyAsync(d_order, order.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = PBS_ERR_HIP;
    } else {
        rc = pbs_digest_chunks_async(dev_data, data_len, base, d_bounds, d_order, n, key, key_len,
                                     d_dig, hip_stream);
        if (rc == PBS_OK &&
            (hipMemcpyAsync(digests, d_dig, n * 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
             hipStreamSynchronize(st) != hipSuccess))
            rc = PBS_ERR_HIP;
    }
    if (d_bounds) (void)hipFree(d_bounds);
    if (d_order) (void)hipFree(d_order);
    if (d_dig) (void)hipFree(d_dig);
    return rc;
}

extern "C" int pbs_known_chunks_device(const uint8_t* digests_dev, size_t n, const uint8_t* known_dev,
                                       size_t k, uint8_t* is_known_dev, size_t* n_known,
                                       void* hip_stream) {
    if (n_known) *n_known = 0;
    if (n == 0) return PBS_OK;
    if (!digests_dev || !is_known_dev || (k && !known_dev) || n > 0xFFFFFFF0u) return PBS_ERR_INVALID;
    hipStream_t st = (hipStream_t)hip_stream;
    uint64_t *key = nullptr, *skey = nullptr;
    uint32_t *idx = nullptr, *sidx = nullptr, *head = nullptr, *rstart = nullptr;
    unsigned int* cnt = nullptr;
    void* tmp = nullptr;
    int rc = PBS_OK;
    size_t tb_sort = 0, tb_scan = 0;
    const unsigned grid = (unsigned)((n + 255) / 256);
    if (hipMalloc(&key, n * 8) != hipSuccess || hipMalloc(&skey, n * 8) != hipSuccess ||
        hipMalloc(&idx, n * 4) != hipSuccess || hipMalloc(&sidx, n * 4) != hipSuccess ||
        hipMalloc(&head, n * 4) != hipSuccess || hipMalloc(&rstart, n * 4) != hipSuccess ||
        hipMalloc(&cnt, 4) != hipSuccess) {
        rc = PBS_ERR_NOMEM;
        goto done;
    }
    if (radix_sort(nullptr, &tb_sort, key, skey, idx, sidx, n, 0, 64, st) != hipSuccess ||
        inclusive_max_u32(nullptr, &tb_scan, head, rstart, n, st) != hipSuccess ||
        hipMalloc(&tmp, std::max(tb_sort, tb_scan)) != hipSuccess) {
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
    for (void* q : {(void*)key, (void*)skey, (void*)idx, (void*)sidx, (void*)head, (void*)rstart, (void*)cnt, tmp})
        if (q) (void)hipFree(q);
    return rc;
}
