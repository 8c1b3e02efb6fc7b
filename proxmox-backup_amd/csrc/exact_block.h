// Exact candidate positions of one 128-byte block, computed by ONE WAVE (shared by
// scan_exact_kernel, scan_blocks_kernel and the fused pass, scan_fused.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbs {

constexpr int kExactBlock = 128;  // bytes per block (= scan_main's lane iteration)

// Bytes before data[0] come from `pre` (the last pre_len <= 63 bytes of the stream
// before this buffer); bytes before that do not exist and contribute nothing, as in
// the reference's fill phase.  Position p is a candidate iff the window is full
// (p + pre_len >= 63) and (H(p) & mask) >= minimum; it is written as base + p.
// Exact hits of one 128-byte block, computed by ONE WAVE (B = block start relative to
// `data`, may be negative on the aligned block grid; window = bytes [B-64, B+128)).
// A per-thread roll is a 192-step dependent chain (~22k cycles for one block); instead
// the window hash is a difference of prefix XORs:
//   h(j) = rotl( P(j) ^ P(j-64), j mod 32 ),   P(j) = XOR_{i<=j} rotr( T[w_i], i mod 32 )
// (rotl(T, j-i) = rotl(rotr(T, i), j), so the rotation of each term only depends on its
// own index; window indices j, i).  Lane l < 48 owns window bytes [4l, 4l+4): one dword
// load, 4 table lookups, a wave-wide prefix XOR (6 DPP steps) and P(j-64) from lane l-16;
// lanes 16..47 test positions j = 64..191, i.e. block positions 4(l-16)+k.
// Bytes that do not exist (before the stream, after `len`) are read with clamped
// addresses: a reportable position (q >= 0, q < len, q + pre_len >= 63) has all 64
// window bytes in existence and its P-difference involves only them; the hit words are
// clipped to reportable positions.  Returns the 4 hit words (bit j = position B + j),
// uniform across the wave.  `pre` has 64 readable bytes; `len` >= 1.
// exact_load: lane l's window dword (the memory half, issued ahead by the caller);
// exact_hits: the hash and test (the compute half).
__device__ __forceinline__ uint32_t exact_load(const uint8_t* __restrict__ data, uint64_t len,
                                               const uint8_t* __restrict__ pre, uint32_t pre_len,
                                               int64_t B, int lane) {
    const int64_t q0 = B - 64;
    const int64_t ilen = (int64_t)len, plen = (int64_t)pre_len;
    uint32_t wv = 0;
    if (lane < 48) {
        const int64_t q = q0 + 4 * lane;
        if (q >= 0 && q + 4 <= ilen && ((uintptr_t)(data + q) & 3) == 0) {
            wv = *reinterpret_cast<const uint32_t*>(data + q);
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int64_t qq = q + b;
                const uint32_t bd = data[qq < 0 ? 0 : (qq >= ilen ? ilen - 1 : qq)];
                const int64_t qp = plen + qq;
                const uint32_t bp = pre[qp < 0 ? 0 : (qp > 63 ? 63 : qp)];
                wv |= (qq < 0 ? bp : bd) << (8 * b);
            }
        }
    }
    return wv;
}

// v moved across lanes by the DPP control CTRL (rows/banks outside the masks, and lanes
// whose source lies outside their row, read 0: the identity of XOR, OR and +).  Callers
// run with all 64 lanes active (wave-uniform control flow), as every caller here does.
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, BANK_MASK, false);
}

// inclusive prefix sum over the 64 lanes (DPP: row shifts, then the row totals)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += dpp_mov<0x111>(v);
    v += dpp_mov<0x112>(v);
    v += dpp_mov<0x114>(v);
    v += dpp_mov<0x118>(v);
    v += dpp_mov<0x142, 0xa>(v);
    v += dpp_mov<0x143, 0xc>(v);
    return v;
}

// ROT = false: `tab` is the plain table (256 words), the test (h & mask) >= minimum
// (chunker.rs:185).  ROT = true: `tab` is the scan kernels' pre-rotated table replicated
// 64x (T' = rotl(T, rot) at dword b*64 + lane, conflict-free for any 64 bytes) and `mask`
// holds thr: T' makes every prefix XOR, and so every window hash, rotl(h, rot), and
// rotl(h, rot) >= thr <=> (h & mask) >= minimum exactly (thr = minimum << rot,
// pbs_chunker_capi.cpp make_params, frame 1).
template <bool ROT = false>
__device__ __forceinline__ uint4 exact_hits(uint32_t wv, uint64_t len, uint32_t pre_len, int64_t B,
                                            const uint32_t* tab, uint32_t mask, uint32_t minimum,
                                            int lane) {
    const int64_t q0 = B - 64;
    const int64_t ilen = (int64_t)len, plen = (int64_t)pre_len;
    uint32_t u[4], acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t j = 4u * (uint32_t)lane + (uint32_t)k;
        const uint32_t byte = (wv >> (8 * k)) & 0xffu;
        uint32_t t = ROT ? tab[byte * 64u + (uint32_t)lane] : tab[byte];
        t = __builtin_amdgcn_alignbit(t, t, j & 31u);  // rotr(t, j)
        acc ^= lane < 48 ? t : 0u;
        u[k] = acc;
    }
    // inclusive prefix XOR over lanes with DPP (VALU lane moves, no LDS round trip):
    // shifts 1, 2, 4, 8 inside each row of 16, then the row totals by row_bcast
    uint32_t S = acc;
    S ^= dpp_mov<0x111>(S);  // row_shr:1
    S ^= dpp_mov<0x112>(S);  // row_shr:2
    S ^= dpp_mov<0x114>(S);  // row_shr:4
    S ^= dpp_mov<0x118>(S);  // row_shr:8
    S ^= dpp_mov<0x142, 0xa>(S);  // row_bcast:15 into rows 1 and 3
    S ^= dpp_mov<0x143, 0xc>(S);  // row_bcast:31 into rows 2 and 3
    const uint32_t E = S ^ acc;  // exclusive
    uint32_t nib = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t P = E ^ u[k];
        const uint32_t Pm = __shfl(P, lane >= 16 ? lane - 16 : lane, 64);
        const uint32_t j = 4u * (uint32_t)lane + (uint32_t)k;
        uint32_t h = P ^ Pm;
        h = __builtin_amdgcn_alignbit(h, h, (32u - (j & 31u)) & 31u);  // rotl(h, j)
        nib |= ((ROT ? h >= mask : (h & mask) >= minimum) ? 1u : 0u) << k;
    }
    const bool tester = lane >= 16 && lane < 48;
    uint32_t v = tester ? nib << (4 * ((lane - 16) & 7)) : 0u;
    v |= dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
    v |= dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
    v |= dpp_mov<0x141>(v);  // row_half_mirror: the other quad of the 8 lanes
    uint4 hit = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)v, 16),
                           (uint32_t)__builtin_amdgcn_readlane((int)v, 24),
                           (uint32_t)__builtin_amdgcn_readlane((int)v, 32),
                           (uint32_t)__builtin_amdgcn_readlane((int)v, 40));
    const bool fast = B >= 64 && B + kExactBlock <= ilen;
    if (!fast) {
        // reportable window indices [cmin, vhi): q >= 0, q + pre_len >= 63, q < len
        int64_t cm = 64;
        if (64 - B > cm) cm = 64 - B;
        if (127 - plen - B > cm) cm = 127 - plen - B;
        const int64_t hi = ilen - q0;
        const int cmin = (int)(cm > 192 ? 192 : cm) - 64;  // bit range [cmin, chi)
        const int chi = (int)(hi < 64 ? 64 : (hi > 192 ? 192 : hi)) - 64;
        uint32_t hw[4] = {hit.x, hit.y, hit.z, hit.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int lo = cmin - 32 * q, up = chi - 32 * q;  // keep bits [lo, up) of word q
            const uint32_t keep_lo = lo <= 0 ? 0xFFFFFFFFu : (lo >= 32 ? 0u : (0xFFFFFFFFu << lo));
            const uint32_t keep_hi = up >= 32 ? 0xFFFFFFFFu : (up <= 0 ? 0u : (0xFFFFFFFFu >> (32 - up)));
            hw[q] &= keep_lo & keep_hi;
        }
        hit = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    }
    return hit;
}

__device__ __forceinline__ uint4 exact_block_wave(const uint8_t* __restrict__ data, uint64_t len,
                                                  const uint8_t* __restrict__ pre,
                                                  uint32_t pre_len, int64_t B, const uint32_t* tab,
                                                  uint32_t mask, uint32_t minimum, int lane) {
    const uint32_t wv = exact_load(data, len, pre, pre_len, B, lane);
    return exact_hits(wv, len, pre_len, B, tab, mask, minimum, lane);
}


}  // namespace pbs
