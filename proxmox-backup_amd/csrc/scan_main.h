// scan_main_kernel: phase A main pass of the gfx950 chunker (geometry and hash
// representation: pbs_chunker_kernels.hip and DESIGN.md "Kernel: scan_main").  Kept in a
// header so the product library and the microbenchmarks (scripts/microbench/) build the
// same code; the rejected design variants live in scripts/microbench/scan_variants.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace pbs {

// MODE 0: product.  MODE 1: loads only (DMA + LDS reads, no hash) and MODE 2: hash
// only (the staged block is re-used, no HBM traffic) -- microbenchmark ablations.
constexpr int kModeFull = 0, kModeLoadOnly = 1, kModeComputeOnly = 2;

#include "roll128_asm.h"  // roll128_asm(): hand-scheduled 128-byte body (gen_roll_asm.py)

constexpr int kWavesPerWG = 8;  // product geometry
constexpr int kIter = 128;                       // bytes per lane per iteration
constexpr int kStagePerWave = 64 * kIter;        // 8 KiB
constexpr int kTableDwords = 256 * 64;           // 64 KiB
constexpr int kSuspBuf = 128;                    // per-wave LDS list of suspect blocks (1 KiB)
// s_getreg_b32 operand for HW_REG_HW_ID (id 4, offset 0, 32 bits): SIMD_ID in bits 5:4
constexpr int kHwRegHwId = 4 | (31 << 11);

__device__ __forceinline__ uint32_t rotl1(uint32_t h) {
    return __builtin_amdgcn_alignbit(h, h, 31);
}
__device__ __forceinline__ uint32_t umax3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t m = a > b ? a : b;
    return m > c ? m : c;
}

// ---------------------------------------------------------------------------------
// 8 waves per CU (one 512-thread workgroup, persistent), 128-byte iterations, one
// 8 KiB LDS stage per wave.  The block of iteration it+1 is staged by 8 LDS-DMA
// instructions (buffer_load_dwordx4 ... lds, nt) issued from a per-tile buffer
// descriptor (SGPR base + SGPR iteration offset + constant per-lane VGPR offset: no
// VALU address math) as soon as iteration it's block is in VGPRs; the hash loop is the
// hand-scheduled roll128_asm_g4 (G = bytes per lgkmcnt wait).  PF > 0 adds an L2
// "touch" DMA PF iterations ahead (measured slower; kept for the microbenchmark).
// Design record of the variants measured against it: DESIGN.md "Kernel: scan_main".
//
// ZS (zero-run skip): the hash of any 64 equal bytes is 0 (rotations k and k+32 of the
// same table word cancel), so a lane whose previous 128-byte block was all zero is in
// the state {h = 0, every ring slot = T'[0]}; an all-zero block leaves that state
// unchanged and holds no candidate (thr > 0), so the lane skips its roll (EXEC-masked;
// a wave whose 64 lanes all skip branches over it).  Detecting it costs ~16 v_or3 per
// 128 bytes.  Measured (profiles/r01/mb_zs_*.log): all-zero input reaches the
// loads-only rate, but random and VM-image data get 2-3% SLOWER -- lanes 32 KiB apart
// are almost never all in zero pages at once, and masked lanes save little -- so the
// product runs ZS = 0.
// FR (hash frame): 1 = h' = rotl(h, 32-n) for every byte, table T' = rotl(T, 32-n)
// replicated 64x (3.5 VALU/byte), exact block test -- the product (kScanFrame); 2 =
// parity frame of roll128_asm_f2 (3 VALU/byte), table = [T0 | T1] (512 words)
// interleaved 32x per 256-byte row, thr = the screening threshold of DESIGN.md section 6
// (a necessary condition; scan_exact re-tests exactly): faster hash-only (7.7-8.0 vs
// 7.2 TB/s) but 2-4 % slower in the full, power-limited kernel (profiles/r01/fr2/).
// DYN (tile order): 0 = static, wave w takes tiles w, w + nw, ...; 1 = the first nw tiles
// static, then each wave takes its next tile from a device counter (one atomic per
// tile, issued at the tile's first iteration, read at its last), so waves on faster CUs
// take more tiles -- and tiles t >= t_big are "small" (segments of SEG / 4), so the
// waves also finish together: the last tiles are a quarter as long.  Measured per-wave
// finish times (scripts/microbench/scan_probe.py): static order 7.4-11.2 ms for the
// 64 GiB stream (the older wave of a SIMD wins the issue arbitration), dynamic
// 10.3-10.7 ms.
#ifdef PBS_SCAN_PROBE
constexpr int kScanProbeMax = 4096;
__device__ uint64_t g_scan_probe[2 * kScanProbeMax];  // finish times, then start times
#endif
template <int SEG, int MODE = kModeFull, int AUX = 2, int G = 4, int PF = 0, int ZS = 0, int FR = 1,
          int DYN = 0>
__global__ __launch_bounds__(kWavesPerWG * 64) void scan_main_kernel(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, unsigned long long* __restrict__ nsusp, uint64_t cap,
    uint32_t* __restrict__ tile_ctr = nullptr, uint64_t t_big = ~0ull, uint32_t balance_on = 0) {
    static_assert(SEG % kIter == 0, "segment must be a multiple of the iteration size");
    constexpr int SEG2 = SEG / 4;  // DYN: segment length of the small tiles (t >= t_big)
    static_assert(SEG2 % kIter == 0, "small segment must be a multiple of the iteration size");
    constexpr int NW = kWavesPerWG;
    // + 256 B per wave: landing area of the L2 "touch" DMAs (PF > 0); + 1 KiB per wave:
    // the wave's suspect list
    __shared__ __attribute__((aligned(16)))
    uint32_t s_lds[kTableDwords + NW * kStagePerWave / 4 + NW * 64 + NW * kSuspBuf * 2];

    __shared__ uint32_t s_simd[NW], s_prog[NW];  // SIMD of each wave; blocks scanned so far

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (lane == 0) {
        s_simd[wave] = (__builtin_amdgcn_s_getreg(kHwRegHwId) >> 4) & 3u;  // HW_ID.SIMD_ID
        s_prog[wave] = 0;
    }
    if constexpr (FR == 2) {
        for (int i = tid; i < kTableDwords; i += NW * 64)
            s_lds[i] = table_rot[((i >> 5) & 1) * 256 + (i >> 6)];
    } else {
        for (int i = tid; i < kTableDwords; i += NW * 64) s_lds[i] = table_rot[i >> 6];
    }
    __syncthreads();
    // balance_on: the wave behind its SIMD partner (the other wave of this workgroup on its
    // SIMD) takes the issue priority -- the arbiter otherwise favours the older wave by ~30 %
    // (scripts/microbench/fused_probe.py), and in the static tile order the younger one then
    // finishes alone
    int partner = wave;
    for (int w = 0; w < NW; ++w)
        if (w != wave && s_simd[w] == s_simd[wave]) partner = w;
    partner = __builtin_amdgcn_readfirstlane(partner);
    const bool balance = balance_on != 0 && partner != wave;
    uint32_t prog = 0;

    uint8_t* stage = (uint8_t*)(s_lds + kTableDwords) + wave * kStagePerWave;
    uint8_t* touch_area = (uint8_t*)(s_lds + kTableDwords + NW * kStagePerWave / 4) + wave * 256;
    const uint32_t voff_touch = (uint32_t)lane * (uint32_t)SEG + 64u;
    // Suspect blocks are collected per wave in LDS and appended to susp[] with one atomic
    // per kSuspBuf - 63 or more: an atomic per suspect (the wave waiting for its return
    // before the store) cost 26 % at 64 KiB averages (~1 suspect per 340 blocks).
    uint64_t* s_susp = (uint64_t*)(s_lds + kTableDwords + NW * kStagePerWave / 4 + NW * 64) + wave * kSuspBuf;
    uint32_t scnt = 0;  // wave-uniform
    auto flush = [&]() {
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(nsusp, (unsigned long long)scnt);
        b = ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
            __builtin_amdgcn_readfirstlane((uint32_t)b);
        for (uint32_t i = lane; i < scnt; i += 64)
            if (b + i < cap) susp[b + i] = s_susp[i];
        scnt = 0;
    };
    const uint32_t lanebase = (uint32_t)lane * 4u;
    const uint32_t lb0 = ((uint32_t)lane & 31u) * 4u, lb1 = lb0 + 128u;
    uint32_t voff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t l = 8u * j + ((uint32_t)lane >> 3);
        const uint32_t k = ((uint32_t)lane & 7u) ^ ((l >> 1) & 7u);
        voff[j] = l * (uint32_t)SEG + k * 16u;
    }
    uint32_t voff2[8];  // DYN: the same offsets for small tiles
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t l = 8u * j + ((uint32_t)lane >> 3);
        const uint32_t k = ((uint32_t)lane & 7u) ^ ((l >> 1) & 7u);
        voff2[j] = l * (uint32_t)SEG2 + k * 16u;
    }
    const uint32_t rd_base = (uint32_t)lane * 128u;
    const uint32_t rsw = ((uint32_t)lane >> 1) & 7u;

    constexpr int NIT = SEG / kIter + 1;  // iteration 0 is the warm-up block [-128, 0)
    const uint64_t nw = (uint64_t)gridDim.x * NW;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave;
#ifdef PBS_SCAN_PROBE
    if (lane == 0 && blockIdx.x * NW + wave < kScanProbeMax)
        g_scan_probe[kScanProbeMax + blockIdx.x * NW + wave] = wall_clock64();
#endif
    if (tile >= ntiles) return;

    // Tile t > 0: base = tile start - 128, iteration offset it*128 (the warm-up block of
    // segment 0 is the previous tile's last line).  Tile 0: base = tile start; its
    // warm-up iteration (it == 0) uses explicit per-lane offsets voff - 128 (segment 0
    // has no bytes before it: it reads offset 0 and its warm-up state is discarded).
    // Offsets must not wrap: the buffer unit range-checks voffset + soffset unwrapped.
    // byte offset of tile t and whether it is a small one (wave-uniform)
    auto tile_off = [&](uint64_t t) -> uint64_t {
        if (DYN != 0 && t >= t_big) return t_big * (64ull * SEG) + (t - t_big) * (64ull * SEG2);
        return t * (64ull * SEG);
    };
    auto issue = [&](uint64_t t, int it) {
        const bool sm = DYN != 0 && t >= t_big;
        const uint8_t* tb = data + tile_off(t);
        const bool first = (t == 0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(first ? tb : tb - kIter), 0, (int)(64u * (sm ? SEG2 : SEG) + kIter), 0x00020000);
        const bool warm0 = first && it == 0;
        const uint32_t soff = warm0 ? 0u : (uint32_t)it * kIter - (first ? (uint32_t)kIter : 0u);
        if (sm) {  // small tiles are never tile 0
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, voff2[j], soff,
                    0, AUX);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t vo = warm0 ? (voff[j] >= (uint32_t)kIter ? voff[j] - kIter : 0u) : voff[j];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, vo, soff, 0,
                    AUX);
            }
        }
        if constexpr (PF > 0) {
            // pull the 64 lines of iteration it+PF into L2 (4 bytes per lane, dummy LDS)
            if (it + PF < NIT)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)touch_area, 4, voff_touch,
                    soff + (uint32_t)PF * kIter, 0, 0);
        }
    };

    uint32_t ring[128];
#pragma unroll
    for (int r = 0; r < 128; ++r) ring[r] = 0;
    uint32_t h = 0;
    bool canon = false;  // ZS: lane state is {h = 0, ring = T'[0]} (last block all zero)
    uint32_t dyn_v = 0;  // DYN: counter value drawn for the tile after this one
    auto next_tile = [&]() -> uint64_t {
        if constexpr (DYN != 0)
            return nw + (uint64_t)__builtin_amdgcn_readfirstlane(dyn_v);
        else
            return tile + nw;
    };
    issue(tile, 0);
    for (;;) {
        if constexpr (DYN != 0) {
            if (lane == 0) dyn_v = atomicAdd(tile_ctr, 1u);
        }
        const bool small = DYN != 0 && tile >= t_big;
        const int nit_cur = small ? SEG2 / kIter + 1 : NIT;
        const uint64_t toff = tile_off(tile);
        const uint32_t seg_cur = small ? (uint32_t)SEG2 : (uint32_t)SEG;
        for (int it = 0; it < nit_cur; ++it) {
            if (PF > 0 && it + PF < NIT)
                asm volatile("s_waitcnt vmcnt(1)" ::: "memory");  // the touch may stay in flight
            else
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
                if (__builtin_amdgcn_readfirstlane(pprog) > prog)
                    __builtin_amdgcn_s_setprio(2);
                else
                    __builtin_amdgcn_s_setprio(0);
                ++prog;
            }
            {
                uint64_t nt = tile;
                int nit = it + 1;
                if (nit == nit_cur) {
                    nt = next_tile();
                    nit = 0;
                }
                if (MODE != kModeComputeOnly && nt < ntiles) issue(nt, nit);
            }
            if (it == 0) {
                h = 0;
                canon = false;
#pragma unroll
                for (int r = 64; r < 128; ++r) ring[r] = 0;
            }
            bool zero = false;
            if constexpr (ZS != 0 && MODE != kModeLoadOnly) {
                uint32_t z = 0;
#pragma unroll
                for (int k = 0; k < 32; ++k) z |= d[k];
                zero = z == 0u;
            }
            uint32_t acc = 0;
            if constexpr (MODE == kModeLoadOnly) {
                acc = 0;
#pragma unroll
                for (int k = 0; k < 32; ++k) acc ^= d[k];
                acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;
            } else if (!(canon && zero)) {
                if constexpr (FR == 2 && G == 2)
                    acc = roll128_asm_f2_g2p12(d, ring, h, lb0, lb1);
                else if constexpr (FR == 2 && G == 3)
                    acc = roll128_asm_f2_g2p10(d, ring, h, lb0, lb1);
                else if constexpr (FR == 2)
                    acc = roll128_asm_f2(d, ring, h, lb0, lb1);
                else if constexpr (G == 4)
                    acc = roll128_asm_g4(d, ring, h, lanebase);
                else
                    acc = roll128_asm(d, ring, h, lanebase);
            }
            canon = zero;
            if (it == 0) {
                if (tile == 0 && lane == 0) {
                    canon = false;
                    h = 0;
#pragma unroll
                    for (int r = 64; r < 128; ++r) ring[r] = 0;
                }
            } else {
                const uint64_t pos =
                    toff + (uint64_t)lane * seg_cur + (uint64_t)(it - 1) * kIter;
                const bool hit = acc >= thr && pos != 0;
                const uint64_t m = __ballot(hit);
                if (m) {
                    const uint32_t pre =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (hit) s_susp[scnt + pre] = pos;
                    scnt += (uint32_t)__popcll(m);
                    if (scnt > (uint32_t)kSuspBuf - 64u) flush();
                }
            }
        }
        tile = next_tile();
        if (tile >= ntiles) break;
    }
    if (scnt) flush();
#ifdef PBS_SCAN_PROBE  // scripts/microbench/scan_probe.py: per-wave finish time
    if (lane == 0 && blockIdx.x * NW + wave < kScanProbeMax)
        g_scan_probe[blockIdx.x * NW + wave] = wall_clock64();
#endif
}

}  // namespace pbs
