// Rejected/experimental variants of scan_main_kernel, kept for the microbenchmarks
// (scripts/microbench/mb_scan.hip); results in DESIGN.md "Kernel: scan_main".
//   v1  C++ or asm roll, LDS-DMA via flat global_load_lds (VALU address math)
//   v2  12 waves, 64-byte iterations, 2 x 4 KiB stages (half-line DMA: bad with nt)
//   v4  register-staged nt loads, 2 iterations in flight (loads 7.1 TB/s, compute slower)
//   v5  per-lane loads straight into VGPRs (uncoalesced; very bad with nt)
#pragma once
#include "scan_main.h"

namespace pbs {

// One 128-byte step of the rolling hash for this lane.  `ring` holds T' of the last
// 64 bytes (the "leave" values); the unrolled body indexes it statically, so it lives
// in 64 VGPRs.  Returns the max of h' over the 128 positions.
__device__ __forceinline__ uint32_t roll128(const uint4 (&d)[8], uint32_t (&ring)[64],
                                            uint32_t& h, const uint32_t* s_tab,
                                            uint32_t lanebase) {
    uint32_t acc = 0, hp = 0;
#pragma unroll
    for (int i = 0; i < 128; ++i) {
        const uint4 q = d[i >> 4];
        const int wi = (i >> 2) & 3;
        const uint32_t w = wi == 0 ? q.x : (wi == 1 ? q.y : (wi == 2 ? q.z : q.w));
        // bytes of {w, lanebase}: result = [0, 0, byte (i&3) of w, lane*4]
        const uint32_t sel = 0x0c0c0000u | ((4u + (uint32_t)(i & 3)) << 8);
        const uint32_t a = __builtin_amdgcn_perm(w, lanebase, sel);
        const uint32_t t = *(const uint32_t*)((const char*)s_tab + a);
        h = __builtin_amdgcn_bitop3_b32(rotl1(h), ring[i & 63], t, 0x96);  // v_bitop3 xor3
        ring[i & 63] = t;
        if (i & 1)
            acc = umax3(acc, hp, h);
        else
            hp = h;
    }
    return acc;
}

template <int SEG, int NWAVES = kWavesPerWG, int MODE = kModeFull, bool ASM = true, int AUX = 0>
__global__ __launch_bounds__(NWAVES * 64) void scan_main_v1(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, uint32_t* __restrict__ nsusp, uint32_t cap) {
    static_assert(SEG % kIter == 0, "segment must be a multiple of the iteration size");
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords + NWAVES * kStagePerWave / 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    uint32_t* s_tab = s_lds;
    for (int i = tid; i < kTableDwords; i += NWAVES * 64) s_tab[i] = table_rot[i >> 6];
    __syncthreads();

    uint8_t* stage = (uint8_t*)(s_lds + kTableDwords) + wave * kStagePerWave;
    const uint32_t lanebase = (uint32_t)lane * 4u;

    // LDS-DMA instruction j, lane i stages chunk k of segment l = 8j + (i>>3) with
    // k = (i & 7) ^ ((l >> 1) & 7), so the linear LDS destination j*1024 + i*16 equals
    // the swizzled slot l*128 + ((k ^ ((l>>1)&7)) * 16).
    uint32_t dma_off[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t l = 8u * j + ((uint32_t)lane >> 3);
        const uint32_t k = ((uint32_t)lane & 7u) ^ ((l >> 1) & 7u);
        dma_off[j] = l * (uint32_t)SEG + k * 16u;
    }
    const uint32_t rd_base = (uint32_t)lane * 128u;
    const uint32_t rsw = ((uint32_t)lane >> 1) & 7u;

    constexpr int NIT = SEG / kIter + 1;  // iteration 0 is the warm-up block [-128, 0)
    const uint64_t nw = (uint64_t)gridDim.x * NWAVES;
    uint64_t tile = (uint64_t)blockIdx.x * NWAVES + wave;
    if (tile >= ntiles) return;

    auto issue = [&](uint64_t t, int it) {
        const uint8_t* tb = data + t * (64ull * SEG);
        const int32_t boff = (it - 1) * kIter;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int32_t off = (int32_t)dma_off[j] + boff;
            // Only segment 0 of the stream has no bytes before it: read any valid
            // bytes there, its warm-up state is discarded below.
            if (t == 0 && off < 0) off = 0;
            __builtin_amdgcn_global_load_lds(
                (const void __attribute__((address_space(1)))*)(tb + off),
                (void __attribute__((address_space(3)))*)(stage + j * 1024), 16, 0, AUX);
        }
    };

    // ASM: 128-entry ring (T' of the previous 128 bytes, leave = R[(i+64)%128]);
    // C++: 64-entry ring.  Either way the ring lives in VGPRs (static indexing).
    constexpr int RING = ASM ? 128 : 64;
    uint32_t ring[RING];
    uint32_t h = 0;
#pragma unroll
    for (int r = 0; r < RING; ++r) ring[r] = 0;
    issue(tile, 0);
    for (;;) {
        for (int it = 0; it < NIT; ++it) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint4 d[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                d[k] = *(const uint4*)(stage + rd_base + (((uint32_t)k ^ rsw) << 4));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // prefetch the next block of this wave (next iteration or next tile)
            {
                uint64_t nt = tile;
                int nit = it + 1;
                if (nit == NIT) {
                    nt = tile + nw;
                    nit = 0;
                }
                if (MODE != kModeComputeOnly && nt < ntiles) issue(nt, nit);
            }
            if (it == 0) {  // warm-up starts from the empty window (zero leave values)
                h = 0;
#pragma unroll
                for (int r = RING - 64; r < RING; ++r) ring[r] = 0;
            }
            uint32_t acc;
            if constexpr (MODE == kModeLoadOnly) {
                acc = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) acc ^= d[k].x ^ d[k].y ^ d[k].z ^ d[k].w;
                acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;  // keep loads live
            } else if constexpr (ASM) {
                uint32_t dw[32];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    dw[4 * k] = d[k].x;
                    dw[4 * k + 1] = d[k].y;
                    dw[4 * k + 2] = d[k].z;
                    dw[4 * k + 3] = d[k].w;
                }
                acc = roll128_asm(dw, ring, h, lanebase);
            } else {
                acc = roll128(d, *reinterpret_cast<uint32_t(*)[64]>(ring), h, s_tab, lanebase);
            }
            if (it == 0) {
                if (tile == 0 && lane == 0) {  // stream segment 0: no warm-up bytes
                    h = 0;
#pragma unroll
                    for (int r = RING - 64; r < RING; ++r) ring[r] = 0;
                }
            } else if (acc >= thr) {
                const uint64_t pos =
                    (tile * 64ull + (uint64_t)lane) * (uint64_t)SEG + (uint64_t)(it - 1) * kIter;
                // block 0 is always re-evaluated by scan_exact_kernel (the `pre` bytes)
                if (pos != 0) {
                    const uint32_t idx = atomicAdd(nsusp, 1u);
                    if (idx < cap) susp[idx] = pos;
                }
            }
        }
        tile += nw;
        if (tile >= ntiles) break;
    }
}


// ---------------------------------------------------------------------------------
// v2: 12 waves per CU.  64-byte iterations, two 4 KiB LDS-DMA stages per wave (the
// DMA of iteration q+2 is issued as soon as iteration q's block is in VGPRs), and
// the 128-entry VGPR ring driven by the two generated 64-byte asm halves.
// LDS: table 64 KiB + NWAVES x 8 KiB staging (160 KiB at 12 waves).
// Stage layout: chunk k (16 B) of lane l's 64-byte block at l*64 + ((k ^ ((l>>2)&3))*16)
// (conflict-free ds_read_b128); DMA instruction j, lane i stages segment
// l = 16j + (i>>2), chunk k = (i&3) ^ ((l>>2)&3).
constexpr int kIter2 = 64;
constexpr int kStage2 = 64 * kIter2;  // 4 KiB per stage

template <int SEG, int NWAVES = 12, int MODE = kModeFull, int AUX = 2>
__global__ __launch_bounds__(NWAVES * 64) void scan_main_v2(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, uint32_t* __restrict__ nsusp, uint32_t cap) {
    static_assert(SEG % (2 * kIter2) == 0, "segment must be a multiple of 128 bytes");
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords + NWAVES * 2 * kStage2 / 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTableDwords; i += NWAVES * 64) s_lds[i] = table_rot[i >> 6];
    __syncthreads();

    uint8_t* stage0 = (uint8_t*)(s_lds + kTableDwords) + wave * 2 * kStage2;
    const uint32_t lanebase = (uint32_t)lane * 4u;
    uint32_t dma_off[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t l = 16u * j + ((uint32_t)lane >> 2);
        const uint32_t k = ((uint32_t)lane & 3u) ^ ((l >> 2) & 3u);
        dma_off[j] = l * (uint32_t)SEG + k * 16u;
    }
    const uint32_t rd_off = (uint32_t)lane * 64u;
    const uint32_t rsw = ((uint32_t)lane >> 2) & 3u;

    constexpr int NIT = SEG / kIter2 + 1;  // iteration 0 is the warm-up block [-64, 0)
    const uint64_t nw = (uint64_t)gridDim.x * NWAVES;
    // the step window (tile, it) of steps q, q+1, q+2 -- wave-uniform (SGPRs)
    uint64_t tile = (uint64_t)blockIdx.x * NWAVES + wave;
    if (tile >= ntiles) return;
    int it = 0;
    uint64_t t1 = tile, t2;
    int it1 = 1, it2;
    if (it1 == NIT) { it1 = 0; t1 += nw; }
    t2 = t1; it2 = it1 + 1;
    if (it2 == NIT) { it2 = 0; t2 += nw; }

    auto issue = [&](uint64_t t, int itx, int buf) {
        const uint8_t* tb = data + t * (64ull * SEG);
        const int32_t boff = (itx - 1) * kIter2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int32_t off = (int32_t)dma_off[j] + boff;
            if (t == 0 && off < 0) off = 0;  // stream segment 0 has no warm-up bytes
            __builtin_amdgcn_global_load_lds(
                (const void __attribute__((address_space(1)))*)(tb + off),
                (void __attribute__((address_space(3)))*)(stage0 + buf * kStage2 + j * 1024), 16, 0,
                AUX);
        }
    };

    uint32_t ring[128];
#pragma unroll
    for (int r = 0; r < 128; ++r) ring[r] = 0;
    uint32_t h = 0;

    // One 64-byte step on ring half HV (= stage buffer HV); false when the wave is done.
    auto step = [&](auto hv_tag) -> bool {
        constexpr int HV = decltype(hv_tag)::value;
        if (MODE != kModeComputeOnly && t1 < ntiles)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // this step's DMA landed
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t d[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v =
                *(const uint4*)(stage0 + HV * kStage2 + rd_off + (((uint32_t)k ^ rsw) << 4));
            d[4 * k] = v.x;
            d[4 * k + 1] = v.y;
            d[4 * k + 2] = v.z;
            d[4 * k + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (MODE != kModeComputeOnly && t2 < ntiles) issue(t2, it2, HV);  // step q+2
        if (it == 0) {  // warm-up from the empty window: zero leave half, h = 0
            h = 0;
#pragma unroll
            for (int r = 0; r < 64; ++r) ring[64 * (1 - HV) + r] = 0;
        }
        uint32_t acc;
        if constexpr (MODE == kModeLoadOnly) {
            acc = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) acc ^= d[k];
            acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;
        } else if constexpr (HV == 0) {
            acc = roll64_asm_h0(d, ring, h, lanebase);
        } else {
            acc = roll64_asm_h1(d, ring, h, lanebase);
        }
        if (it == 0) {
            if (tile == 0 && lane == 0) {  // stream segment 0: no warm-up bytes
                h = 0;
#pragma unroll
                for (int r = 0; r < 64; ++r) ring[64 * HV + r] = 0;
            }
        } else if (acc >= thr) {
            const uint64_t pos =
                (tile * 64ull + (uint64_t)lane) * (uint64_t)SEG + (uint64_t)(it - 1) * kIter2;
            if (pos != 0) {  // block 0 is always re-evaluated by scan_exact_kernel
                const uint32_t idx = atomicAdd(nsusp, 1u);
                if (idx < cap) susp[idx] = pos;
            }
        }
        tile = t1;
        it = it1;
        t1 = t2;
        it1 = it2;
        if (++it2 == NIT) {
            it2 = 0;
            t2 += nw;
        }
        return tile < ntiles;
    };

    issue(tile, 0, 0);
    if (MODE != kModeComputeOnly && t1 < ntiles) issue(t1, it1, 1);
    for (;;) {
        if (!step(std::integral_constant<int, 0>{})) break;
        if (!step(std::integral_constant<int, 1>{})) break;
    }
}

// ---------------------------------------------------------------------------------
// v4: register-staged loads, two iterations in flight per wave.  Each iteration the
// wave's 8 x 1 KiB pieces (8 segments x 128-byte lines each) arrive by
// buffer_load_dwordx4 (nt) into one of two 32-VGPR batches, are written to the wave's
// 8 KiB LDS stage (linear, conflict-free ds_write_b128) and read back transposed
// (each lane its own 128 bytes, swizzled ds_read_b128).  Loads for step q+2 are
// issued as soon as step q's batch is in LDS, so ~2 iterations hide HBM latency
// without a second LDS stage.
template <int SEG, int MODE = kModeFull, int AUX = 2, int G = 4>
__global__ __launch_bounds__(kWavesPerWG * 64) void scan_main_v4(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, uint32_t* __restrict__ nsusp, uint32_t cap) {
    static_assert(SEG % kIter == 0, "segment must be a multiple of the iteration size");
    constexpr int NW = kWavesPerWG;
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords + NW * kStagePerWave / 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTableDwords; i += NW * 64) s_lds[i] = table_rot[i >> 6];
    __syncthreads();

    uint8_t* stage = (uint8_t*)(s_lds + kTableDwords) + wave * kStagePerWave;
    const uint32_t lanebase = (uint32_t)lane * 4u;
    uint32_t voff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t l = 8u * j + ((uint32_t)lane >> 3);
        const uint32_t k = ((uint32_t)lane & 7u) ^ ((l >> 1) & 7u);
        voff[j] = l * (uint32_t)SEG + k * 16u;
    }
    const uint32_t wr_base = (uint32_t)lane * 16u;  // piece j lands at j*1024 + lane*16
    const uint32_t rd_base = (uint32_t)lane * 128u;
    const uint32_t rsw = ((uint32_t)lane >> 1) & 7u;

    constexpr int NIT = SEG / kIter + 1;
    const uint64_t nw = (uint64_t)gridDim.x * NW;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave;
    if (tile >= ntiles) return;
    int it = 0;
    uint64_t t1 = tile, t2;
    int it1 = 1, it2;
    if (it1 == NIT) { it1 = 0; t1 += nw; }
    t2 = t1; it2 = it1 + 1;
    if (it2 == NIT) { it2 = 0; t2 += nw; }

    typedef int v4i __attribute__((ext_vector_type(4)));
    auto load = [&](uint64_t t, int itx, v4i (&g)[8]) {
        const uint8_t* tb = data + t * (64ull * SEG);
        const bool first = (t == 0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(first ? tb : tb - kIter), 0, (int)(64u * SEG + kIter), 0x00020000);
        const uint32_t soff = (uint32_t)itx * kIter - (first ? (uint32_t)kIter : 0u);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff[j], soff, AUX);
    };

    uint32_t ring[128];
#pragma unroll
    for (int r = 0; r < 128; ++r) ring[r] = 0;
    uint32_t h = 0;
    v4i gA[8], gB[8];

    auto step = [&](v4i (&g)[8]) -> bool {
        // batch -> LDS stage (linear) -> own 128 bytes (swizzled)
#pragma unroll
        for (int j = 0; j < 8; ++j) *(v4i*)(stage + j * 1024 + wr_base) = g[j];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint32_t d[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint4 v = *(const uint4*)(stage + rd_base + (((uint32_t)k ^ rsw) << 4));
            d[4 * k] = v.x;
            d[4 * k + 1] = v.y;
            d[4 * k + 2] = v.z;
            d[4 * k + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (MODE != kModeComputeOnly && t2 < ntiles) load(t2, it2, g);  // step q+2
        if (it == 0) {
            h = 0;
#pragma unroll
            for (int r = 64; r < 128; ++r) ring[r] = 0;
        }
        uint32_t acc;
        if constexpr (MODE == kModeLoadOnly) {
            acc = 0;
#pragma unroll
            for (int k = 0; k < 32; ++k) acc ^= d[k];
            acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;
        } else if constexpr (G == 4) {
            acc = roll128_asm_g4(d, ring, h, lanebase);
        } else {
            acc = roll128_asm(d, ring, h, lanebase);
        }
        if (it == 0) {
            if (tile == 0 && lane == 0) {
                h = 0;
#pragma unroll
                for (int r = 64; r < 128; ++r) ring[r] = 0;
            }
        } else if (acc >= thr) {
            const uint64_t pos =
                (tile * 64ull + (uint64_t)lane) * (uint64_t)SEG + (uint64_t)(it - 1) * kIter;
            if (pos != 0) {
                const uint32_t idx = atomicAdd(nsusp, 1u);
                if (idx < cap) susp[idx] = pos;
            }
        }
        tile = t1;
        it = it1;
        t1 = t2;
        it1 = it2;
        if (++it2 == NIT) {
            it2 = 0;
            t2 += nw;
        }
        return tile < ntiles;
    };

    load(tile, 0, gA);
    if (t1 < ntiles) load(t1, it1, gB);
    else {
#pragma unroll
        for (int j = 0; j < 8; ++j) gB[j] = v4i{0, 0, 0, 0};
    }
    for (;;) {
        if (!step(gA)) break;
        if (!step(gB)) break;
    }
}

// ---------------------------------------------------------------------------------
// v6: v4 with the loads in inline asm and hand-counted vmcnt (the compiler drained
// both batches at the loop head in v4).  v4: register-staged loads, two iterations in flight per wave.  Each iteration the
// wave's 8 x 1 KiB pieces (8 segments x 128-byte lines each) arrive by
// buffer_load_dwordx4 (nt) into one of two 32-VGPR batches, are written to the wave's
// 8 KiB LDS stage (linear, conflict-free ds_write_b128) and read back transposed
// (each lane its own 128 bytes, swizzled ds_read_b128).  Loads for step q+2 are
// issued as soon as step q's batch is in LDS, so ~2 iterations hide HBM latency
// without a second LDS stage.
template <int SEG, int MODE = kModeFull, int AUX = 2, int G = 4>
__global__ __launch_bounds__(kWavesPerWG * 64) void scan_main_v6(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, uint32_t* __restrict__ nsusp, uint32_t cap) {
    static_assert(SEG % kIter == 0, "segment must be a multiple of the iteration size");
    constexpr int NW = kWavesPerWG;
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords + NW * kStagePerWave / 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTableDwords; i += NW * 64) s_lds[i] = table_rot[i >> 6];
    __syncthreads();

    uint8_t* stage = (uint8_t*)(s_lds + kTableDwords) + wave * kStagePerWave;
    const uint32_t lanebase = (uint32_t)lane * 4u;
    uint32_t voff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t l = 8u * j + ((uint32_t)lane >> 3);
        const uint32_t k = ((uint32_t)lane & 7u) ^ ((l >> 1) & 7u);
        voff[j] = l * (uint32_t)SEG + k * 16u;
    }
    const uint32_t wr_base = (uint32_t)lane * 16u;  // piece j lands at j*1024 + lane*16
    const uint32_t rd_base = (uint32_t)lane * 128u;
    const uint32_t rsw = ((uint32_t)lane >> 1) & 7u;

    constexpr int NIT = SEG / kIter + 1;
    const uint64_t nw = (uint64_t)gridDim.x * NW;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave;
    if (tile >= ntiles) return;
    int it = 0;
    uint64_t t1 = tile, t2;
    int it1 = 1, it2;
    if (it1 == NIT) { it1 = 0; t1 += nw; }
    t2 = t1; it2 = it1 + 1;
    if (it2 == NIT) { it2 = 0; t2 += nw; }

    typedef int v4i __attribute__((ext_vector_type(4)));
    auto load = [&](uint64_t t, int itx, v4i (&g)[8]) {
        const uint8_t* tb = data + t * (64ull * SEG);
        const bool first = (t == 0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(first ? tb : tb - kIter), 0, (int)(64u * SEG + kIter), 0x00020000);
        const uint32_t soff = (uint32_t)itx * kIter - (first ? (uint32_t)kIter : 0u);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen nt" : "=v"(g[j]) : "v"(voff[j]), "s"(rs), "s"(soff) : "memory");
    };

    uint32_t ring[128];
#pragma unroll
    for (int r = 0; r < 128; ++r) ring[r] = 0;
    uint32_t h = 0;
    v4i gA[8], gB[8];

    auto step = [&](v4i (&g)[8]) -> bool {
        // this step's batch landed; the next step's batch (8 loads) may stay in flight
        if (t1 < ntiles && MODE != kModeComputeOnly)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // batch -> LDS stage (linear) -> own 128 bytes (swizzled)
#pragma unroll
        for (int j = 0; j < 8; ++j) *(v4i*)(stage + j * 1024 + wr_base) = g[j];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint32_t d[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint4 v = *(const uint4*)(stage + rd_base + (((uint32_t)k ^ rsw) << 4));
            d[4 * k] = v.x;
            d[4 * k + 1] = v.y;
            d[4 * k + 2] = v.z;
            d[4 * k + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (MODE != kModeComputeOnly && t2 < ntiles) load(t2, it2, g);  // step q+2
        if (it == 0) {
            h = 0;
#pragma unroll
            for (int r = 64; r < 128; ++r) ring[r] = 0;
        }
        uint32_t acc;
        if constexpr (MODE == kModeLoadOnly) {
            acc = 0;
#pragma unroll
            for (int k = 0; k < 32; ++k) acc ^= d[k];
            acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;
        } else if constexpr (G == 4) {
            acc = roll128_asm_g4(d, ring, h, lanebase);
        } else {
            acc = roll128_asm(d, ring, h, lanebase);
        }
        if (it == 0) {
            if (tile == 0 && lane == 0) {
                h = 0;
#pragma unroll
                for (int r = 64; r < 128; ++r) ring[r] = 0;
            }
        } else if (acc >= thr) {
            const uint64_t pos =
                (tile * 64ull + (uint64_t)lane) * (uint64_t)SEG + (uint64_t)(it - 1) * kIter;
            if (pos != 0) {
                const uint32_t idx = atomicAdd(nsusp, 1u);
                if (idx < cap) susp[idx] = pos;
            }
        }
        tile = t1;
        it = it1;
        t1 = t2;
        it1 = it2;
        if (++it2 == NIT) {
            it2 = 0;
            t2 += nw;
        }
        return tile < ntiles;
    };

    load(tile, 0, gA);
    if (t1 < ntiles) load(t1, it1, gB);
    else {
#pragma unroll
        for (int j = 0; j < 8; ++j) gB[j] = v4i{0, 0, 0, 0};
    }
    for (;;) {
        if (!step(gA)) break;
        if (!step(gB)) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------
// v5 (experiment): every lane loads its own segment's 128 bytes straight into VGPRs
// (8 x buffer_load_dwordx4 at per-lane offset lane*SEG, 64 lines per instruction),
// two iterations in flight, no LDS staging.
template <int SEG, int MODE = kModeFull, int AUX = 2>
__global__ __launch_bounds__(kWavesPerWG * 64) void scan_main_v5(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, uint32_t* __restrict__ nsusp, uint32_t cap) {
    constexpr int NW = kWavesPerWG;
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTableDwords; i += NW * 64) s_lds[i] = table_rot[i >> 6];
    __syncthreads();
    const uint32_t lanebase = (uint32_t)lane * 4u;
    const uint32_t voff = (uint32_t)lane * (uint32_t)SEG;
    constexpr int NIT = SEG / kIter + 1;
    const uint64_t nw = (uint64_t)gridDim.x * NW;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave;
    if (tile >= ntiles) return;
    int it = 0;
    uint64_t t1 = tile, t2;
    int it1 = 1, it2;
    if (it1 == NIT) { it1 = 0; t1 += nw; }
    t2 = t1; it2 = it1 + 1;
    if (it2 == NIT) { it2 = 0; t2 += nw; }
    typedef int v4i __attribute__((ext_vector_type(4)));
    auto load = [&](uint64_t t, int itx, v4i (&g)[8]) {
        const uint8_t* tb = data + t * (64ull * SEG);
        const bool first = (t == 0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(first ? tb : tb - kIter), 0, (int)(64u * SEG + kIter), 0x00020000);
        const uint32_t soff = (uint32_t)itx * kIter - (first ? (uint32_t)kIter : 0u);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u * j, soff, AUX);
    };
    uint32_t ring[128];
#pragma unroll
    for (int r = 0; r < 128; ++r) ring[r] = 0;
    uint32_t h = 0;
    v4i gA[8], gB[8];
    auto step = [&](v4i (&g)[8]) -> bool {
        uint32_t d[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            d[4 * k] = g[k].x;
            d[4 * k + 1] = g[k].y;
            d[4 * k + 2] = g[k].z;
            d[4 * k + 3] = g[k].w;
        }
        uint32_t acc;
        if constexpr (MODE == kModeLoadOnly) {
            acc = 0;
#pragma unroll
            for (int k = 0; k < 32; ++k) acc ^= d[k];
            acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;
        } else {
            if (it == 0) {
                h = 0;
#pragma unroll
                for (int r = 64; r < 128; ++r) ring[r] = 0;
            }
            acc = roll128_asm_g4(d, ring, h, lanebase);
        }
        if (MODE != kModeComputeOnly && t2 < ntiles) load(t2, it2, g);
        if (it == 0) {
            if (tile == 0 && lane == 0) {
                h = 0;
#pragma unroll
                for (int r = 64; r < 128; ++r) ring[r] = 0;
            }
        } else if (acc >= thr) {
            const uint64_t pos =
                (tile * 64ull + (uint64_t)lane) * (uint64_t)SEG + (uint64_t)(it - 1) * kIter;
            if (pos != 0) {
                const uint32_t idx = atomicAdd(nsusp, 1u);
                if (idx < cap) susp[idx] = pos;
            }
        }
        tile = t1; it = it1; t1 = t2; it1 = it2;
        if (++it2 == NIT) { it2 = 0; t2 += nw; }
        return tile < ntiles;
    };
    load(tile, 0, gA);
    if (t1 < ntiles) load(t1, it1, gB);
    else {
#pragma unroll
        for (int j = 0; j < 8; ++j) gB[j] = v4i{0, 0, 0, 0};
    }
    for (;;) {
        if (!step(gA)) break;
        if (!step(gB)) break;
    }
}

// ---------------------------------------------------------------------------------
// R96 (measured slower, profiles/r01/fr2/mb_r96_*.log): 12 waves per CU (3 per SIMD), parity frame, 96-register ring.  The ring only
// has to hold the 64 leave values plus the reads in flight, so 96 slots suffice; the
// slot pattern then repeats every three 128-byte iterations (roll128_r96_p0..2).  That
// frees the VGPRs for a third wave per SIMD (<= 168), and the LDS holds the 64 KiB
// parity-frame table + 12 x 8 KiB stages = 160 KiB.  DMA offsets use one VGPR per
// swizzle parity + SGPR soffsets (8j*SEG per instruction).
constexpr int kR96Waves = 12;
template <int SEG, int MODE = kModeFull, int AUX = 2>
__global__ __launch_bounds__(kR96Waves * 64) void scan_main_r96(
    const uint8_t* __restrict__ data, uint64_t ntiles, const uint32_t* __restrict__ table_rot,
    uint32_t thr, uint64_t* __restrict__ susp, uint32_t* __restrict__ nsusp, uint32_t cap) {
    static_assert(SEG % kIter == 0, "segment must be a multiple of the iteration size");
    constexpr int NW = kR96Waves;
    __shared__ __attribute__((aligned(16))) uint32_t s_lds[kTableDwords + NW * kStagePerWave / 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kTableDwords; i += NW * 64)
        s_lds[i] = table_rot[((i >> 5) & 1) * 256 + (i >> 6)];
    __syncthreads();

    uint8_t* stage = (uint8_t*)(s_lds + kTableDwords) + wave * kStagePerWave;
    const uint32_t lb0 = ((uint32_t)lane & 31u) * 4u, lb1 = lb0 + 128u;
    // DMA j (0..7) covers segments 8j .. 8j+7: lane L reads segment 8j + (L>>3), chunk
    // k = (L&7) ^ ((segment>>1)&7); (segment>>1)&7 = (4j + (L>>4)) & 7 depends on j's parity.
    const uint32_t lsub = (uint32_t)lane >> 3;
    const uint32_t voff_e = lsub * (uint32_t)SEG + ((((uint32_t)lane & 7u) ^ (((uint32_t)lane >> 4) & 7u)) << 4);
    const uint32_t voff_o = lsub * (uint32_t)SEG + ((((uint32_t)lane & 7u) ^ ((4u + ((uint32_t)lane >> 4)) & 7u)) << 4);
    const uint32_t rd_base = (uint32_t)lane * 128u;
    const uint32_t rsw = ((uint32_t)lane >> 1) & 7u;

    constexpr int NIT = SEG / kIter + 1;  // iteration 0 is the warm-up block [-128, 0)
    const uint64_t nw = (uint64_t)gridDim.x * NW;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave;
    if (tile >= ntiles) return;

    auto issue = [&](uint64_t t, int it) {
        const uint8_t* tb = data + t * (64ull * SEG);
        const bool first = (t == 0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(first ? tb : tb - kIter), 0, (int)(64u * SEG + kIter), 0x00020000);
        const bool warm0 = first && it == 0;
        const uint32_t soff = warm0 ? 0u : (uint32_t)it * kIter - (first ? (uint32_t)kIter : 0u);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t vo = (j & 1) ? voff_o : voff_e;
            uint32_t so = soff + (uint32_t)j * 8u * (uint32_t)SEG;
            if (warm0) {  // tile 0's warm-up: the 128 bytes before each segment (segment 0: none)
                if (j == 0) vo = vo >= (uint32_t)kIter ? vo - kIter : 0u;
                else so -= kIter;
            }
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(stage + j * 1024), 16, vo, so, 0, AUX);
        }
    };

    uint32_t ring[96];
#pragma unroll
    for (int r = 0; r < 96; ++r) ring[r] = 0;
    uint32_t h = 0;
    int it = 0;
    issue(tile, 0);
    // One step = one 128-byte iteration in ring phase PH; the three phases are emitted as
    // straight-line code so every ring slot keeps one register.
    auto step = [&](auto PHC) -> bool {
        constexpr int PH = decltype(PHC)::value;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t d[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint4 v = *(const uint4*)(stage + rd_base + (((uint32_t)k ^ rsw) << 4));
            d[4 * k] = v.x;
            d[4 * k + 1] = v.y;
            d[4 * k + 2] = v.z;
            d[4 * k + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint64_t nt = tile;
        int nit = it + 1;
        if (nit == NIT) {
            nt = tile + nw;
            nit = 0;
        }
        if (MODE != kModeComputeOnly && nt < ntiles) issue(nt, nit);
        if (it == 0) {  // warm-up block: no leave values for its first 64 bytes
            h = 0;
#pragma unroll
            for (int i = 0; i < 64; ++i) ring[(128 * PH + i + 32) % 96] = 0;
        }
        uint32_t acc = 0;
        if constexpr (MODE == kModeLoadOnly) {
#pragma unroll
            for (int k = 0; k < 32; ++k) acc ^= d[k];
            acc = (acc == 0x9E3779B9u && lane == 65) ? 0xFFFFFFFFu : 0u;
        } else if constexpr (PH == 0) {
            acc = roll128_r96_p0(d, ring, h, lb0, lb1);
        } else if constexpr (PH == 1) {
            acc = roll128_r96_p1(d, ring, h, lb0, lb1);
        } else {
            acc = roll128_r96_p2(d, ring, h, lb0, lb1);
        }
        if (it == 0) {
            if (tile == 0 && lane == 0) {  // stream segment 0: no bytes before it
                h = 0;
#pragma unroll
                for (int i = 0; i < 64; ++i) ring[(128 * (PH + 1) + i + 32) % 96] = 0;
            }
        } else if (acc >= thr) {
            const uint64_t pos =
                (tile * 64ull + (uint64_t)lane) * (uint64_t)SEG + (uint64_t)(it - 1) * kIter;
            if (pos != 0) {
                const uint32_t idx = atomicAdd(nsusp, 1u);
                if (idx < cap) susp[idx] = pos;
            }
        }
        tile = nt;
        it = nit;
        return tile < ntiles;
    };
    for (;;) {
        if (!step(std::integral_constant<int, 0>{})) break;
        if (!step(std::integral_constant<int, 1>{})) break;
        if (!step(std::integral_constant<int, 2>{})) break;
    }
}

}  // namespace pbs
