// Compressed DataBlob images of every chunk on the GPU (second
// half): `DataBlob::encode(data, None, compress = true)` (pbs-datastore/src/data_blob.rs:
// 139-176) -- a zstd frame of the chunk (`zstd::stream::copy_encode(data, .., 1)`, :151)
// behind the 12-byte header {COMPRESSED_BLOB_MAGIC_1_0, CRC} when it is shorter than the
// chunk, else the uncompressed blob {UNCOMPRESSED_BLOB_MAGIC_1_0, CRC, bytes}; the CRC
// (`compute_crc`, :70-75) covers everything after the header.  C ABI: include/pbs_blob.h.
//
// The frame (zstd_enc.h) is built from independent 64 KiB zstd blocks, one workgroup per
// block (a 64 GiB stream is 1 M blocks), the block staged in LDS (16-byte loads of its
// aligned span; every byte and word read after that is LDS: 2 workgroups per CU):
//   1. RLE test (every byte equal: a 4-byte RLE block -- the zero pages of a VM image);
//   2. each wave parses its own 16 KiB sub-block with its own 512-entry LDS table, in
//      rounds of 256 sampled positions (4 per lane; every step-th byte: step 1 after a
//      round with a match, doubling to 8 while rounds find none): hash of the 4 bytes at
//      p -> candidate = the last sampled position of an earlier round with that hash
//      (`ds_max` inserts after the round's lookups) or the run candidate p - 1, the
//      longer match winning; the 4-byte compares and all LDS reads issued
//      unconditionally; matches capped at 32
//      and at the sub-block end; positions inside a chosen match skipped;
//   3. the wave's greedy parse over the round's match masks (ballots, registers): from
//      the current position the next matching position starts a sequence, a capped match
//      is extended 256 bytes per step (a word per lane, ballot of mismatches) -- no
//      workgroup barrier until the four waves' sequences are combined (literals carry
//      over sub-block ends);
//   4. wave 0 lane 0 writes the FSE-coded sequences (predefined tables) while waves 1-3
//      copy the literal runs; raw block if that is not shorter.
// Then per chunk: frame size, compressed-or-not (the reference's "only if shorter",
// :153), blob offsets by an exclusive scan, the blocks gathered into the blob images,
// and the blob CRC by the CRC kernel of pbs_blob.hip (12-byte header skipped).
//
// The parse is the host twin's (oracle/zstd_twin.cpp) step for step, so the bytes are
// compared exactly; libzstd decodes every frame back to the chunk (tests).  The bytes are
// not libzstd's level 1 (parity unpinned).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "pbs_blob.h"
#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"
#include "zstd_enc.h"

namespace pbs {
namespace {

using namespace zstd;

constexpr int kZThreads = 256;
constexpr uint32_t kZSub = 16384;                 // one wave's sub-block of a block
constexpr uint32_t kZRound = 256, kZHashLog = 9, kZCap = 32, kZMaxStep = 8;
constexpr int kZPer = kZRound / 64;              // positions per lane and round
constexpr uint32_t kSubSeq = kZSub / 4;          // sequences one sub-block can hold
constexpr uint32_t kWaveLdsSeq = 64;             // of them kept in LDS (the rest in global scratch)
constexpr uint64_t kSlot = kEncBlock + 128;  // block header + up to 64 KiB + slack for 8-byte flushes
constexpr uint32_t kMaxSeq = kEncBlock / 4;
constexpr uint32_t kStageWords = kEncBlock / 16 + 1;  // 16-byte words covering a block at any alignment
constexpr int kZGroupsPerCu = 2;                    // LDS: 77 KiB per workgroup

// pbs-datastore/src/file_formats.rs:9, :12
constexpr uint8_t kUncompressedMagic[8] = {66, 171, 56, 7, 190, 131, 112, 161};
constexpr uint8_t kCompressedMagic[8] = {49, 185, 88, 66, 111, 182, 163, 127};

struct ZTables {
    FseCTable ll, ml, of;
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));


// The block staged in LDS: 16-byte words of the aligned span around it; block byte i is
// LDS byte i + r (r = the block's address & 15).
struct Stage {
    const uint32_t* w;  // LDS words
    uint32_t r;
    __device__ __forceinline__ uint32_t byte(uint32_t i) const {
        return reinterpret_cast<const uint8_t*>(w)[i + r];
    }
    // little-endian 4 bytes at block position i (i + 3 inside the staged span)
    __device__ __forceinline__ uint32_t word(uint32_t i) const {
        const uint32_t o = i + r;
        return __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], o & 3);
    }
};

// Common prefix of the block at positions c < p, at most lim bytes: word compares, the
// first differing byte from the lowest set bit of the XOR.
__device__ __forceinline__ uint32_t common_prefix(const Stage& s, uint32_t c, uint32_t p, uint32_t lim) {
    uint32_t L = 0;
    while (L + 4 <= lim) {
        const uint32_t x = s.word(c + L) ^ s.word(p + L);
        if (x) return L + ((uint32_t)__builtin_ctz(x) >> 3);
        L += 4;
    }
    while (L < lim && s.byte(c + L) == s.byte(p + L)) ++L;
    return L;
}

// cnt bytes of the staged block from position `from` to global dst: head bytes up to a
// 4-aligned dst, then dword stores (one LDS word read each), then the tail; threads t of nt.
__device__ __forceinline__ void copy_from_stage(uint8_t* dst, const Stage& S, uint32_t from, uint32_t cnt,
                                                uint32_t t, uint32_t nt) {
    uint32_t head = (uint32_t)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);
    if (head > cnt) head = cnt;
    if (t < head) dst[t] = (uint8_t)S.byte(from + t);
    const uint32_t nwd = (cnt - head) >> 2;
    uint32_t* const dw = reinterpret_cast<uint32_t*>(dst + head);
    for (uint32_t w = t; w < nwd; w += nt) dw[w] = S.word(from + head + 4 * w);
    for (uint32_t i = head + 4 * nwd + t; i < cnt; i += nt) dst[i] = (uint8_t)S.byte(from + i);
}

// n bytes global -> global at any alignments: 16-byte stores at 16-aligned dst, each built
// from the five aligned source dwords around it (v_alignbyte; never a page past a source
// byte), head and tail bytewise.
__device__ __forceinline__ void copy_global(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t t,
                                            uint32_t nt) {
    uint64_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    if (head > n) head = n;
    if (t < head) dst[t] = src[t];
    const uint8_t* const s2 = src + head;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(s2) & 3);
    const uint32_t* const sa = reinterpret_cast<const uint32_t*>(s2 - sh);
    const uint64_t nq = (n - head) >> 4;
    uint4* const dq = reinterpret_cast<uint4*>(dst + head);
    for (uint64_t q = t; q < nq; q += nt) {
        const uint32_t* const w = sa + 4 * q;
        uint4 v;
        if (sh) {
            const uint32_t a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
            v = make_uint4(__builtin_amdgcn_alignbyte(b, a, sh), __builtin_amdgcn_alignbyte(c, b, sh),
                           __builtin_amdgcn_alignbyte(d, c, sh), __builtin_amdgcn_alignbyte(e, d, sh));
        } else {
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        dq[q] = v;
    }
    for (uint64_t i = head + 16 * nq + t; i < n; i += nt) dst[i] = src[i];
}

// PBS_ZSTD_PROBE=1 (diagnostics): workgroup 0 adds wall-clock ticks (100 MHz) per phase
// into g_zprobe: 0 stage, 1 RLE test, 2 wave 0's sub-block (lookups, matches, parse), 3
// combine (barrier included), 4 encode + literal copy, 5 raw copy, 6 items, 7 sequences.
__device__ unsigned long long g_zprobe[8];

template <bool PROBE>
__global__ __launch_bounds__(kZThreads) void zstd_block_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint64_t* __restrict__ items, uint64_t nitems, const ZTables* __restrict__ zt,
    uint8_t* __restrict__ slots, uint64_t* __restrict__ sizes, Seq* __restrict__ seq_scratch,
    Seq* __restrict__ seq_out_scratch) {
    __shared__ uint4 blk[kStageWords + 1];
    __shared__ uint32_t table[kZThreads / 64][1u << kZHashLog];  // one per wave
    __shared__ uint32_t s_wave[kZThreads / 64][3];               // per wave: sequences, matched bytes, end
    __shared__ Seq s_wseq[kZThreads / 64][kWaveLdsSeq];            // each wave's first sequences
    __shared__ ZTables s_zt;
    __shared__ uint32_t s_u[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t i = tid; i < sizeof(ZTables) / 4; i += kZThreads)
        reinterpret_cast<uint32_t*>(&s_zt)[i] = reinterpret_cast<const uint32_t*>(zt)[i];
    Seq* const wseq = seq_scratch + (uint64_t)blockIdx.x * kMaxSeq + (uint64_t)wave * kSubSeq;  // positions
    Seq* const gseq = seq_out_scratch + (uint64_t)blockIdx.x * kMaxSeq;

    const bool probe = PROBE && blockIdx.x == 0 && tid == 0;
    uint64_t tp = probe ? wall_clock64() : 0;
    auto mark = [&](int ph) {
        if (probe) {
            const uint64_t t = wall_clock64();
            g_zprobe[ph] += t - tp;
            tp = t;
        }
    };
    // the next item's metadata loads while this one is compressed
    uint64_t it_n = blockIdx.x < nitems ? items[blockIdx.x] : 0;
    uint64_t b0_n = blockIdx.x < nitems ? bounds[it_n >> 32] : 0, b1_n = blockIdx.x < nitems ? bounds[(it_n >> 32) + 1] : 0;
    for (uint64_t k = blockIdx.x; k < nitems; k += gridDim.x) {
        __syncthreads();  // LDS of the previous item
        const uint64_t it = it_n, bb0 = b0_n, bb1 = b1_n;
        if (k + gridDim.x < nitems) {
            it_n = items[k + gridDim.x];
            b0_n = bounds[it_n >> 32];
            b1_n = bounds[(it_n >> 32) + 1];
        }
        if (probe) g_zprobe[6] += 1;
        const uint64_t ci = it >> 32, j = (uint32_t)it;
        (void)ci;
        const uint64_t len = bb1 - bb0, off = j * (uint64_t)kEncBlock;
        const uint32_t n = (uint32_t)(len > off ? (len - off < kEncBlock ? len - off : kEncBlock) : 0);
        const bool last = off + n == len;
        const uint8_t* const src = data + (bb0 - base) + off;
        uint8_t* const out = slots + k * kSlot;
        if (n == 0) {  // the empty chunk's frame: one empty raw block
            if (tid == 0) {
                write_block_header(out, true, 0, 0);
                sizes[k] = 3;
            }
            continue;
        }
        // stage: the aligned 16-byte words holding [src, src + n) (never past a page that
        // holds a block byte); all of a thread's loads in flight before the LDS stores
        const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 15);
        const uint8_t* const a0 = src - r;  // pointer arithmetic keeps the loads global (not flat)
        const uint32_t nw = (n + r + 15) >> 4;
        for (uint32_t i0 = tid; i0 < nw; i0 += 5 * kZThreads) {  // 5 loads in flight per thread
            v4u v[5];
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const uint32_t i = i0 + kZThreads * q;
                if (i < nw) v[q] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a0) + i);
            }
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                const uint32_t i = i0 + kZThreads * q;
                if (i < nw) blk[i] = make_uint4(v[q].x, v[q].y, v[q].z, v[q].w);
            }
        }
        if (tid == 0) blk[nw] = make_uint4(0, 0, 0, 0);  // word reads past the end stay defined
        __syncthreads();
        mark(0);
        const Stage S{reinterpret_cast<const uint32_t*>(blk), r};
        const uint32_t b0 = S.byte(0), b4 = b0 * 0x01010101u;
        int same = 1;
        for (uint32_t q = tid; q < nw; q += kZThreads) {  // staged word q = block bytes 16q - r ..
            if (16 * q >= r && 16 * q + 16 - r <= n) {
                const uint4 w = blk[q];
                same &= (w.x == b4) & (w.y == b4) & (w.z == b4) & (w.w == b4);
            } else {
                for (uint32_t i = 0; i < 16; ++i) {
                    const int64_t pos = (int64_t)(16 * q + i) - (int64_t)r;
                    if (pos >= 0 && pos < (int64_t)n) same &= S.byte((uint32_t)pos) == b0;
                }
            }
        }
        const int rle = __syncthreads_and(same);
        mark(1);
        if (rle) {
            if (tid == 0) {
                write_block_header(out, last, 1, n);
                out[3] = (uint8_t)b0;
                sizes[k] = 4;
            }
            continue;
        }
        // each wave parses its own 16 KiB sub-block with its own table: no workgroup
        // barrier until the sequences are combined (a shared 1024-position round needed two
        // per round and left the parse to one wave)
        const uint32_t s0 = (uint32_t)wave * kZSub;
        uint32_t ns = 0, msum = 0, cur = s0;  // wave-uniform
        if (s0 < n) {
            const uint32_t se = s0 + kZSub < n ? s0 + kZSub : n;
            uint32_t* const tw = table[wave];
#pragma unroll
            for (int i = 0; i < (1 << kZHashLog) / 64; ++i) tw[lane + 64 * i] = 0;
            const uint32_t plim = n >= 4 ? n - 4 : 0;
            uint32_t step = 1;  // positions sampled per round: 1 after a match, doubling to 8 without
            for (uint32_t r0 = s0, rn; r0 < se; r0 = rn) {
                rn = r0 + kZRound * step;  // the next round starts where this one's samples end
                // branch-free lookups: every LDS read issued at a clamped address, the value
                // selected after (conditional reads became a branch and a wait each)
                uint32_t h[kZPer], c1[kZPer], wp[kZPer], wm[kZPer];
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    const uint32_t p = r0 + (lane + 64 * i) * step;
                    const uint32_t pc = p < plim ? p : plim;
                    wp[i] = S.word(pc);
                    wm[i] = S.word(pc ? pc - 1 : 0);  // p - 1: the run candidate (lane 0)
                }
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    const uint32_t p = r0 + (lane + 64 * i) * step;
                    h[i] = (wp[i] * 2654435761u) >> (32 - kZHashLog);
                    const uint32_t t = tw[h[i]];
                    // an AND, not a select: a select let the compiler sink the read into a branch
                    c1[i] = t & (0u - (uint32_t)(p + 4 <= n && p < se && p >= cur));
                }
                uint32_t wc[kZPer], wr[kZPer];
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    wc[i] = S.word(c1[i] ? c1[i] - 1 : 0);
                    const uint32_t up = (uint32_t)__shfl_up((int)wp[i], 1, 64);
                    wr[i] = lane && step == 1 ? up : wm[i];
                }
                uint32_t Lm[kZPer], Cm[kZPer];
                unsigned long long m[kZPer];
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    const uint32_t p = r0 + (lane + 64 * i) * step;
                    const bool live = p + 4 <= n && p < se && p >= cur;
                    const bool mt = live && c1[i] && wc[i] == wp[i];
                    const bool mr = live && p > 0 && wr[i] == wp[i];
                    uint32_t L = 0, c = c1[i] - 1;
                    if (mt || mr) {  // rare: matches extended to the cap (within the sub-block);
                        // the run candidate p - 1 wins when longer (ties: the table's)
                        const uint32_t lim = se - p < kZCap ? se - p : kZCap;
                        if (lim >= 4) {
                            const uint32_t Lt = mt ? 4 + common_prefix(S, c + 4, p + 4, lim - 4) : 0;
                            const uint32_t Lr = mr ? 4 + common_prefix(S, p + 3, p + 4, lim - 4) : 0;
                            L = Lt;
                            if (Lr > Lt) {
                                L = Lr;
                                c = p - 1;
                            }
                        }
                    }
                    Lm[i] = L;
                    Cm[i] = c;
                    m[i] = __ballot(L != 0);
                }
                // this round's inserts, after every lookup of the round (program order)
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    const uint32_t p = r0 + (lane + 64 * i) * step;
                    atomicMax(&tw[h[i]], p + 4 <= n && p < se ? p + 1 : 0u);
                }
                // greedy parse of the round from the match masks (wave-uniform); bit q is
                // position r0 + q * step
                bool found = false;
                uint32_t q = cur > r0 ? (cur - r0 + step - 1) / step : 0;
                while (q < kZRound) {
                    uint32_t w = q >> 6;
                    unsigned long long mm = 0;
                    for (; w < (uint32_t)kZPer; ++w) {
                        mm = (w == 0 ? m[0] : w == 1 ? m[1] : w == 2 ? m[2] : m[3]) &
                             (w == (q >> 6) ? (~0ull << (q & 63)) : ~0ull);
                        if (mm) break;
                    }
                    if (!mm) break;
                    const int l = __builtin_ctzll(mm);
                    const uint32_t pp = r0 + (w * 64 + (uint32_t)l) * step;
                    const uint32_t Lw = w == 0 ? Lm[0] : w == 1 ? Lm[1] : w == 2 ? Lm[2] : Lm[3];
                    const uint32_t Cw = w == 0 ? Cm[0] : w == 1 ? Cm[1] : w == 2 ? Cm[2] : Cm[3];
                    uint32_t ml = (uint32_t)__builtin_amdgcn_readlane((int)Lw, l);
                    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)Cw, l);
                    if (ml == kZCap) {  // extend to the sub-block end: a word per lane, 256 bytes a step
                        for (;;) {
                            const uint32_t x = pp + ml + 4 * lane;
                            uint32_t mis = 4;  // first mismatching byte of my 4 (4: none)
                            if (x + 4 <= se) {
                                const uint32_t d = S.word(c + ml + 4 * lane) ^ S.word(x);
                                if (d) mis = (uint32_t)__builtin_ctz(d) >> 3;
                            } else {
                                mis = 0;
                                while (x + mis < se && S.byte(c + ml + 4 * lane + mis) == S.byte(x + mis)) ++mis;
                                if (x >= se) mis = 0;
                            }
                            const unsigned long long bad = __ballot(mis < 4 || x + 4 > se);
                            if (bad) {
                                const int f = __builtin_ctzll(bad);
                                ml += 4 * (uint32_t)f + (uint32_t)__builtin_amdgcn_readlane((int)mis, f);
                                break;
                            }
                            ml += 256;
                        }
                    }
                    if (lane == 0) {  // position form: ll comes later
                        if (ns < kWaveLdsSeq)
                            s_wseq[wave][ns] = Seq{pp, ml, pp - c};
                        else
                            wseq[ns] = Seq{pp, ml, pp - c};
                    }
                    ++ns;
                    msum += ml;
                    cur = pp + ml;
                    q = (cur - r0 + step - 1) / step;
                    found = true;
                }
                step = found ? 1 : (2 * step < kZMaxStep ? 2 * step : kZMaxStep);
            }
        }
        if (lane == 0) {
            s_wave[wave][0] = ns;
            s_wave[wave][1] = msum;
            s_wave[wave][2] = cur;
        }
        mark(2);
        __syncthreads();
        // combine the waves' sequences: literal length = position - end of the previous
        // match (across sub-blocks: literals carry over), into LDS (the tables are free) or,
        // when they do not fit, a contiguous global list
        static_assert(kZThreads / 64 == 4, "four sub-blocks per block");
        const uint32_t b1 = s_wave[0][0], b2 = b1 + s_wave[1][0], b3 = b2 + s_wave[2][0];
        const uint32_t matched = s_wave[0][1] + s_wave[1][1] + s_wave[2][1] + s_wave[3][1];
        ns = b3 + s_wave[3][0];
        if (probe) g_zprobe[7] += ns;
        constexpr uint32_t kLdsSeq = sizeof(table) / sizeof(Seq);
        Seq* const sq = ns <= kLdsSeq ? reinterpret_cast<Seq*>(&table[0][0]) : gseq;
        const Seq* const pos0 = seq_scratch + (uint64_t)blockIdx.x * kMaxSeq;
        auto at = [&](uint32_t q) -> Seq {  // q-th sequence (position form), selects only
            const uint32_t w = (uint32_t)(q >= b1) + (uint32_t)(q >= b2) + (uint32_t)(q >= b3);
            const uint32_t b = w == 0 ? 0 : w == 1 ? b1 : w == 2 ? b2 : b3;
            const uint32_t j = q - b;
            return j < kWaveLdsSeq ? s_wseq[w][j] : pos0[(uint64_t)w * kSubSeq + j];
        };
        for (uint32_t q = tid; q < ns; q += kZThreads) {
            const Seq e = at(q);
            uint32_t prev_end = 0;
            if (q) {
                const Seq f = at(q - 1);
                prev_end = f.ll + f.ml;
            }
            sq[q] = Seq{e.ll - prev_end, e.ml, e.off};
        }
        uint32_t tail_start = 0;  // end of the last match
        for (int w = kZThreads / 64 - 1; w >= 0; --w)
            if (s_wave[w][0]) {
                tail_start = s_wave[w][2];
                break;
            }
        __syncthreads();
        mark(3);
        const uint32_t nlit = n - matched;
        const uint32_t lith = nlit < 32 ? 1 : nlit < 4096 ? 2 : 3;
        const uint32_t seq_at = 3 + lith + nlit;
        bool raw = seq_at - 3 >= n;
        if (!raw) {
            if (wave == 0) {
                if (lane == 0) {
                    const size_t sz = write_sequences(out + seq_at, sq, ns, s_zt.ll, s_zt.ml, s_zt.of,
                                                      out + 3 + n);
                    s_u[3] = sz == SIZE_MAX ? 0xFFFFFFFFu : (uint32_t)sz;
                }
            } else {  // waves 1-3: the literal runs in order (run ns: after the last match)
                uint8_t* const lo = out + 3 + lith;
                uint32_t from = 0, to = 0;
                for (uint32_t q = 0; q <= ns; ++q) {
                    uint32_t cnt;
                    if (q < ns) {
                        const Seq e = sq[q];
                        cnt = e.ll;
                        copy_from_stage(lo + to, S, from, cnt, tid - 64, kZThreads - 64);
                        from += cnt + e.ml;
                    } else {
                        cnt = n - tail_start;
                        copy_from_stage(lo + to, S, tail_start, cnt, tid - 64, kZThreads - 64);
                    }
                    to += cnt;
                }
            }
            __syncthreads();
            mark(4);
            const uint32_t sz = s_u[3];
            if (sz == 0xFFFFFFFFu || seq_at + sz - 3 >= n) {
                raw = true;
            } else if (tid == 0) {
                write_block_header(out, last, 2, seq_at + sz - 3);
                write_raw_literals_header(out + 3, nlit);
                sizes[k] = seq_at + sz;
            }
        }
        if (raw) {
            copy_from_stage(out + 3, S, 0, n, tid, kZThreads);
            if (tid == 0) {
                write_block_header(out, last, 0, n);
                sizes[k] = 3 + (uint64_t)n;
            }
        }
        if (PROBE) {
            __syncthreads();
            mark(5);
        }
    }
}

// Per chunk: frame size, compressed-or-not, blob size.  fsz[n] = 0 (scan padding).
__global__ void zstd_frame_sizes_kernel(const uint64_t* __restrict__ bounds, const uint64_t* __restrict__ first,
                                        const uint64_t* __restrict__ sizes, uint64_t n, int compress,
                                        uint64_t* __restrict__ bsz, uint8_t* __restrict__ comp) {
    const uint64_t ci = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ci > n) return;
    if (ci == n) {
        bsz[n] = 0;
        return;
    }
    const uint64_t len = bounds[ci + 1] - bounds[ci];
    bool c = false;
    uint64_t fs = 0;
    if (compress) {
        fs = frame_header_size(len);
        for (uint64_t k = first[ci]; k < first[ci + 1]; ++k) fs += sizes[k];
        c = fs < len;  // data_blob.rs:153: only if shorter
    }
    comp[ci] = c ? 1 : 0;
    bsz[ci] = 12 + (c ? fs : len);
}

// Per item: its part of the blob image.  Compressed chunk: the block (and, for the first
// block, the magic and the frame header); otherwise the item's 128 KiB of chunk bytes.
__global__ __launch_bounds__(kZThreads) void zstd_assemble_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint64_t* __restrict__ items, uint64_t nitems, const uint64_t* __restrict__ first,
    const uint8_t* __restrict__ slots, const uint64_t* __restrict__ sizes, const uint64_t* __restrict__ ipre,
    const uint64_t* __restrict__ boff, const uint8_t* __restrict__ comp, uint8_t* __restrict__ blobs) {
    for (uint64_t k = blockIdx.x; k < nitems; k += gridDim.x) {
        const uint64_t it = items[k];
        const uint64_t ci = it >> 32, j = (uint32_t)it;
        const uint64_t len = bounds[ci + 1] - bounds[ci];
        uint8_t* const blob = blobs + boff[ci];
        const bool c = comp[ci] != 0;
        const uint32_t fh = frame_header_size(len);
        if (j == 0 && threadIdx.x < 8) blob[threadIdx.x] = c ? kCompressedMagic[threadIdx.x] : kUncompressedMagic[threadIdx.x];
        if (c) {
            if (j == 0 && threadIdx.x == 0) write_frame_header(blob + 12, len);
            uint8_t* const dst = blob + 12 + fh + (ipre[k] - ipre[first[ci]]);
            copy_global(dst, slots + k * kSlot, sizes[k], threadIdx.x, kZThreads);
        } else {
            const uint64_t off = j * (uint64_t)kEncBlock;
            const uint64_t n = len > off ? (len - off < kEncBlock ? len - off : kEncBlock) : 0;
            const uint8_t* const src = data + (bounds[ci] - base) + off;
            copy_global(blob + 12 + off, src, n, threadIdx.x, kZThreads);
        }
    }
}

__global__ void blob_crc_header_kernel(const uint64_t* __restrict__ boff, const uint32_t* __restrict__ crc,
                                       uint64_t n, uint8_t* __restrict__ blobs) {
    const uint64_t ci = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ci >= n) return;
    uint8_t* const h = blobs + boff[ci] + 8;
    const uint32_t v = crc[ci];
    h[0] = (uint8_t)v;
    h[1] = (uint8_t)(v >> 8);
    h[2] = (uint8_t)(v >> 16);
    h[3] = (uint8_t)(v >> 24);
}

// Per-device scratch kept for the process: the block slots (~ the input size), the
// sequence lists of the resident workgroups and the FSE tables.
struct ZScratch {
    std::mutex mu;
    int dev = -1;
    uint8_t* slots = nullptr;
    size_t slots_cap = 0;
    Seq* seqs = nullptr;
    Seq* seqs_out = nullptr;  // the combined list when it does not fit in LDS
    size_t groups = 0;
    ZTables* zt = nullptr;
};
ZScratch& zscratch() {
    static ZScratch* z = new ZScratch;  // never destroyed (HIP may be torn down first at exit)
    return *z;
}

template <typename T>
bool grow(T** p, size_t* cap, size_t need) {
    if (*cap >= need) return true;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, need * sizeof(T)) != hipSuccess) return false;
    *cap = need;
    return true;
}

}  // namespace
}  // namespace pbs

using namespace pbs;

extern "C" size_t pbs_zstd_frame_bound(size_t len) { return (size_t)zstd::frame_bound(len); }

// Frees the blob encoder's cached device scratch (~ the bytes of the largest call).
extern "C" void pbs_blob_encode_release(void) {
    ZScratch& z = zscratch();
    std::lock_guard<std::mutex> lk(z.mu);
    if (z.dev >= 0) {
        DeviceGuard dg(z.dev);
        for (void* p : {(void*)z.slots, (void*)z.seqs, (void*)z.seqs_out, (void*)z.zt})
            if (p) (void)hipFree(p);
    }
    z.slots = nullptr;
    z.seqs = nullptr;
    z.seqs_out = nullptr;
    z.zt = nullptr;
    z.slots_cap = 0;
    z.groups = 0;
    z.dev = -1;
}

extern "C" size_t pbs_blob_stream_bound(const uint64_t* bounds, size_t n) {
    if (!bounds || n == 0) return 0;
    return 12 * n + (size_t)(bounds[n] - bounds[0]);
}

extern "C" int pbs_blob_encode_chunks_device(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                             const uint64_t* bounds, size_t n, int compress, uint8_t* blobs_dev,
                                             size_t blobs_cap, uint64_t* blob_offsets, uint32_t* crcs,
                                             uint8_t* compressed, pbs_blob_encode_timing* timing,
                                             void* hip_stream) {
    using Clock = std::chrono::steady_clock;
    const Clock::time_point t0 = Clock::now();
    if (timing) std::memset(timing, 0, sizeof(*timing));
    if (!blob_offsets) return PBS_ERR_INVALID;
    blob_offsets[0] = 0;
    if (n == 0) return PBS_OK;
    if (!bounds || !blobs_dev || (data_len && !dev_data) || n >= 0xFFFFFFFFull) return PBS_ERR_INVALID;
    for (size_t i = 0; i < n; ++i)
        if (bounds[i] > bounds[i + 1] || bounds[i] < base || bounds[i + 1] - base > data_len)
            return PBS_ERR_INVALID;
    // the reference refuses blobs over MAX_BLOB_SIZE (data_blob.rs:92, 128 MiB, :13)
    for (size_t i = 0; i < n; ++i)
        if (bounds[i + 1] - bounds[i] > (128ull << 20)) return PBS_ERR_INVALID;
    hipStream_t st = (hipStream_t)hip_stream;
    int dev = 0, ncu = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return PBS_ERR_NO_DEVICE;
    // every allocation of this call (and the cached scratch) lives on the stream's device
    DeviceGuard dg(dev);
    if (!dg.ok) return PBS_ERR_NO_DEVICE;

    // items: (chunk, 64 KiB block) pairs; an empty chunk is one item
    std::vector<uint64_t> items, first(n + 1);
    for (size_t i = 0; i < n; ++i) {
        first[i] = items.size();
        const uint64_t len = bounds[i + 1] - bounds[i];
        const uint64_t nb = len ? (len + zstd::kEncBlock - 1) / zstd::kEncBlock : 1;
        for (uint64_t j = 0; j < nb; ++j) items.push_back((uint64_t)i << 32 | j);
    }
    first[n] = items.size();
    const uint64_t ni = items.size();

    uint64_t *d_bounds = nullptr, *d_items = nullptr, *d_first = nullptr, *d_sizes = nullptr, *d_ipre = nullptr,
             *d_bsz = nullptr, *d_boff = nullptr;
    uint8_t* d_comp = nullptr;
    uint32_t* d_crc = nullptr;
    void* d_tmp = nullptr;
    hipEvent_t ev[4] = {};
    int rc = PBS_OK;
    auto fail = [&](int r) {
        if (rc == PBS_OK) rc = r;
        return false;
    };
    auto ok = [&](hipError_t e) { return e == hipSuccess || fail(PBS_ERR_HIP); };
    size_t t1b = 0, t2b = 0;
    (void)exclusive_sum_u64(nullptr, &t1b, nullptr, nullptr, (uint32_t)(n + 1), st);
    (void)exclusive_sum_u64(nullptr, &t2b, nullptr, nullptr, (uint32_t)(ni + 1), st);
    size_t tmpb = std::max(t1b, t2b);
    if (hipMalloc(&d_bounds, (n + 1) * 8) != hipSuccess || hipMalloc(&d_items, ni * 8) != hipSuccess ||
        hipMalloc(&d_first, (n + 1) * 8) != hipSuccess || hipMalloc(&d_sizes, (ni + 1) * 8) != hipSuccess ||
        hipMalloc(&d_ipre, (ni + 1) * 8) != hipSuccess || hipMalloc(&d_bsz, (n + 1) * 8) != hipSuccess ||
        hipMalloc(&d_boff, (n + 1) * 8) != hipSuccess || hipMalloc(&d_comp, n) != hipSuccess ||
        hipMalloc(&d_crc, n * 4) != hipSuccess || hipMalloc(&d_tmp, std::max<size_t>(tmpb, 256)) != hipSuccess)
        fail(PBS_ERR_NOMEM);
    for (auto& e : ev)
        if (rc == PBS_OK) ok(hipEventCreate(&e));
    ZScratch& zs = zscratch();
    std::lock_guard<std::mutex> lk(zs.mu);
    const unsigned grid = (unsigned)std::min<uint64_t>(ni, (uint64_t)ncu * kZGroupsPerCu);
    if (rc == PBS_OK && compress) {
        if (zs.dev != dev) {  // first use, or another device: free the old scratch there
            if (zs.dev >= 0) {
                DeviceGuard og(zs.dev);
                for (void* p : {(void*)zs.slots, (void*)zs.seqs, (void*)zs.seqs_out, (void*)zs.zt})
                    if (p) (void)hipFree(p);
            }
            zs.slots = nullptr;
            zs.slots_cap = 0;
            zs.seqs = nullptr;
            zs.seqs_out = nullptr;
            zs.groups = 0;
            zs.zt = nullptr;
            zs.dev = dev;
        }
        size_t seq_cap = zs.groups * kMaxSeq, run_cap = zs.groups * kMaxSeq;
        if (!grow(&zs.slots, &zs.slots_cap, ni * kSlot) || !grow(&zs.seqs, &seq_cap, (size_t)grid * kMaxSeq) ||
            !grow(&zs.seqs_out, &run_cap, (size_t)grid * kMaxSeq)) {
            fail(PBS_ERR_NOMEM);
        } else {
            zs.groups = std::max<size_t>(zs.groups, grid);
        }
        if (rc == PBS_OK && !zs.zt) {
            ZTables h;
            zstd::build_ctable(h.ll, zstd::kLLNorm, 36, zstd::kLLLog);
            zstd::build_ctable(h.ml, zstd::kMLNorm, 53, zstd::kMLLog);
            zstd::build_ctable(h.of, zstd::kOFNorm, 29, zstd::kOFLog);
            if (hipMalloc(&zs.zt, sizeof(ZTables)) != hipSuccess ||
                hipMemcpy(zs.zt, &h, sizeof(ZTables), hipMemcpyHostToDevice) != hipSuccess) {
                zs.zt = nullptr;
                fail(PBS_ERR_NOMEM);
            }
        }
    }
    if (rc == PBS_OK)
        ok(hipMemcpyAsync(d_bounds, bounds, (n + 1) * 8, hipMemcpyHostToDevice, st)) &&
            ok(hipMemcpyAsync(d_items, items.data(), ni * 8, hipMemcpyHostToDevice, st)) &&
            ok(hipMemcpyAsync(d_first, first.data(), (n + 1) * 8, hipMemcpyHostToDevice, st)) &&
            ok(hipMemsetAsync(d_sizes, 0, (ni + 1) * 8, st));
    if (rc == PBS_OK) {
        (void)hipGetLastError();
        ok(hipEventRecord(ev[0], st));
        static const bool probe = [] {
            const char* e = std::getenv("PBS_ZSTD_PROBE");
            return e && e[0] == '1';
        }();
        if (compress && probe) {
            const unsigned long long z[8] = {};
            (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_zprobe), z, sizeof z, 0, hipMemcpyHostToDevice, st);
            hipLaunchKernelGGL(zstd_block_kernel<true>, dim3(grid), dim3(kZThreads), 0, st, dev_data, base, d_bounds,
                               d_items, ni, zs.zt, zs.slots, d_sizes, zs.seqs, zs.seqs_out);
            unsigned long long h[8] = {};
            (void)hipMemcpyFromSymbolAsync(h, HIP_SYMBOL(g_zprobe), sizeof h, 0, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            std::fprintf(stderr,
                         "zstd probe (workgroup 0, us): stage %.1f rle %.1f sub-block %.1f combine %.1f encode+lits %.1f "
                         "raw %.1f | items %llu seqs %llu\n",
                         h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0, h[4] / 100.0, h[5] / 100.0, h[6], h[7]);
        } else if (compress) {
            hipLaunchKernelGGL(zstd_block_kernel<false>, dim3(grid), dim3(kZThreads), 0, st, dev_data, base, d_bounds,
                               d_items, ni, zs.zt, zs.slots, d_sizes, zs.seqs, zs.seqs_out);
        }
        hipLaunchKernelGGL(zstd_frame_sizes_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st,
                           d_bounds, d_first, d_sizes, (uint64_t)n, compress, d_bsz, d_comp);
        ok(hipGetLastError()) && ok(exclusive_sum_u64(d_tmp, &tmpb, d_bsz, d_boff,
                                                      (uint32_t)(n + 1), st)) &&
            (!compress ||
             ok(exclusive_sum_u64(d_tmp, &tmpb, d_sizes, d_ipre, (uint32_t)(ni + 1), st))) &&
            ok(hipEventRecord(ev[1], st)) &&
            ok(hipMemcpyAsync(blob_offsets, d_boff, (n + 1) * 8, hipMemcpyDeviceToHost, st)) &&
            ok(hipStreamSynchronize(st));
    }
    if (rc == PBS_OK && blob_offsets[n] > blobs_cap) fail(PBS_ERR_CAPACITY);
    if (rc == PBS_OK) {
        hipLaunchKernelGGL(zstd_assemble_kernel, dim3((unsigned)std::min<uint64_t>(ni, (uint64_t)ncu * 8)),
                           dim3(kZThreads), 0, st, dev_data, base, d_bounds, d_items, ni, d_first, zs.slots,
                           d_sizes, d_ipre, d_boff, d_comp, blobs_dev);
        ok(hipGetLastError()) && ok(hipEventRecord(ev[2], st));
    }
    if (rc == PBS_OK) {
        const hipError_t e = launch_crc32_skip(blobs_dev, d_boff, n, 12, d_crc, st);
        if (e != hipSuccess) fail(e == hipErrorOutOfMemory ? PBS_ERR_NOMEM : PBS_ERR_HIP);
    }
    if (rc == PBS_OK) {
        hipLaunchKernelGGL(blob_crc_header_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_boff,
                           d_crc, (uint64_t)n, blobs_dev);
        ok(hipGetLastError()) && ok(hipEventRecord(ev[3], st)) &&
            (!crcs || ok(hipMemcpyAsync(crcs, d_crc, n * 4, hipMemcpyDeviceToHost, st))) &&
            (!compressed || ok(hipMemcpyAsync(compressed, d_comp, n, hipMemcpyDeviceToHost, st))) &&
            ok(hipStreamSynchronize(st));
    }
    if (rc == PBS_OK && timing) {
        float a = 0, b = 0, c = 0;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&b, ev[1], ev[2]);
        (void)hipEventElapsedTime(&c, ev[2], ev[3]);
        timing->compress_ms = a;
        timing->assemble_ms = b;
        timing->crc_ms = c;
        timing->bytes_in = bounds[n] - bounds[0];
        timing->bytes_out = blob_offsets[n];
        timing->blocks = ni;
        if (compressed)
            for (size_t i = 0; i < n; ++i) timing->compressed_chunks += compressed[i];
    }
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    for (void* p : {(void*)d_bounds, (void*)d_items, (void*)d_first, (void*)d_sizes, (void*)d_ipre, (void*)d_bsz,
                    (void*)d_boff, (void*)d_comp, (void*)d_crc, d_tmp})
        if (p) (void)hipFree(p);
    if (timing) timing->total_ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    return rc;
}
