// HIP kernels of the MI355X (gfx950) content-defined chunker.
//
// Reference semantics: pbs-datastore/src/chunker.rs:112-186 (Chunker::scan / shall_break).
// The reference rolls one 32-bit Buzhash over the stream byte by byte.  This file
// computes the same cut boundaries in two phases (DESIGN.md "Algorithm"):
//
//   Phase A  (scan_main_kernel + scan_exact_kernel): the hash test
//            (h & mask) >= mask-2 (chunker.rs:185) at EVERY stream position p >= 63.
//            Once the 64-byte window is full, h at p is a pure function of the 64
//            bytes ending at p (rotl by 64 = identity, chunker.rs:146), so positions
//            are independent and are evaluated in parallel: each lane rolls the
//            hash over its own contiguous segment after a 128-byte warm-up.
//   Phase B  (resolve_* kernels): the min/max chunk-size rule (chunker.rs:172-183)
//            applied to the sorted candidate list.  The chain of cuts is a pointer
//            chain over candidates (next[j] = the cut taken after a cut at candidate
//            j); the nodes on the chain from the stream start are marked by pointer
//            doubling, then emitted with an exclusive scan.
//
// No MFMA: this is a byte scan bound by HBM bandwidth (and, on MI355X, by board power:
// DESIGN.md section 6).  The per-byte work of the main scan is one v_perm_b32 (LDS
// address), one ds_read_b32 (replicated table), 1.5 hash ops (v_bitop3_b32 3-input XOR,
// a v_alignbit_b32 rotate every second byte) and half a v_max3_u32.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "buzhash_table.h"
#include "pbs_chunker_internal.h"
#include "exact_block.h"  // exact candidate positions of one 128-byte block (one wave)
#include "scan_main.h"  // scan_main_kernel (phase A main pass)
#include "scan_fused.h"  // scan_fused_kernel (phase A + exact + resolve in one launch)
#include "scan_server.h"  // scan_server_kernel (the low-latency scan() path)

namespace pbs {

// ---------------------------------------------------------------------------------
// Phase A, main kernel
// ---------------------------------------------------------------------------------
// Geometry.  One workgroup of 8 waves per CU (persistent).  A wave owns a "wave tile"
// of 64 contiguous segments of SEG bytes; lane l rolls the hash over segment l.  Each
// iteration every lane consumes 128 bytes of its segment; the wave stages the
// 64 x 128-byte block (8 KiB) through LDS with 8 LDS-DMA instructions
// (global_load_lds_dwordx4), each covering 8 full 128-byte lines.
//
// LDS (128 KiB per workgroup):
//   table  [0, 64 KiB):  row b (256 B) = T0[b] x 32 | T1[b] x 32, byte address
//                        b*256 + u*128 + (lane&31)*4 for byte parity u: ds_read_b32
//                        banks by (a/4) mod 32 per 32-lane half, so a wave64 read of
//                        random bytes is conflict-free and the address is ONE
//                        v_perm_b32 of the data dword and a per-parity lane base.
//   stage  [64, 128 KiB): 8 KiB per wave.  Chunk k (16 B) of lane l's 128-byte block
//                        sits at l*128 + ((k ^ ((l>>1)&7)) * 16): the XOR swizzle
//                        makes the per-lane ds_read_b128 conflict-free.
//
// Hash representation (parity frame): byte i of a lane's block
// keeps g_i = rotl(h_i, c - (i & 1)), c = 33 - popcount(mask); odd bytes need only the
// 3-input XOR with T1 = rotl(T, c-1), even bytes a rotate by 2 and the XOR with
// T0 = rotl(T, c).  In both frames a candidate's top n-1 bits read >= 2^(n-1) - 3, so
// the max over a 128-byte block (v_max3_u32) against one threshold flags the rare
// blocks that may hold a candidate; scan_exact_kernel re-evaluates them exactly.

// ---------------------------------------------------------------------------------
// Phase A, exact evaluation of 128-byte blocks (suspect blocks, stream head, tail)
// ---------------------------------------------------------------------------------
// exact_load / exact_hits / exact_block_wave: exact_block.h

// One wave per work item (suspect blocks, the stream's first block with the carry bytes,
// tail blocks past the last wave tile); 16 waves per workgroup, grid-stride over the
// items.  Hits go to a per-workgroup LDS list (LDS atomics) that is flushed with ONE
// global atomic per workgroup at the end: per-candidate (or per-round) atomics on the
// single output counter serialise in L2 (~10 ns each; 4096 of them cost 40 us).
constexpr int kExactWaves = 16;
constexpr uint32_t kExactLds = 2048;  // candidates buffered per workgroup
__global__ __launch_bounds__(kExactWaves * 64) void scan_exact_kernel(
    const uint8_t* __restrict__ data, uint64_t len, const uint8_t* __restrict__ pre,
    uint32_t pre_len, const uint64_t* __restrict__ susp,
    const unsigned long long* __restrict__ nsusp, uint64_t susp_cap, uint64_t ext_first,
    uint64_t ext_count, int head, uint32_t mask, uint32_t minimum, uint64_t base,
    uint64_t* __restrict__ cand, unsigned long long* __restrict__ ncand, uint64_t cand_cap) {
    __shared__ uint32_t tab[256];
    __shared__ uint64_t lbuf[kExactLds];
    __shared__ uint32_t lcnt;
    __shared__ uint64_t gbase;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = kBuzhashTable[i];
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t ns0 = nsusp ? *nsusp : 0ull;
    const uint64_t ns = ns0 < susp_cap ? ns0 : susp_cap;
    const uint64_t total = ns + (uint64_t)(head ? 1 : 0) + ext_count;
    const uint64_t stride = (uint64_t)gridDim.x * kExactWaves;
    auto item = [&](uint64_t w) -> uint64_t {
        if (w < ns) return susp[w];
        if (head && w == ns) return 0;
        return (ext_first + (w - ns - (head ? 1 : 0))) * (uint64_t)kIter;
    };
    // batches of 64 items per wave: lane j fetches the block position of item j up front,
    // and the window of item j+1 is loaded while item j is hashed
    for (uint64_t w0 = (uint64_t)blockIdx.x * kExactWaves + wave; w0 < total; w0 += 64 * stride) {
        const uint64_t wj = w0 + (uint64_t)lane * stride;
        const uint64_t Bj = wj < total ? item(wj) : 0;
        const uint32_t Blo = (uint32_t)Bj, Bhi = (uint32_t)(Bj >> 32);
        const uint64_t left = (total - w0 + stride - 1) / stride;
        const int cnt = left < 64 ? (int)left : 64;
        auto getB = [&](int j) -> uint64_t {
            return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)Blo, j) |  // j is wave-uniform
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)Bhi, j) << 32);
        };
        uint64_t B = getB(0);
        uint32_t wv = exact_load(data, len, pre, pre_len, (int64_t)B, lane);
        for (int j = 0; j < cnt; ++j) {
            uint64_t Bn = 0;
            uint32_t wvn = 0;
            if (j + 1 < cnt) {
                Bn = getB(j + 1);
                wvn = exact_load(data, len, pre, pre_len, (int64_t)Bn, lane);
            }
            const uint4 hit = exact_hits(wv, len, pre_len, (int64_t)B, tab, mask, minimum, lane);
            if (lane < 4) {  // lane q writes the positions of hit word q
                const uint32_t words[4] = {hit.x, hit.y, hit.z, hit.w};
                uint32_t m = words[lane];
                const uint32_t c = __builtin_popcount(m);
                if (c) {
                    // slots [idx, kExactLds) of the LDS list are all filled; what does not fit
                    // goes straight to the output with its own atomic
                    const uint32_t idx = atomicAdd(&lcnt, c);
                    const uint32_t inl = idx >= kExactLds ? 0u : (c < kExactLds - idx ? c : kExactLds - idx);
                    const uint64_t gidx = c > inl ? atomicAdd(ncand, (unsigned long long)(c - inl)) : 0ull;
                    uint32_t k = 0;
                    while (m) {
                        const int bit = __builtin_ctz(m);
                        m &= m - 1;
                        const uint64_t v = base + B + (uint64_t)(lane * 32 + bit);
                        if (k < inl)
                            lbuf[idx + k] = v;
                        else if (gidx + (k - inl) < cand_cap)
                            cand[gidx + (k - inl)] = v;
                        ++k;
                    }
                }
            }
            B = Bn;
            wv = wvn;
        }
    }
    __syncthreads();
    const uint32_t nl = lcnt < kExactLds ? lcnt : kExactLds;
    if (threadIdx.x == 0) gbase = nl ? atomicAdd(ncand, (unsigned long long)nl) : 0ull;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
        if (gbase + i < cand_cap) cand[gbase + i] = lbuf[i];
}

// Every 128-byte block of a small input (the fused host path): hit mask per block, one
// wave per block.  The block grid sits on 16-byte-aligned addresses: block b starts at
// 128*b - misalign relative to `data` (misalign = data & 15).
__global__ __launch_bounds__(256) void scan_blocks_kernel(const uint8_t* __restrict__ data,
                                                          uint64_t len,
                                                          const uint8_t* __restrict__ pre,
                                                          uint32_t pre_len, uint32_t mask,
                                                          uint32_t minimum, uint4* __restrict__ hits,
                                                          uint64_t nblk) {
    __shared__ uint32_t tab[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = kBuzhashTable[i];
    __syncthreads();
    const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nblk) return;
    const int lane = threadIdx.x & 63;
    const int64_t misalign = (int64_t)((uintptr_t)data & 15);
    const uint4 hit = exact_block_wave(data, len, pre, pre_len, (int64_t)(b * kIter) - misalign, tab,
                                       mask, minimum, lane);
    if (lane == 0) hits[b] = hit;
}

// ---------------------------------------------------------------------------------
// Phase B: resolve the min/max rule over the sorted candidate list
// ---------------------------------------------------------------------------------
// Node j < m: "a cut was taken at candidate C[j]" (next chunk starts at C[j]+1).
// Node m: the stream/buffer state (chunk starts at s0).  Node m+1: sink ("undecided":
// the open chunk needs bytes beyond `end`).
__device__ __forceinline__ uint32_t lower_bound_u64(const uint64_t* __restrict__ C, uint32_t lo,
                                                    uint32_t hi, uint64_t key) {
    // galloping from lo, then binary search
    uint32_t step = 1, prev = lo;
    uint32_t cur = lo;
    while (cur < hi && C[cur] < key) {
        prev = cur + 1;
        cur = lo + step;
        step <<= 1;
        if (cur > hi) cur = hi;
    }
    uint32_t a = prev, b = cur;
    while (a < b) {
        const uint32_t mid = a + ((b - a) >> 1);
        if (C[mid] < key)
            a = mid + 1;
        else
            b = mid;
    }
    return a;
}

// m_dev != nullptr: the node count is m_base + *m_dev, known on the device only (the host
// launched with an upper bound; threads past it exit).  jcopy: a second copy of nxt (the
// pointer doubling's input)
__device__ __forceinline__ uint32_t node_count(uint32_t m, const uint64_t* m_dev, uint32_t m_base) {
    return m_dev ? m_base + (uint32_t)*m_dev : m;
}

__global__ __launch_bounds__(256) void resolve_next_kernel(const uint64_t* __restrict__ C,
                                                           uint32_t m_arg, ResolveParams p,
                                                           uint32_t* __restrict__ nxt,
                                                           uint64_t* __restrict__ nforced,
                                                           uint32_t* __restrict__ on,
                                                           const uint64_t* __restrict__ m_dev, uint32_t m_base,
                                                           uint32_t* __restrict__ jcopy) {
    const uint32_t m = node_count(m_arg, m_dev, m_base);
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t none = m + 1;
    if (j > m + 1) return;
    if (j == m + 1) {
        nxt[j] = none;
        jcopy[j] = none;
        nforced[j] = 0;
        on[j] = 0;
        return;
    }
    uint64_t s = (j == m) ? p.s0 : C[j] + 1;
    uint32_t i = (j == m) ? 0u : j + 1;
    uint64_t nf = 0;
    uint32_t res = none;
    for (;;) {
        const uint64_t lo = s + p.min_eff - 1, hi = s + p.max_eff - 1;
        i = lower_bound_u64(C, i, m, lo);
        if (i < m && C[i] <= hi) {
            res = i;
            break;
        }
        if (hi >= p.end) break;  // undecided: needs bytes beyond `end`
        uint64_t k;
        if (i < m) {
            k = (C[i] - hi + p.max_eff - 1) / p.max_eff;  // forced cuts before C[i] fits
        } else {
            k = (p.end - s) / p.max_eff;  // forced cuts until the data ends
            nf += k;
            s += k * p.max_eff;
            break;
        }
        nf += k;
        s += k * p.max_eff;
    }
    nxt[j] = res;
    jcopy[j] = res;
    nforced[j] = nf;
    on[j] = (j == m) ? 1u : 0u;
}

// Pointer doubling, three rounds per launch.  One round: J_{t+1} = J_t o J_t, and every
// marked node marks its 2^t-th successor (after round t the chain's first 2^(t+1) nodes
// are marked).  Here, from J_t and the marks of the first 2^t nodes, every marked node
// marks its i * 2^t-th successors (i = 1..7, gathered along J_t) and J_{t+3} = J_t^8:
// the same result as three rounds with a third of the launches.  Races on `on` are
// benign: marks only go 0 -> 1, and any node marked is on the chain.
__global__ __launch_bounds__(256) void resolve_double3_kernel(uint32_t n_arg, const uint32_t* __restrict__ jin,
                                                              uint32_t* __restrict__ jout,
                                                              uint32_t* on, const uint64_t* __restrict__ m_dev,
                                                              uint32_t m_base) {
    const uint32_t n = m_dev ? node_count(0, m_dev, m_base) + 2 : n_arg;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const bool mk = on[j] != 0u;
    uint32_t x = j;
#pragma unroll
    for (int i = 1; i <= 8; ++i) {
        x = jin[x];
        if (mk && i < 8) on[x] = 1u;
    }
    jout[j] = x;
}

__device__ __forceinline__ uint32_t slot_of(uint32_t j, uint32_t m) { return j == m ? 0u : j + 1u; }

__global__ __launch_bounds__(256) void resolve_count_kernel(uint32_t m_arg, const uint32_t* __restrict__ nxt,
                                                            const uint64_t* __restrict__ nforced,
                                                            const uint32_t* __restrict__ on,
                                                            uint64_t* __restrict__ cnt,
                                                            const uint64_t* __restrict__ m_dev, uint32_t m_base) {
    const uint32_t m = node_count(m_arg, m_dev, m_base);
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > m) {  // nodes 0..m; slots past them (an upper-bound launch) count nothing
        if (j <= m_arg) cnt[j] = 0;
        return;
    }
    // slot 0 = the start node m (its cuts come first), slot j+1 = candidate node j
    cnt[slot_of(j, m)] = on[j] ? nforced[j] + (nxt[j] != m + 1 ? 1u : 0u) : 0u;
}

// out[] = chunk END offsets (absolute, exclusive).  res[0] = number of cuts,
// res[1] = start of the open (undecided) chunk, res[2] = index of the first
// candidate >= res[1].
__global__ __launch_bounds__(256) void resolve_emit_kernel(
    const uint64_t* __restrict__ C, uint32_t m_arg, ResolveParams p, const uint32_t* __restrict__ nxt,
    const uint64_t* __restrict__ nforced, const uint32_t* __restrict__ on,
    const uint64_t* __restrict__ cnt, const uint64_t* __restrict__ off, uint64_t* __restrict__ out,
    uint64_t out_cap, uint64_t* __restrict__ res, const uint64_t* __restrict__ m_dev, uint32_t m_base) {
    const uint32_t m = node_count(m_arg, m_dev, m_base);
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > m || !on[j]) return;
    const uint64_t s = (j == m) ? p.s0 : C[j] + 1;
    const uint64_t o = off[slot_of(j, m)];
    const uint64_t nf = nforced[j];
    for (uint64_t t = 0; t < nf; ++t)
        if (o + t < out_cap) out[o + t] = s + (t + 1) * p.max_eff;
    if (nxt[j] != m + 1) {
        if (o + nf < out_cap) out[o + nf] = C[nxt[j]] + 1;
    } else {
        const uint64_t s_open = s + nf * p.max_eff;
        res[0] = o + cnt[slot_of(j, m)];
        res[1] = s_open;
        res[2] = lower_bound_u64(C, 0, m, s_open);
    }
}

// ---------------------------------------------------------------------------------
// Phase B for small batches, one workgroup (the 64 GiB / 4 MiB-average stream has
// ~14k candidates): the multi-kernel path above costs ~20 launches, a device-wide
// radix sort and a device-wide scan; here the keys are bucket-sorted in LDS, the
// pointer doubling runs on 16-bit successor arrays in LDS, and the cut list is copied
// straight into mapped pinned host memory, so the host needs one sync.  Same
// node/slot semantics as resolve_next/double/count/emit.  One CU cannot hide latency
// with parallel slack, so every phase issues its independent loads in batches.
// ---------------------------------------------------------------------------------
constexpr uint32_t kSmallThreads = 1024;
constexpr uint32_t kSmallBig = 64;        // nodes with many forced cuts, filled by the block
constexpr uint32_t kSmallBigMin = 256;    // forced-cut run length handed to the block
constexpr uint32_t kSmallJ = kSmallResolveMax;  // u16 successor array stride (>= m + 2)

constexpr uint32_t kSmallBuckets = 4096;
constexpr uint32_t kSmallBucketMax = 256;  // larger buckets (skewed input): bitonic fallback
constexpr uint32_t kSmallPer = (kSmallJ + kSmallThreads - 1) / kSmallThreads;  // nodes per thread
constexpr uint32_t kSmallChunk = 10;  // slots per batch of independent global loads

// Buckets of 2^shift bytes from s0, shift = the smallest with span >> shift < kSmallBuckets
// (a shift, not a 64-bit division: those are long software sequences on the GPU).
__device__ __forceinline__ uint32_t small_bucket(uint64_t key, uint64_t lo, uint32_t shift) {
    return (uint32_t)((key - lo) >> shift);
}

// Exclusive scan of one value per thread over the block (Hillis-Steele in `part`).
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t* part, uint64_t v, uint32_t tid,
                                                        uint64_t* total = nullptr) {
    // wave-level inclusive scan by shuffles, then the 16 wave totals (3 barriers instead
    // of 20 for a Hillis-Steele pass over LDS)
    constexpr uint32_t W = kSmallThreads / 64;
    const uint32_t lane = tid & 63, w = tid >> 6;
    unsigned long long x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    if (w == 0) {
        unsigned long long t = lane < W ? part[lane] : 0ull;
#pragma unroll
        for (int d = 1; d < (int)W; d <<= 1) {
            const unsigned long long y = __shfl_up(t, d, 64);
            if (lane >= (uint32_t)d) t += y;
        }
        if (lane < W) part[lane] = t;  // inclusive wave prefixes
    }
    __syncthreads();
    const uint64_t r = (w ? part[w - 1] : 0ull) + x - v;
    if (total) *total = part[W - 1];
    __syncthreads();  // part is reused by the caller's next scan
    return r;
}

// FUSED = 0: resolve `nnew` unsorted candidates (newc) after `np` sorted pending ones
//            (C[0..np)).
// FUSED = 1: small inputs (the host path's 256 KiB pieces): the kernel also scans the
//            input itself -- every 128-byte block with exact_block, hits compacted in
//            block order, so the keys come out sorted -- after the pending candidates
//            (fa.pend), then resolves; one launch per call instead of ~10.
// FUSED = 2: scan only; the sorted candidates go to fa.cand_out (mapped host memory).
// More than kSmallResolveMax - 2 keys in a fused call: res_host[12] = 1 and nothing else
// is written (the host reruns the call on the multi-kernel path).
template <int FUSED>
__global__ __launch_bounds__(kSmallThreads) void resolve_small_kernel(
    const uint64_t* __restrict__ newc, uint32_t nnew, uint64_t* C, uint32_t np, ResolveParams p,
    uint32_t* nxt, uint64_t* nforced, uint64_t* __restrict__ out, uint64_t out_cap,
    uint64_t* __restrict__ out_host, uint64_t host_cap, uint64_t* __restrict__ keep_host,
    uint64_t keep_cap, uint64_t* __restrict__ res, uint64_t* __restrict__ res_host,
    FusedScanArgs fa) {
    __shared__ __attribute__((aligned(16))) uint64_t sk[kSmallResolveMax];  // keys; later ja | jb | on | nx16 | nf8
    __shared__ uint64_t part[kSmallThreads];
    __shared__ uint64_t big[kSmallBig][3];
    __shared__ uint64_t open_info[3];
    __shared__ uint32_t bcnt[kSmallBuckets];
    __shared__ uint32_t nbig, bmax;
    // after the sort, sk holds ja | jb (u16) | on (u8) | nx16 (u16) | nf8 (u8)
    static_assert(3 * kSmallJ * 2 + 2 * kSmallJ <= sizeof(uint64_t) * kSmallResolveMax, "LDS reuse");
    static_assert(kSmallPer <= 32, "on-mask bits");

    const uint32_t tid = threadIdx.x, T = kSmallThreads;
    if constexpr (FUSED == 0) {
        if (fa.counts) {  // speculative: the candidate count is only known on the device
            const uint64_t ns = fa.counts[0], nc = fa.counts[1];
            if (fa.counts_host && tid < 2) fa.counts_host[tid] = tid ? nc : ns;
            if (fa.tail_host && tid < fa.tail_len) fa.tail_host[tid] = fa.tail_src[tid];
            const bool fits = ns <= fa.susp_cap && nc <= fa.cand_cap &&
                              (uint64_t)np + nc + 2 <= kSmallResolveMax;
            if (tid == 0) res_host[12] = fits ? 0u : 1u;
            if (!fits) return;  // uniform
            nnew = (uint32_t)nc;
        }
    }
    uint32_t m = np + nnew;

    const uint64_t t_start = wall_clock64();
    uint64_t t_hist = t_start, t_bscan = t_start, t_scatter = t_start;
    uint32_t bshift = 0;
    if constexpr (FUSED != 0) {
        // 1'. pending keys, then the candidates of the input's 128-byte blocks (hit masks
        //     from scan_blocks_kernel), compacted in block order -- so already sorted.
        //     Thread t owns the contiguous blocks [t*per, (t+1)*per).
        for (uint32_t i = tid; i < np; i += T) sk[i] = fa.pend[i];
        if (tid == 0) nbig = 0;
        const uint32_t per = (uint32_t)((fa.nblk + T - 1) / T);
        const uint64_t b_lo = min((uint64_t)tid * per, fa.nblk);
        const uint64_t b_hi = min(b_lo + per, fa.nblk);
        uint32_t k = 0;
        for (uint64_t b = b_lo; b < b_hi; ++b) {
            const uint4 hm = fa.hits[b];
            k += __builtin_popcount(hm.x) + __builtin_popcount(hm.y) + __builtin_popcount(hm.z) +
                 __builtin_popcount(hm.w);
        }
        uint64_t total;
        uint32_t idx = np + (uint32_t)block_exclusive_scan(part, k, tid, &total);
        if (np + total + 2 > kSmallResolveMax) {  // uniform
            if (tid == 0) res_host[12] = 1;
            return;
        }
        for (uint64_t b = b_lo; b < b_hi; ++b) {
            const uint4 hm = fa.hits[b];
            const uint32_t w4[4] = {hm.x, hm.y, hm.z, hm.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t mm = w4[q];
                while (mm) {
                    const int bit = __builtin_ctz(mm);
                    mm &= mm - 1;
                    sk[idx++] = fa.base + b * kBlockBytes + (uint64_t)(q * 32 + bit);
                }
            }
        }
        m = np + (uint32_t)total;
        __syncthreads();
        if constexpr (FUSED == 2) {
            if (m - np <= fa.cand_cap)
                for (uint32_t i = np + tid; i < m; i += T) fa.cand_out[i - np] = sk[i];
            if (tid == 0) {
                res_host[0] = m - np;
                res_host[12] = 0;
            }
            return;
        }
        if (tid == 0) {
            res_host[12] = 0;
            res_host[13] = m;
            bmax = kSmallBucketMax + 1;  // no bucket index: plain searches below
        }
        __syncthreads();
    }
    const uint32_t none = m + 1;
    if constexpr (FUSED == 0) {

    // 1. sort the keys into LDS.  All keys lie in [s0, end) (pending >= chunk_start,
    //    new < end), so a bucket sort over kSmallBuckets equal ranges of that span
    //    (histogram, scan, scatter, insertion sort per bucket) is O(m); a bucket
    //    holding more than kSmallBucketMax keys (skewed input) falls back to a
    //    bitonic sort of the whole set.
    const uint64_t span = p.end > p.s0 ? p.end - p.s0 : 1;
    while ((span >> bshift) >= kSmallBuckets) ++bshift;
    for (uint32_t b = tid; b < kSmallBuckets; b += T) bcnt[b] = 0;
    if (tid == 0) {
        nbig = 0;
        bmax = 0;
    }
    __syncthreads();
    for (uint32_t i = tid; i < m; i += T) {
        const uint64_t key = i < np ? C[i] : newc[i - np];
        atomicAdd(&bcnt[small_bucket(key, p.s0, bshift)], 1u);
    }
    __syncthreads();
    t_hist = wall_clock64();
    {
        constexpr uint32_t per_b = kSmallBuckets / kSmallThreads;
        uint32_t c[per_b], bsum = 0, bm = 0;
#pragma unroll
        for (int q = 0; q < (int)per_b; ++q) {
            c[q] = bcnt[tid * per_b + q];
            bsum += c[q];
            bm = c[q] > bm ? c[q] : bm;
        }
        atomicMax(&bmax, bm);
        const uint64_t before = block_exclusive_scan(part, bsum, tid);
        uint32_t o = (uint32_t)before;
#pragma unroll
        for (int q = 0; q < (int)per_b; ++q) {
            bcnt[tid * per_b + q] = o;  // bucket start
            o += c[q];
        }
    }
    __syncthreads();
    t_bscan = wall_clock64();
    t_scatter = t_bscan;
    if (bmax <= kSmallBucketMax) {
        for (uint32_t i = tid; i < m; i += T) {
            const uint64_t key = i < np ? C[i] : newc[i - np];
            sk[atomicAdd(&bcnt[small_bucket(key, p.s0, bshift)], 1u)] = key;
        }
        __syncthreads();  // bcnt[b] = end of bucket b
        t_scatter = wall_clock64();
        // final index of a key = its bucket's start + #smaller keys in the bucket
        // (positions are distinct); kept in registers until every thread has ranked,
        // then placed in LDS (and in C, which the later steps read)
        static_assert(kSmallPer * kSmallThreads >= kSmallResolveMax, "keys per thread");
        uint64_t kq[kSmallPer];
        uint32_t dq[kSmallPer];
#pragma unroll
        for (uint32_t q = 0; q < kSmallPer; ++q) {
            const uint32_t i = tid + q * T;
            kq[q] = 0;
            dq[q] = ~0u;
            if (i < m) {
                const uint64_t key = sk[i];
                const uint32_t b = small_bucket(key, p.s0, bshift);
                const uint32_t lo = b ? bcnt[b - 1] : 0u, hi = bcnt[b];
                uint32_t rank = 0;
                for (uint32_t k = lo; k < hi; ++k) rank += sk[k] < key ? 1u : 0u;
                kq[q] = key;
                dq[q] = lo + rank;
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < kSmallPer; ++q)
            if (dq[q] != ~0u) {
                sk[dq[q]] = kq[q];
                C[dq[q]] = kq[q];
            }
        __syncthreads();
    } else {
        uint32_t N = 2;
        while (N < m) N <<= 1;
        for (uint32_t i = tid; i < N; i += T) sk[i] = i < np ? C[i] : (i < m ? newc[i - np] : ~0ull);
        __syncthreads();
        for (uint32_t k = 2; k <= N; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < N / 2; i += T) {
                    const uint32_t a = ((i & ~(j - 1)) << 1) | (i & (j - 1));
                    const uint32_t b = a | j;
                    const uint64_t x = sk[a], y = sk[b];
                    if ((x > y) == ((a & k) == 0)) {
                        sk[a] = y;
                        sk[b] = x;
                    }
                }
                __syncthreads();
            }
        }
    }
    }  // FUSED == 0
    const uint64_t t_sorted = wall_clock64();
    const bool bucketed = bmax <= kSmallBucketMax;

    // 2. sorted keys -> C; successor candidate and forced-cut count of every node.  The
    //    search for the first key >= lo starts at lo's bucket (bucket b starts at the
    //    end of bucket b-1), so it gallops over at most one bucket.
    if (!bucketed)
        for (uint32_t i = tid; i < m; i += T) C[i] = sk[i];
    for (uint32_t j = tid; j <= m; j += T) {
        uint64_t s = (j == m) ? p.s0 : sk[j] + 1;
        uint32_t i = (j == m) ? 0u : j + 1;
        uint64_t nf = 0;
        uint32_t r = none;
        for (;;) {
            const uint64_t lo = s + p.min_eff - 1, hi = s + p.max_eff - 1;
            if (lo >= p.end) {
                i = m;
            } else {
                if (bucketed) {
                    const uint32_t b = small_bucket(lo, p.s0, bshift);
                    const uint32_t bs = b ? bcnt[b - 1] : 0u;
                    i = bs > i ? bs : i;
                }
                i = lower_bound_u64(sk, i, m, lo);
            }
            if (i < m && sk[i] <= hi) {
                r = i;
                break;
            }
            if (hi >= p.end) break;
            uint64_t k;
            if (i < m) {
                k = (sk[i] - hi + p.max_eff - 1) / p.max_eff;
            } else {
                k = (p.end - s) / p.max_eff;
                nf += k;
                break;
            }
            nf += k;
            s += k * p.max_eff;
        }
        nxt[j] = r;
        nforced[j] = nf;
    }
    __syncthreads();
    const uint64_t t_next = wall_clock64();

    // 3. pointer doubling in LDS (marks only go 0 -> 1; see resolve_double3_kernel)
    uint16_t* ja = reinterpret_cast<uint16_t*>(sk);
    uint16_t* jb = ja + kSmallJ;
    uint8_t* on = reinterpret_cast<uint8_t*>(jb + kSmallJ);
    // successor and forced-cut count kept in LDS for the emit step (nf8 = 255: see nforced)
    uint16_t* nx16 = reinterpret_cast<uint16_t*>(on + kSmallJ);
    uint8_t* nf8 = reinterpret_cast<uint8_t*>(nx16 + kSmallJ);
    const uint32_t n = m + 2;
    // every slot of the arrays is initialised: nodes >= n point to the sink (m + 1, a
    // self-loop) and are never marked, so the rounds below need no bounds checks
    for (uint32_t j = tid; j < kSmallJ; j += T) {
        const uint32_t x = j <= m ? nxt[j] : none;  // own writes from step 2
        const uint64_t f = j <= m ? nforced[j] : 0;
        ja[j] = (uint16_t)x;
        nx16[j] = (uint16_t)x;
        nf8[j] = (uint8_t)(f < 255 ? f : 255);
        on[j] = j == m ? 1 : 0;
    }
    __syncthreads();
    // thread t owns the 16 consecutive nodes [16t, 16t + 16): its successors and marks
    // come in with two ds_read_b128 + one ds_read_b128, the 16 gathers are issued before
    // any is used (one LDS latency per round), the new successors leave with two
    // ds_write_b128
    static_assert(kSmallPer == 16 && kSmallJ == kSmallPer * kSmallThreads, "doubling layout");
    const uint32_t j0 = tid * kSmallPer;
    for (uint32_t rnd = 1; rnd < n; rnd <<= 1) {
        const uint4 a0 = *reinterpret_cast<const uint4*>(ja + j0);
        const uint4 a1 = *reinterpret_cast<const uint4*>(ja + j0 + 8);
        const uint4 ov = *reinterpret_cast<const uint4*>(on + j0);
        const uint32_t aw[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const uint32_t ow[4] = {ov.x, ov.y, ov.z, ov.w};
        uint32_t J[16], JJ[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) J[q] = (aw[q >> 1] >> (16 * (q & 1))) & 0xffffu;
#pragma unroll
        for (int q = 0; q < 16; ++q) JJ[q] = ja[J[q]];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if ((ow[q >> 2] >> (8 * (q & 3))) & 0xffu) on[J[q]] = 1;
        uint4 b0, b1;
        b0.x = JJ[0] | (JJ[1] << 16);
        b0.y = JJ[2] | (JJ[3] << 16);
        b0.z = JJ[4] | (JJ[5] << 16);
        b0.w = JJ[6] | (JJ[7] << 16);
        b1.x = JJ[8] | (JJ[9] << 16);
        b1.y = JJ[10] | (JJ[11] << 16);
        b1.z = JJ[12] | (JJ[13] << 16);
        b1.w = JJ[14] | (JJ[15] << 16);
        *reinterpret_cast<uint4*>(jb + j0) = b0;
        *reinterpret_cast<uint4*>(jb + j0 + 8) = b1;
        __syncthreads();
        uint16_t* t = ja;
        ja = jb;
        jb = t;
    }
    const uint64_t t_doubled = wall_clock64();

    // 4. per-thread contiguous slot ranges (slot 0 = start node m, slot j+1 = node j),
    //    block-wide exclusive scan of the cut counts
    const uint32_t slots = m + 1;
    const uint32_t per = (slots + T - 1) / T;
    const uint32_t s_lo = min(tid * per, slots), s_hi = min(s_lo + per, slots);
    uint64_t sum = 0;
    for (uint32_t c0 = s_lo; c0 < s_hi; c0 += kSmallChunk) {
        uint64_t nfq[kSmallChunk];
        uint32_t nxq[kSmallChunk];
#pragma unroll
        for (uint32_t q = 0; q < kSmallChunk; ++q) {
            const uint32_t sl = c0 + q;
            const uint32_t j = sl == 0 ? m : sl - 1;
            const bool live = sl < s_hi && on[j];
            const uint32_t f8 = live ? nf8[j] : 0u;
            nfq[q] = f8 == 255 ? nforced[j] : f8;
            nxq[q] = live ? nx16[j] : none;
        }
#pragma unroll
        for (uint32_t q = 0; q < kSmallChunk; ++q) sum += nfq[q] + (nxq[q] != none ? 1u : 0u);
    }
    uint64_t o = block_exclusive_scan(part, sum, tid);
    const uint64_t t_scanned = wall_clock64();

    // 5. emit
    for (uint32_t c0 = s_lo; c0 < s_hi; c0 += kSmallChunk) {
      uint32_t jq[kSmallChunk], nxq[kSmallChunk];
      uint64_t nfq[kSmallChunk], cj[kSmallChunk], cn[kSmallChunk];
      uint32_t live = 0;
#pragma unroll
      for (uint32_t q = 0; q < kSmallChunk; ++q) {
          const uint32_t sl = c0 + q;
          jq[q] = sl == 0 ? m : sl - 1;
          const bool l = sl < s_hi && on[jq[q]];
          live |= l ? (1u << q) : 0u;
          const uint32_t f8 = l ? nf8[jq[q]] : 0u;
          nfq[q] = f8 == 255 ? nforced[jq[q]] : f8;
          nxq[q] = l ? nx16[jq[q]] : none;
          cj[q] = (l && jq[q] != m) ? C[jq[q]] : 0u;
      }
#pragma unroll
      for (uint32_t q = 0; q < kSmallChunk; ++q) cn[q] = nxq[q] != none ? C[nxq[q]] : 0u;
#pragma unroll
      for (uint32_t q = 0; q < kSmallChunk; ++q) {
        if (!(live & (1u << q))) continue;
        const uint32_t j = jq[q];
        const uint64_t s = (j == m) ? p.s0 : cj[q] + 1;
        const uint64_t nf = nfq[q];
        bool done = false;
        if (nf >= kSmallBigMin) {
            const uint32_t b = atomicAdd(&nbig, 1u);
            if (b < kSmallBig) {
                big[b][0] = s;
                big[b][1] = o;
                big[b][2] = nf;
                done = true;
            }
        }
        if (!done)
            for (uint64_t t = 0; t < nf; ++t)
                if (o + t < out_cap) out[o + t] = s + (t + 1) * p.max_eff;
        if (nxq[q] != none) {
            if (o + nf < out_cap) out[o + nf] = cn[q] + 1;
            o += nf + 1;
        } else {
            open_info[0] = o + nf;              // cuts before the open chunk = all cuts
            open_info[1] = s + nf * p.max_eff;  // start of the open chunk
            o += nf;
        }
      }
    }
    __syncthreads();
    const uint32_t nb = min(nbig, kSmallBig);
    for (uint32_t b = 0; b < nb; ++b)
        for (uint64_t t = tid; t < big[b][2]; t += T)
            if (big[b][1] + t < out_cap) out[big[b][1] + t] = big[b][0] + (t + 1) * p.max_eff;
    __syncthreads();  // open_info[1] (the open chunk's start) is set
    {
        // index of the first candidate >= the open chunk's start: C is sorted, so it is the
        // number of smaller keys (one round of independent loads instead of a serial
        // gallop + binary search through L2)
        const uint64_t key = open_info[1];
        uint64_t cnt = 0;
        for (uint32_t i = tid; i < m; i += T) cnt += C[i] < key ? 1u : 0u;
        uint64_t below = 0;
        (void)block_exclusive_scan(part, cnt, tid, &below);
        if (tid == 0) open_info[2] = below;
    }
    __syncthreads();
    const uint64_t t_emit = wall_clock64();
    // cut list -> mapped pinned host memory, 16-byte coalesced stores
    const uint64_t ncut = open_info[0];
    if (ncut <= host_cap && ncut <= out_cap) {
        const uint64_t pairs = ncut / 2;
        const uint4* src = reinterpret_cast<const uint4*>(out);
        uint4* dst = reinterpret_cast<uint4*>(out_host);
        for (uint64_t i = tid; i < pairs; i += T) dst[i] = src[i];
        if (tid == 0 && (ncut & 1)) out_host[ncut - 1] = out[ncut - 1];
    }
    const uint64_t idx = open_info[2];
    if (tid < 3) {
        res[tid] = open_info[tid];
        res_host[tid] = open_info[tid];
    }
    if (tid == 0) {  // phase durations (100 MHz ticks), read by diagnostics only
        const uint64_t t_end = wall_clock64();
        const uint64_t ph[9] = {t_hist - t_start,    t_bscan - t_hist,     t_scatter - t_bscan,
                                t_sorted - t_scatter, t_next - t_sorted,    t_doubled - t_next,
                                t_scanned - t_doubled, t_emit - t_scanned,  t_end - t_emit};
        for (int q = 0; q < 9; ++q) res_host[3 + q] = ph[q];
    }
    if (m - idx <= keep_cap)
        for (uint64_t i = idx + tid; i < m; i += T) keep_host[i - idx] = C[i];
}

// ---------------------------------------------------------------------------------
// Synthetic stream generator (bench / tests; same bytes as oracle/chunker_oracle.c)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void gen_kernel(uint64_t* __restrict__ out, uint64_t nwords,
                                                  uint64_t seed, uint64_t word_offset, int kind) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += stride) {
        const uint64_t gw = word_offset + w;  // global word index
        uint64_t v;
        if (kind == kGenCounter) {
            const uint32_t i0 = (uint32_t)(2 * gw), i1 = (uint32_t)(2 * gw + 1);
            v = (uint64_t)i0 | ((uint64_t)i1 << 32);
        } else if (kind == kGenRandom) {
            v = splitmix64(seed ^ gw);
        } else {
            const uint64_t x = gw << 3;
            const uint64_t g = x >> 30;
            const uint64_t ext = (splitmix64(seed ^ kVmSeedExt ^ g) & 15u) << 26;
            const uint64_t in_g = x & ((1ull << 30) - 1);
            if (in_g >= ext && in_g < ext + (1ull << 26))
                v = 0;
            else if (splitmix64(seed ^ kVmSeedPage ^ (x >> 12)) % 100u < 40u)
                v = 0;
            else
                v = splitmix64(seed ^ kVmSeedWord ^ gw);
        }
        out[w] = v;
    }
}

// ---------------------------------------------------------------------------------
// Host-side launchers (called from pbs_chunker_capi.cpp)
// ---------------------------------------------------------------------------------
int scan_main_plan(uint64_t len, int cu, uint64_t* ntiles, bool* dyn, uint64_t* t_big) {
    // Tile order: dynamic (waves draw tiles from a counter, so waves on faster CUs take
    // more) once every wave gets >= 16 tiles of 16 KiB segments; measured same-process
    // A/B on MI355X (scripts/ab_dyn.py, profiles/r01/dyn/): 64 GiB 11.13 -> 10.55 ms
    // (static 32 KiB -> dynamic 16 KiB; 10.92 -> 10.66 on another box, where dynamic
    // 8 KiB / 4 KiB took 10.86 / 11.26: more warm-up re-reads), 64 GiB at 256 KiB
    // 11.85 -> 11.02; at 1-8 GiB (2-4 tiles per wave) static is 2-3 % faster.  Static: the largest segment that
    // still gives every wave >= 2 tiles; the 128-byte warm-up per segment costs 128/SEG
    // of the work and traffic.
    const uint64_t waves = (uint64_t)cu * kWavesPerWG;
    int cap = 32768;  // PBS_MAX_SEG / PBS_SCAN_DYN: experiment knobs (A/B sweeps)
    if (const char* e = std::getenv("PBS_MAX_SEG")) cap = std::atoi(e);
    bool d = len / (64ull * 16384) >= 16 * waves;
    if (const char* e = std::getenv("PBS_SCAN_DYN")) d = e[0] == '1';
    int seg = 0;
    if (d) {
        for (int s : {16384, 8192})
            if (s <= cap && len / (64ull * s) >= 2 * waves) {
                seg = s;
                break;
            }
    }
    if (seg == 0) {
        d = false;
        seg = 4096;
        for (int s : {32768, 16384, 8192}) {
            if (s <= cap && len / (64ull * s) >= 2 * waves) {
                seg = s;
                break;
            }
        }
    }
    *dyn = d;
    *ntiles = len / (64ull * seg);
    *t_big = *ntiles;
    // dynamic order: end with 2 small tiles (segments of seg / 4) per wave, so the waves
    // finish within a quarter tile of each other (PBS_SCAN_SMALL=0: no small tiles)
    const char* es = std::getenv("PBS_SCAN_SMALL");
    if (d && !(es && es[0] == '0')) {
        const uint64_t big = 64ull * seg, small = big / 4, small_bytes = 2 * waves * small;
        if (len > small_bytes + big) {
            *t_big = (len - small_bytes) / big;
            *ntiles = *t_big + (len - *t_big * big) / small;
        }
    }
    return seg;
}

uint64_t scan_main_covered(uint64_t ntiles, uint64_t t_big, int seg) {
    return t_big >= ntiles ? ntiles * 64ull * seg : t_big * 64ull * seg + (ntiles - t_big) * 16ull * seg;
}

hipError_t launch_scan_main(const uint8_t* data, uint64_t ntiles, int seg,
                            const uint32_t* table_rot, uint32_t thr, uint64_t* susp,
                            unsigned long long* nsusp, uint64_t cap, int grid, hipStream_t stream,
                            uint32_t* tile_ctr, bool dynamic, uint64_t t_big, bool balance) {
    if (ntiles == 0) return hipSuccess;
    (void)hipGetLastError();  // launch errors below must not be confused with stale ones
    const uint64_t need = (ntiles + kWavesPerWG - 1) / kWavesPerWG;
    const int g = (uint64_t)grid < need ? grid : (int)need;
    const dim3 gd(g), bd(kWavesPerWG * 64);
    const bool dyn = tile_ctr && dynamic;  // tile_ctr: a zeroed device counter
    const uint32_t bal = balance ? 1u : 0u;
#define PBS_SCAN_CASE(S)                                                                          \
    case S:                                                                                       \
        if (dyn)                                                                                  \
            hipLaunchKernelGGL((scan_main_kernel<S, kModeFull, 2, 4, 0, 0, kScanFrame, 1>), gd, bd, 0, \
                               stream, data, ntiles, table_rot, thr, susp, nsusp, cap, tile_ctr,    \
                               t_big, bal);                                                        \
        else                                                                                      \
            hipLaunchKernelGGL((scan_main_kernel<S, kModeFull, 2, 4, 0, 0, kScanFrame, 0>), gd, bd, 0, \
                               stream, data, ntiles, table_rot, thr, susp, nsusp, cap, nullptr,     \
                               ~0ull, bal);                                                        \
        break;
    switch (seg) {
        PBS_SCAN_CASE(32768)
        PBS_SCAN_CASE(16384)
        PBS_SCAN_CASE(8192)
        PBS_SCAN_CASE(4096)
        default:
            return hipErrorInvalidValue;
    }
#undef PBS_SCAN_CASE
    return hipGetLastError();
}

hipError_t launch_scan_fused(const FusedPassArgs& a, int seg, bool dyn, int grid, hipStream_t stream) {
    if (a.ntiles + a.ntail == 0 || grid < 1) return hipErrorInvalidValue;
    (void)hipGetLastError();
    const dim3 gd(grid), bd(kWavesPerWG * 64);
    // the dynamic tile order only ever uses 16 / 8 KiB segments (scan_main_plan); the
    // static order has runtime segment lengths up to kFusedStaticSeg (fused_static_plan)
    if (dyn && seg == 16384)
        hipLaunchKernelGGL((scan_fused_kernel<16384, 1>), gd, bd, 0, stream, a);
    else if (dyn && seg == 8192)
        hipLaunchKernelGGL((scan_fused_kernel<8192, 1>), gd, bd, 0, stream, a);
    else if (!dyn && a.seg_q + (a.t_long ? 1u : 0u) <= (uint32_t)kFusedStaticSeg / kBlockBytes &&
             a.seg_qs + (a.t_small_long ? 1u : 0u) <= (uint32_t)kFusedStaticSeg / kBlockBytes &&
             a.t_small <= a.ntiles)
        hipLaunchKernelGGL((scan_fused_kernel<kFusedStaticSeg, 0>), gd, bd, 0, stream, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---- scan pass (scan_fused_kernel without resolver waves): records -> candidates in order
__global__ void fused_rec_counts_kernel(const unsigned long long* __restrict__ rec, uint64_t nrec, uint32_t epoch,
                                        uint64_t* __restrict__ counts, uint64_t* __restrict__ res) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nrec) return;
    uint64_t c = 0;
    if (i < nrec) {
        const uint64_t r = rec[i];
        // a record of an earlier launch (another epoch) is a group this launch left empty
        if ((uint32_t)(r >> 48) == epoch) {
            c = (r >> 32) & 0xFFFFu;
            if (c == kRecOverflow) {
                res[1] = 1;
                c = 0;
            }
        }
    }
    counts[i] = c;
}

// res (mapped host memory): [0] candidates gathered, [1] overflow (counts kernel), [2] flagged
// blocks, [3] candidates listed (the scan kernel's counters); the batch's last tl bytes go to
// tail_dst (mapped) -- the host reads all of it after one sync, no copies
__global__ void fused_gather_kernel(const unsigned long long* __restrict__ rec, uint64_t nrec, uint32_t epoch,
                                    const uint64_t* __restrict__ offs, const uint64_t* __restrict__ cand,
                                    uint64_t* __restrict__ out, uint64_t* __restrict__ res,
                                    const unsigned long long* __restrict__ counters, const uint8_t* __restrict__ tail_src,
                                    uint32_t tl, uint8_t* __restrict__ tail_dst, uint64_t* __restrict__ count_dev) {
    const int lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); r < nrec; r += nwaves) {
        const uint64_t v = rec[r];
        if ((uint32_t)(v >> 48) != epoch) continue;
        const uint32_t c = (uint32_t)(v >> 32) & 0xFFFFu;
        if (c == kRecOverflow) continue;
        const uint64_t idx = (uint32_t)v, o = offs[r];
        for (uint32_t j = (uint32_t)lane; j < c; j += 64) out[o + j] = cand[idx + j];
    }
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            res[0] = offs[nrec];
            count_dev[0] = offs[nrec];  // (device memory: what the resolve kernels read)
            res[2] = counters[0];
            res[3] = counters[1];
        }
        if (threadIdx.x < tl) tail_dst[threadIdx.x] = tail_src[threadIdx.x];
    }
}

// The open chunk's candidates C[idx, m) (idx = res[2], written by resolve_emit_kernel) to
// mapped host memory when they fit keep_cap, else res[3] = 1 (the host copies them)
__global__ void resolve_keep_kernel(const uint64_t* __restrict__ C, uint32_t m_arg, uint64_t* res, uint64_t* __restrict__ keep,
                                    uint64_t keep_cap, const uint64_t* __restrict__ m_dev, uint32_t m_base) {
    const uint32_t m = node_count(m_arg, m_dev, m_base);
    const uint64_t idx = res[2];
    const uint64_t nk = m > idx ? m - idx : 0;
    if (nk > keep_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) res[3] = 1;
        return;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nk; i += (uint64_t)gridDim.x * blockDim.x)
        keep[i] = C[idx + i];
}

hipError_t launch_resolve_keep(const uint64_t* C, uint32_t m, uint64_t* res, uint64_t* keep, uint64_t keep_cap,
                               const uint64_t* m_dev, uint32_t m_base, hipStream_t stream) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(resolve_keep_kernel, dim3(16), dim3(256), 0, stream, C, m, res, keep, keep_cap, m_dev, m_base);
    return hipGetLastError();
}

hipError_t launch_fused_gather(const unsigned long long* rec, uint64_t nrec, uint32_t epoch, const uint64_t* cand,
                               uint64_t* out, uint64_t* counts, uint64_t* offs, void* scan_tmp, size_t scan_tmp_bytes,
                               uint64_t* res, const unsigned long long* counters, const uint8_t* tail_src, uint32_t tl,
                               uint8_t* tail_dst, uint64_t* count_dev, hipStream_t stream) {
    if (tl > 256) return hipErrorInvalidValue;
    if (nrec + 1 > 0xFFFFFFFFull) return hipErrorInvalidValue;
    (void)hipGetLastError();
    hipLaunchKernelGGL(fused_rec_counts_kernel, dim3((unsigned)((nrec + 256) / 256)), dim3(256), 0, stream, rec, nrec,
                       epoch, counts, res);
    hipError_t e = exclusive_sum_u64(scan_tmp, &scan_tmp_bytes, counts, offs, (uint32_t)(nrec + 1), stream);
    if (e != hipSuccess) return e;
    // a wave per record, every record at once (a grid-stride loop of 25 records per wave
    // chained three memory round trips per record: 37 us at 64 KiB averages)
    const uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>((nrec + 3) / 4, 1), 1u << 20);
    hipLaunchKernelGGL(fused_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, rec, nrec, epoch, offs, cand,
                       out, res, counters, tail_src, tl, tail_dst, count_dev);
    return hipGetLastError();
}

hipError_t launch_scan_server(ServerMailbox* mb_dev, const ServerReq* req_dev, ServerDispatch* disp_dev,
                              const uint8_t* slot_dev, const uint8_t* hslot_dev, const uint32_t* table_rot,
                              uint32_t thr, uint64_t last_seq, uint64_t idle_ticks, uint32_t flags, uint32_t n_wg,
                              uint32_t epoch, hipStream_t stream) {
    (void)hipGetLastError();
    if (n_wg < 1 || n_wg > kSrvMaxWgs || (n_wg > 1 && !disp_dev)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(scan_server_kernel, dim3(n_wg), dim3(kSrvThreads), 0, stream, mb_dev, req_dev, disp_dev,
                       slot_dev, hslot_dev, table_rot, thr, last_seq, idle_ticks, flags, n_wg, epoch);
    return hipGetLastError();
}

hipError_t launch_scan_exact(const uint8_t* data, uint64_t len, const uint8_t* pre,
                             uint32_t pre_len, const uint64_t* susp,
                             const unsigned long long* nsusp, uint64_t susp_cap, uint64_t ext_first,
                             uint64_t ext_count, int head, uint32_t mask, uint32_t minimum,
                             uint64_t base, uint64_t* cand, unsigned long long* ncand,
                             uint64_t cand_cap, uint64_t max_items, hipStream_t stream) {
    (void)hipGetLastError();
    // one item per wave; at most 2 workgroups per CU (one flush atomic each)
    uint64_t blocks = (max_items + kExactWaves - 1) / kExactWaves;
    if (blocks < 1) blocks = 1;
    if (blocks > 512) blocks = 512;
    hipLaunchKernelGGL(scan_exact_kernel, dim3((unsigned)blocks), dim3(kExactWaves * 64), 0, stream, data, len,
                       pre, pre_len, susp, nsusp, susp_cap, ext_first, ext_count, head, mask,
                       minimum, base, cand, ncand, cand_cap);
    return hipGetLastError();
}

hipError_t launch_resolve(const uint64_t* C, uint32_t m, const ResolveParams& p, uint32_t* nxt,
                          uint32_t* jtmp, uint64_t* nforced, uint32_t* on, uint64_t* cnt,
                          uint64_t* off, void* scan_tmp, size_t scan_tmp_bytes, uint64_t* out,
                          uint64_t out_cap, uint64_t* res, hipStream_t stream, const uint64_t* m_dev,
                          uint32_t m_base) {
    // m_dev: the node count lives on the device (m is its upper bound, grids sized by it)
    const uint32_t n = m + 2;
    const unsigned blocks = (n + 255) / 256;
    (void)hipGetLastError();
    // nxt, and its copy in jtmp that the pointer doubling consumes (nxt is kept for emission)
    uint32_t* ja = jtmp;
    uint32_t* jb = jtmp + n;
    hipLaunchKernelGGL(resolve_next_kernel, dim3(blocks), dim3(256), 0, stream, C, m, p, nxt,
                       nforced, on, m_dev, m_base, ja);
    for (uint64_t span = 1; span < n; span <<= 3) {  // three rounds per launch
        hipLaunchKernelGGL(resolve_double3_kernel, dim3(blocks), dim3(256), 0, stream, n, ja, jb, on, m_dev, m_base);
        uint32_t* t = ja;
        ja = jb;
        jb = t;
    }
    hipLaunchKernelGGL(resolve_count_kernel, dim3(blocks), dim3(256), 0, stream, m, nxt, nforced,
                       on, cnt, m_dev, m_base);
    size_t tb = scan_tmp_bytes;
    hipError_t e = exclusive_sum_u64(scan_tmp, &tb, cnt, off, m + 1, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(resolve_emit_kernel, dim3(blocks), dim3(256), 0, stream, C, m, p, nxt,
                       nforced, on, cnt, off, out, out_cap, res, m_dev, m_base);
    return hipGetLastError();
}

hipError_t launch_resolve_small(const uint64_t* newc, uint32_t nnew, uint64_t* C, uint32_t np,
                                const ResolveParams& p, uint32_t* nxt, uint64_t* nforced,
                                uint64_t* out, uint64_t out_cap, uint64_t* out_host,
                                uint64_t host_cap, uint64_t* keep_host, uint64_t keep_cap,
                                uint64_t* res, uint64_t* res_host, hipStream_t stream,
                                const unsigned long long* counts, uint64_t susp_cap, uint64_t cand_cap,
                                uint64_t* counts_host, const uint8_t* tail_src, uint8_t* tail_host,
                                uint32_t tail_len) {
    if ((uint64_t)np + (counts ? 0 : nnew) + 2 > kSmallResolveMax) return hipErrorInvalidValue;
    (void)hipGetLastError();
    FusedScanArgs fa{};
    fa.counts = counts;
    fa.susp_cap = susp_cap;
    fa.cand_cap = cand_cap;
    fa.counts_host = counts_host;
    fa.tail_src = tail_src;
    fa.tail_host = tail_host;
    fa.tail_len = tail_len;
    hipLaunchKernelGGL(resolve_small_kernel<0>, dim3(1), dim3(kSmallThreads), 0, stream, newc,
                       nnew, C, np, p, nxt, nforced, out, out_cap, out_host, host_cap, keep_host,
                       keep_cap, res, res_host, fa);
    return hipGetLastError();
}

hipError_t launch_scan_resolve_small(const FusedScanArgs& fa, int resolve, uint64_t* C,
                                     uint32_t np, const ResolveParams& p, uint32_t* nxt,
                                     uint64_t* nforced, uint64_t* out, uint64_t out_cap,
                                     uint64_t* out_host, uint64_t host_cap, uint64_t* keep_host,
                                     uint64_t keep_cap, uint64_t* res, uint64_t* res_host,
                                     hipStream_t stream) {
    if ((uint64_t)np + 2 > kSmallResolveMax || fa.nblk * kBlockBytes > kFusedMaxBytes + kBlockBytes)
        return hipErrorInvalidValue;
    (void)hipGetLastError();
    if (fa.nblk)
        hipLaunchKernelGGL(scan_blocks_kernel, dim3((unsigned)((fa.nblk + 3) / 4)), dim3(256), 0,
                           stream, fa.data, fa.len, fa.pre, fa.pre_len, fa.mask, fa.minimum,
                           const_cast<uint4*>(fa.hits), fa.nblk);
    if (resolve)
        hipLaunchKernelGGL(resolve_small_kernel<1>, dim3(1), dim3(kSmallThreads), 0, stream,
                           nullptr, 0u, C, np, p, nxt, nforced, out, out_cap, out_host, host_cap,
                           keep_host, keep_cap, res, res_host, fa);
    else
        hipLaunchKernelGGL(resolve_small_kernel<2>, dim3(1), dim3(kSmallThreads), 0, stream,
                           nullptr, 0u, C, np, p, nxt, nforced, out, out_cap, out_host, host_cap,
                           keep_host, keep_cap, res, res_host, fa);
    return hipGetLastError();
}

hipError_t launch_gen(uint64_t* out, uint64_t nwords, uint64_t seed, uint64_t word_offset,
                      int kind, hipStream_t stream) {
    (void)hipGetLastError();
    uint64_t blocks = (nwords + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, out, nwords,
                       seed, word_offset, kind);
    return hipGetLastError();
}

}  // namespace pbs

#ifdef PBS_SCAN_PROBE
// probe build only (scripts/microbench/scan_probe.py): the per-wave finish times of the
// last scan_main launch, wall_clock64 ticks (100 MHz)
extern "C" int pbs_fused_probe_read(uint64_t* out) {  // 4 * 4096: start, tiles done, done, SIMD
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pbs::g_fused_probe), sizeof(pbs::g_fused_probe)) == hipSuccess
               ? 0 : -1;
}
extern "C" int pbs_scan_probe_read(uint64_t* out) {  // 2 * 4096: finish, then start times
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pbs::g_scan_probe), sizeof(pbs::g_scan_probe)) == hipSuccess
               ? 0 : -1;
}
#endif
