// In-house device sort and scan for the chunker's multi-launch paths (the multi-kernel
// resolve's candidate sort and cut-count scan, the sharded phase A, and the known-chunk
// test of pbs_digest.hip).  The one-launch pass (scan_fused.h) needs neither: its
// candidates come out of the tile records already in stream order.
//
// radix_sort: stable LSD radix sort of u64 keys (optionally carrying u32 values) over bits
// [begin_bit, end_bit), 8 bits per pass, three launches per pass:
//   histogram  one workgroup per 4096-key tile counts its digits in LDS -> hist[digit][tile]
//   scan       exclusive sum over hist (digit-major): every (digit, tile) slice's offset
//   scatter    the tile again, 16 rounds of 256 keys in input order; a key's rank among
//              equal digits is the running count of earlier rounds + the counts of the
//              earlier waves of its round + its rank inside its wave (an 8-ballot digit
//              match: no LDS atomics, so the sort is stable)
// scan: the classic three-phase device scan (tile reduce, scan of the tile totals in one
// workgroup, tile scan with its offset), for u32/u64 sums and u32 max.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "pbs_chunker_internal.h"

namespace pbs {
namespace {

constexpr int kSortThreads = 256;
constexpr int kSortPer = 16;                       // keys per thread
constexpr int kSortTile = kSortThreads * kSortPer;  // 4096 keys per workgroup
constexpr int kRadix = 256;

__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                                  int shift, uint32_t* __restrict__ hist,
                                                                  uint32_t ntiles) {
    __shared__ uint32_t h[kRadix];
    const uint32_t tid = threadIdx.x, b = blockIdx.x;
    h[tid] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)b * kSortTile;
#pragma unroll 4
    for (int r = 0; r < kSortPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kSortThreads + tid;
        if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[(uint64_t)tid * ntiles + b] = h[tid];
}

template <bool PAIRS>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ vout, uint64_t n, int shift, const uint32_t* __restrict__ offs, uint32_t ntiles) {
    __shared__ uint32_t run[kRadix];                             // keys of each digit placed so far
    __shared__ uint32_t wcnt[kSortThreads / 64][kRadix];         // this round's per-wave digit counts
    const uint32_t tid = threadIdx.x, b = blockIdx.x, lane = tid & 63, wave = tid >> 6;
    run[tid] = offs[(uint64_t)tid * ntiles + b];
    const unsigned long long below = (1ull << lane) - 1;
    const uint64_t base = (uint64_t)b * kSortTile;
    for (int r = 0; r < kSortPer; ++r) {
#pragma unroll
        for (int w = 0; w < kSortThreads / 64; ++w) wcnt[w][tid] = 0;
        const uint64_t i = base + (uint64_t)r * kSortThreads + tid;
        const bool v = i < n;
        const uint64_t k = v ? kin[i] : 0;
        const uint32_t d = (uint32_t)(k >> shift) & 0xFFu;
        unsigned long long eq = __ballot(v);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const unsigned long long m = __ballot((d >> bit) & 1u);
            eq &= ((d >> bit) & 1u) ? m : ~m;
        }
        __syncthreads();  // wcnt zeroed
        const uint32_t rank = (uint32_t)__popcll(eq & below);
        if (v && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(eq);
        __syncthreads();
        if (v) {
            uint32_t pos = run[d] + rank;
            for (uint32_t w = 0; w < wave; ++w) pos += wcnt[w][d];
            kout[pos] = k;
            if constexpr (PAIRS) vout[pos] = vin[i];
        }
        __syncthreads();  // every key of the round placed before `run` moves on
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < kSortThreads / 64; ++w) add += wcnt[w][tid];
        run[tid] += add;
        __syncthreads();
    }
}

// ---- scans ---------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;
constexpr int kScanTile = kScanThreads * kScanPer;

template <class T, bool MAX>
__device__ __forceinline__ T op(T a, T b) {
    if constexpr (MAX) return a > b ? a : b;
    else return a + b;
}

// inclusive scan of one value per thread over the workgroup; total in *total
template <class T, bool MAX>
__device__ __forceinline__ T block_incl(T x, T* wsum, T* total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x = op<T, MAX>(x, y);
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    T before = T(0);
    for (uint32_t w = 0; w < wave; ++w) before = op<T, MAX>(before, wsum[w]);
    T all = T(0);
    for (uint32_t w = 0; w < blockDim.x / 64; ++w) all = op<T, MAX>(all, wsum[w]);
    __syncthreads();
    *total = all;
    return op<T, MAX>(before, x);
}

template <class T, bool MAX>
__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(const T* __restrict__ in, uint64_t n,
                                                                   T* __restrict__ part) {
    __shared__ T wsum[kScanThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    T x = T(0);
    for (int q = 0; q < kScanPer; ++q)
        if (base + q < n) x = op<T, MAX>(x, in[base + q]);
    T total;
    (void)block_incl<T, MAX>(x, wsum, &total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

// exclusive scan of the tile totals in place, one workgroup of 1024 threads
template <class T, bool MAX>
__global__ __launch_bounds__(1024) void scan_parts_kernel(T* __restrict__ part, uint64_t np) {
    __shared__ T wsum[1024 / 64];
    __shared__ T incl_s[1024];
    T carry = T(0);  // the identity of both ops on unsigned values
    for (uint64_t c0 = 0; c0 < np; c0 += 1024) {
        const uint64_t i = c0 + threadIdx.x;
        const T x = i < np ? part[i] : T(0);
        T total;
        incl_s[threadIdx.x] = block_incl<T, MAX>(x, wsum, &total);
        __syncthreads();
        if (i < np) part[i] = op<T, MAX>(carry, threadIdx.x ? incl_s[threadIdx.x - 1] : T(0));
        carry = op<T, MAX>(carry, total);
        __syncthreads();
    }
}

template <class T, bool MAX, bool EXCL>
__global__ __launch_bounds__(kScanThreads) void scan_tile_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                                 uint64_t n, const T* __restrict__ part) {
    __shared__ T wsum[kScanThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    T v[kScanPer];
    T x = T(0);
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        v[q] = base + q < n ? in[base + q] : T(0);
        x = op<T, MAX>(x, v[q]);
    }
    T total;
    const T incl = block_incl<T, MAX>(x, wsum, &total);
    // this thread's exclusive start: tile offset (op) the preceding threads' total
    T run;
    if constexpr (MAX) {
        const T prev = __shfl_up(incl, 1, 64);
        const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        T before = T(0);
        for (uint32_t w = 0; w < wave; ++w) before = op<T, MAX>(before, wsum[w]);
        run = op<T, MAX>(part[blockIdx.x], lane ? op<T, MAX>(before, prev) : before);
    } else {
        run = part[blockIdx.x] + (incl - x);
    }
#pragma unroll
    for (int q = 0; q < kScanPer; ++q) {
        if (base + q >= n) break;
        const T nx = op<T, MAX>(run, v[q]);
        out[base + q] = EXCL ? run : nx;
        run = nx;
    }
}

template <class T, bool MAX, bool EXCL>
hipError_t scan_impl(const T* in, T* out, uint64_t n, void* tmp, size_t* tmp_bytes, hipStream_t st) {
    const uint64_t nt = (n + kScanTile - 1) / kScanTile;
    const size_t need = std::max<uint64_t>(nt, 1) * sizeof(T);
    if (!tmp) {
        *tmp_bytes = need;
        return hipSuccess;
    }
    if (*tmp_bytes < need) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    T* part = static_cast<T*>(tmp);
    (void)hipGetLastError();
    hipLaunchKernelGGL((scan_reduce_kernel<T, MAX>), dim3((unsigned)nt), dim3(kScanThreads), 0, st, in, n, part);
    hipLaunchKernelGGL((scan_parts_kernel<T, MAX>), dim3(1), dim3(1024), 0, st, part, nt);
    hipLaunchKernelGGL((scan_tile_kernel<T, MAX, EXCL>), dim3((unsigned)nt), dim3(kScanThreads), 0, st, in, out,
                       n, part);
    return hipGetLastError();
}

}  // namespace

hipError_t exclusive_sum_u64(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, uint32_t n,
                             hipStream_t stream) {
    return scan_impl<unsigned long long, false, true>(
        reinterpret_cast<const unsigned long long*>(in), reinterpret_cast<unsigned long long*>(out), n, tmp,
        tmp_bytes, stream);
}

hipError_t inclusive_max_u32(void* tmp, size_t* tmp_bytes, const uint32_t* in, uint32_t* out, uint64_t n,
                             hipStream_t stream) {
    return scan_impl<uint32_t, true, false>(in, out, n, tmp, tmp_bytes, stream);
}

hipError_t radix_sort(void* tmp, size_t* tmp_bytes, const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                      uint32_t* vout, uint64_t n, int begin_bit, int end_bit, hipStream_t st) {
    const uint64_t ntiles = std::max<uint64_t>((n + kSortTile - 1) / kSortTile, 1);
    const uint64_t nh = ntiles * kRadix;
    size_t scan_tmp = 0;
    (void)scan_impl<uint32_t, false, true>(nullptr, nullptr, nh, nullptr, &scan_tmp, st);
    // [alt keys | alt values | hist | offsets | scan partials]
    const size_t kb = (n * 8 + 255) & ~(size_t)255, vb = vin ? ((n * 4 + 255) & ~(size_t)255) : 0;
    const size_t hb = (nh * 4 + 255) & ~(size_t)255;
    const size_t need = kb + vb + 2 * hb + scan_tmp;
    if (!tmp) {
        *tmp_bytes = need;
        return hipSuccess;
    }
    if (*tmp_bytes < need || ntiles > 0xFFFFFFFFull) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    uint8_t* t = static_cast<uint8_t*>(tmp);
    uint64_t* kalt = reinterpret_cast<uint64_t*>(t);
    uint32_t* valt = vin ? reinterpret_cast<uint32_t*>(t + kb) : nullptr;
    uint32_t* hist = reinterpret_cast<uint32_t*>(t + kb + vb);
    uint32_t* offs = reinterpret_cast<uint32_t*>(t + kb + vb + hb);
    void* stmp = t + kb + vb + 2 * hb;
    const int passes = std::max(1, (end_bit - begin_bit + 7) / 8);
    const uint64_t* ks = kin;
    const uint32_t* vs = vin;
    for (int p = 0; p < passes; ++p) {
        // the last pass writes the output: every other one before it the alternate buffer
        const bool to_out = ((passes - 1 - p) & 1) == 0;
        uint64_t* kd = to_out ? kout : kalt;
        uint32_t* vd = to_out ? vout : valt;
        const int shift = begin_bit + 8 * p;
        (void)hipGetLastError();
        hipLaunchKernelGGL(radix_hist_kernel, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st, ks, n, shift, hist,
                           (uint32_t)ntiles);
        size_t sb = scan_tmp;
        hipError_t e = scan_impl<uint32_t, false, true>(hist, offs, nh, stmp, &sb, st);
        if (e != hipSuccess) return e;
        if (vin)
            hipLaunchKernelGGL(radix_scatter_kernel<true>, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st, ks, kd,
                               vs, vd, n, shift, offs, (uint32_t)ntiles);
        else
            hipLaunchKernelGGL(radix_scatter_kernel<false>, dim3((unsigned)ntiles), dim3(kSortThreads), 0, st, ks,
                               kd, nullptr, nullptr, n, shift, offs, (uint32_t)ntiles);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        ks = kd;
        vs = vd;
    }
    return hipSuccess;
}

hipError_t sort_u64(void* tmp, size_t* tmp_bytes, const uint64_t* in, uint64_t* out, uint32_t n, int end_bit,
                    hipStream_t stream) {
    return radix_sort(tmp, tmp_bytes, in, out, nullptr, nullptr, n, 0, end_bit, stream);
}

}  // namespace pbs
