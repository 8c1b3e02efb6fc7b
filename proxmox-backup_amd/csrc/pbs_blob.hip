// Per-chunk blob CRC on the GPU: `DataBlob::compute_crc`
// (pbs-datastore/src/data_blob.rs:70-75), crc32fast's CRC-32/ISO-HDLC over the blob
// payload, set by `DataBlob::encode` (:87-179) and checked by `verify_crc` (:78-84).
// C ABI: include/pbs_blob.h.
//
// CRC-32 is linear over GF(2), so one chunk is split over the 256 lanes of a workgroup
// instead of one lane walking it byte by byte.  The chunk is cut into 4096-byte rows at
// absolute (4096-aligned) addresses; lane t owns the 16-byte word at 16 t of every row,
// loaded as one dwordx4 (a row is one fully coalesced 4 KiB read of the workgroup).
// Lane t computes the raw CRC (register 0, no final XOR) of ITS bytes with all other
// lanes' bytes read as zero.  Going from one of its words to the next is one linear map:
// absorb 16 bytes, then 4080 zero bytes, r' = F(r ^ w) with
//     F(x) = XOR_i TF[i][byte i of x],  TF[i][v] = T[v] * x^(8 (4095 - i)) mod P,
// 16 LDS lookups per 16 bytes (the reference's crc32fast does 1 table step per byte on
// one core).  A lane's LAST word is absorbed byte by byte, so its register covers the
// chunk up to c_t <= end exactly; a multiply by x^(8 (end - c_t)) mod P (table X8, a
// 32-step carry-less product) aligns every lane to the chunk end, and the XOR of the 256
// registers is the raw CRC of the chunk.  Zero bytes in front of the chunk leave a zero
// register unchanged, so rows need not start at the chunk; the CRC's init value
// 0xFFFFFFFF is the same as XOR-ing 0xFF into the first four message bytes, which the
// lanes holding them do at load time (chunks shorter than 4 bytes: one lane, serially).
// Only bytes inside [start, end) are ever read: words crossing either end are gathered
// byte by byte.  The workgroups are persistent (the 17 KiB of tables are staged into LDS
// once per workgroup) and take the chunks longest first: the first gridDim.x
// statically, then each draws its next chunk from a per-stream device counter, so
// workgroups on faster CUs take more (64 GiB / 4 MiB: 11.01 -> 10.66 ms against the
// static stride, profiles/r01/blob/ab_crc_dynamic.log; PBS_CRC_DYN=0 restores it).
//
// Roofline: HBM, L bytes read per chunk; per 16 bytes one dwordx4 load, 16 ds_read_b32
// and ~40 VALU (byte extract, address, XOR).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "dev_arena.h"
#include <numeric>
#include <thread>
#include <vector>

#include "pbs_blob.h"
#include "pbs_chunker.h"
#include "pbs_chunker_internal.h"

namespace pbs {
namespace {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected 0x04C11DB7
constexpr int kRow = 4096;
constexpr int kCrcThreads = kRow / 16;  // one 16-byte word per lane and row
constexpr int kCrcGroupsPerCu = 8;

struct CrcTables {
    uint32_t tf[16 * 256];  // TF[i][v]: byte v at position i of a word, then the row's zeros
    uint32_t t[256];        // the byte-at-a-time table
    uint32_t x8[kRow];      // x^(8 d) mod P, d < 4096 (x^0 = bit 31, reflected)
};

// a(x) * b(x) mod P, reflected (zlib's multmodp, fixed 32 steps)
__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) {
        p ^= b & (0u - ((a >> k) & 1u));
        b = (b >> 1) ^ (kPoly & (0u - (b & 1u)));
    }
    return p;
}

void make_tables(CrcTables& tb) {
    for (uint32_t v = 0; v < 256; ++v) {
        uint32_t c = v;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
        tb.t[v] = c;
    }
    tb.x8[0] = 1u << 31;
    for (int d = 1; d < kRow; ++d) {
        uint32_t p = tb.x8[d - 1];
        for (int k = 0; k < 8; ++k) p = (p >> 1) ^ (kPoly & (0u - (p & 1u)));
        tb.x8[d] = p;
    }
    for (int i = 0; i < 16; ++i)
        for (int v = 0; v < 256; ++v) tb.tf[i * 256 + v] = multmodp(tb.x8[kRow - 1 - i], tb.t[v]);
}

// device copy of the tables, made once per device and kept for the process
const CrcTables* device_tables(int dev) {
    static std::mutex mu;
    static std::map<int, CrcTables*> tabs;
    std::lock_guard<std::mutex> g(mu);
    auto it = tabs.find(dev);
    if (it != tabs.end()) return it->second;
    static CrcTables host;
    static bool made = false;
    if (!made) {
        make_tables(host);
        made = true;
    }
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    CrcTables* d = nullptr;
    bool ok = hipMalloc(&d, sizeof(CrcTables)) == hipSuccess;
    // landed before any launch on another stream: copied on a private non-blocking stream
    // and waited for there (the null stream would also wait for every blocking stream's
    // work -- e.g. the pipeline's persistent digest queue, pbs_pipeline.cpp)
    hipStream_t cs = nullptr;
    if (ok && (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess ||
               hipMemcpyAsync(d, &host, sizeof(CrcTables), hipMemcpyHostToDevice, cs) != hipSuccess ||
               hipStreamSynchronize(cs) != hipSuccess)) {
        (void)hipFree(d);
        ok = false;
    }
    if (cs) (void)hipStreamDestroy(cs);
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return nullptr;
    tabs[dev] = d;
    return d;
}

// counter of the dynamic chunk order, one per (device, stream), allocated on the stream's
// own device and zeroed by a 8-byte memset on that stream before every launch (launches
// on one stream are ordered, so a counter is never shared by two running launches, and
// an aborted launch cannot leave a stale value behind).  The null stream and
// hipStreamPerThread are the same handle on every device and in every thread, so their
// key also names the calling thread: two threads on the null stream would otherwise
// interleave memset, memset, launch, launch on one counter.  release_stream_counter()
// frees a stream's entry before the stream is destroyed (pbs_pipeline.cpp).
struct CtrKey {
    int dev;
    hipStream_t st;
    std::thread::id th;
    bool operator<(const CtrKey& o) const {
        if (dev != o.dev) return dev < o.dev;
        if (st != o.st) return st < o.st;
        return th < o.th;
    }
};
std::mutex g_ctr_mu;
std::map<CtrKey, unsigned long long*> g_ctrs;

CtrKey ctr_key(hipStream_t st, int dev) {
    const bool shared = st == nullptr || st == hipStreamPerThread;
    return CtrKey{dev, st, shared ? std::this_thread::get_id() : std::thread::id()};
}

// A thread's counters of the shared stream handles (null stream, hipStreamPerThread) are
// freed when the thread exits (or by release_thread_counters), so threads that come and
// go leave no device allocations behind.
void free_thread_counters(std::thread::id th) {
    std::lock_guard<std::mutex> g(g_ctr_mu);
    for (auto it = g_ctrs.begin(); it != g_ctrs.end();) {
        if (it->first.th == th && th != std::thread::id()) {
            int cur = -1;
            const bool have = hipGetDevice(&cur) == hipSuccess;
            if (hipSetDevice(it->first.dev) == hipSuccess) (void)hipFree(it->second);
            if (have) (void)hipSetDevice(cur);
            it = g_ctrs.erase(it);
        } else {
            ++it;
        }
    }
}
struct ThreadCounters {
    bool armed = false;
    ~ThreadCounters() {
        if (armed) free_thread_counters(std::this_thread::get_id());
    }
};
thread_local ThreadCounters t_counters;
void arm_thread_counters() { t_counters.armed = true; }

unsigned long long* stream_counter(hipStream_t st, int dev) {
    const CtrKey key = ctr_key(st, dev);
    if (key.th != std::thread::id()) arm_thread_counters();
    std::lock_guard<std::mutex> g(g_ctr_mu);
    auto it = g_ctrs.find(key);
    if (it != g_ctrs.end()) return it->second;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    unsigned long long* d = nullptr;
    const bool ok = hipMalloc(&d, sizeof(unsigned long long)) == hipSuccess;
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return nullptr;
    g_ctrs[key] = d;
    return d;
}

ArenaPool& crc_pool() {
    static ArenaPool* p = new ArenaPool;  // never destroyed (HIP may be torn down first at exit)
    return *p;
}

}  // namespace

void release_thread_counters() { free_thread_counters(std::this_thread::get_id()); }

void release_stream_counter(hipStream_t st) {
    int dev = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess) return;
    std::lock_guard<std::mutex> g(g_ctr_mu);
    auto it = g_ctrs.find(ctr_key(st, dev));
    if (it == g_ctrs.end()) return;
    (void)hipFree(it->second);
    g_ctrs.erase(it);
}

namespace {

// byte p of the chunk's message: zero outside [as, ae), the first four bytes XOR 0xFF
__device__ __forceinline__ uint32_t msg_byte(uintptr_t p, uintptr_t as, uintptr_t ae) {
    if (p < as || p >= ae) return 0;
    const uint32_t b = *reinterpret_cast<const uint8_t*>(p);
    return p < as + 4 ? b ^ 0xFFu : b;
}

__device__ __forceinline__ uint4 gather_word(uintptr_t w, uintptr_t as, uintptr_t ae) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = msg_byte(w + 4 * j, as, ae) | msg_byte(w + 4 * j + 1, as, ae) << 8 |
               msg_byte(w + 4 * j + 2, as, ae) << 16 | msg_byte(w + 4 * j + 3, as, ae) << 24;
    return make_uint4(v[0], v[1], v[2], v[3]);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// streaming 16-byte load (read once: non-temporal)
__device__ __forceinline__ uint4 load_nt(uintptr_t w) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t lut4(const uint32_t* tf, int i, uint32_t x) {
    return tf[(i + 0) * 256 + (x & 0xFFu)] ^ tf[(i + 1) * 256 + ((x >> 8) & 0xFFu)] ^
           tf[(i + 2) * 256 + ((x >> 16) & 0xFFu)] ^ tf[(i + 3) * 256 + (x >> 24)];
}

// one row step: absorb the 16-byte word (register XOR-ed into its first 4 bytes), then
// the 4080 zero bytes up to the lane's next word
__device__ __forceinline__ uint32_t row_step(const uint32_t* tf, uint32_t r, uint4 w) {
    return lut4(tf, 0, w.x ^ r) ^ lut4(tf, 4, w.y) ^ lut4(tf, 8, w.z) ^ lut4(tf, 12, w.w);
}

__global__ __launch_bounds__(kCrcThreads) void crc32_chunks_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint32_t* __restrict__ order, uint64_t n, const CrcTables* __restrict__ tab,
    uint32_t* __restrict__ out, unsigned long long* __restrict__ next_ctr, uint64_t skip) {
    __shared__ __attribute__((aligned(16))) uint32_t tf[16 * 256];
    __shared__ uint32_t tb[256];
    __shared__ uint32_t red[kCrcThreads / 64];
    __shared__ uint64_t s_next;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 16 * 256 / 4; i += kCrcThreads)
        reinterpret_cast<uint4*>(tf)[i] = reinterpret_cast<const uint4*>(tab->tf)[i];
    tb[tid] = tab->t[tid];
    __syncthreads();

    // chunk order: the first gridDim.x statically, then (next_ctr) each workgroup draws
    // its next chunk from a counter, so workgroups on faster CUs take more
    for (uint64_t k = blockIdx.x; k < n;) {
        if (next_ctr) {
            if (tid == 0) s_next = gridDim.x + atomicAdd(next_ctr, 1ull);
        }
        const uint64_t ci = order ? order[k] : k;
        const uint64_t s = bounds[ci] - base + skip, e = bounds[ci + 1] - base;
        if (e - s < 4) {  // shorter than the init register: serially, one lane
            if (tid == 0) {
                uint32_t r = 0xFFFFFFFFu;
                for (uint64_t p = s; p < e; ++p) r = (r >> 8) ^ tb[(r ^ data[p]) & 0xFFu];
                out[ci] = ~r;
            }
            if (next_ctr) {
                __syncthreads();
                k = s_next;
                __syncthreads();
            } else {
                k += gridDim.x;
            }
            continue;
        }
        const uintptr_t as = reinterpret_cast<uintptr_t>(data) + s;
        const uintptr_t ae = reinterpret_cast<uintptr_t>(data) + e;
        const uintptr_t w0 = (as & ~(uintptr_t)(kRow - 1)) + 16 * tid;  // row 0 word
        uint32_t r = 0;
        if (w0 < ae) {
            const uint64_t kf = (w0 + 16 > as) ? 0 : 1;
            const uint64_t kl = (ae - 1 - w0) / kRow;
            if (kf <= kl) {
                uintptr_t w = w0 + kf * kRow;
                uint64_t rows = kl - kf;  // words before the last one
                if (rows) {               // the first word may cross the start / init bytes
                    r = row_step(tf, r, gather_word(w, as, ae));
                    w += kRow;
                    --rows;
                }
                // middle words: entirely inside the chunk, past the init bytes
                for (; rows >= 4; rows -= 4, w += 4 * kRow) {
                    uint4 v[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        v[j] = load_nt(w + j * kRow);
#pragma unroll
                    for (int j = 0; j < 4; ++j) r = row_step(tf, r, v[j]);
                }
                for (; rows; --rows, w += kRow)
                    r = row_step(tf, r, load_nt(w));
                // last word: byte by byte up to the chunk end, then align to the end
                const uintptr_t c = w + 16 < ae ? w + 16 : ae;
                for (uintptr_t p = w; p < c; ++p) r = (r >> 8) ^ tb[(r ^ msg_byte(p, as, ae)) & 0xFFu];
                if (r) r = multmodp(tab->x8[ae - c], r);
            }
        }
        // XOR of the 256 lane registers
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) r ^= __shfl_xor(r, off, 64);
        if ((tid & 63) == 0) red[tid >> 6] = r;
        __syncthreads();
        if (tid == 0) {
            uint32_t x = 0;
#pragma unroll
            for (int i = 0; i < kCrcThreads / 64; ++i) x ^= red[i];
            out[ci] = ~x;
        }
        __syncthreads();  // red (and s_next) are reused by the next chunk
        if (next_ctr) {
            k = s_next;
            __syncthreads();
        } else {
            k += gridDim.x;
        }
    }
}

}  // namespace
}  // namespace pbs

using namespace pbs;

// Blob images [bounds[i], bounds[i+1]) with a `skip`-byte header: the CRC of each payload
// (pbs_zstd.hip; static chunk order, the blobs are in stream order).
hipError_t pbs::launch_crc32_skip(const uint8_t* data, const uint64_t* bounds_dev, uint64_t n, uint64_t skip,
                                  uint32_t* out, hipStream_t st) {
    int dev = 0, ncu = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return hipErrorInvalidDevice;
    const CrcTables* tab = device_tables(dev);
    if (!tab) return hipErrorOutOfMemory;
    const unsigned grid = (unsigned)std::min<uint64_t>(n, (uint64_t)ncu * kCrcGroupsPerCu);
    unsigned long long* ctr = nullptr;
    if (n > grid) {
        ctr = stream_counter(st, dev);
        if (!ctr) return hipErrorOutOfMemory;
        const hipError_t e = hipMemsetAsync(ctr, 0, sizeof(unsigned long long), st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(crc32_chunks_kernel, dim3(grid), dim3(kCrcThreads), 0, st, data, (uint64_t)0, bounds_dev,
                       (const uint32_t*)nullptr, n, tab, out, ctr, skip);
    return hipGetLastError();
}

extern "C" int pbs_crc32_chunks_async(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                      const uint64_t* bounds_dev, const uint32_t* order_dev, size_t n,
                                      uint32_t* crcs_dev, void* hip_stream) {
    if (n == 0) return PBS_OK;
    if (!bounds_dev || !crcs_dev || (data_len && !dev_data)) return PBS_ERR_INVALID;
    // the stream's own device (not the calling thread's current one) holds the tables and
    // the counter
    const hipStream_t st = (hipStream_t)hip_stream;
    int dev = 0, ncu = 0;
    if (hipStreamGetDevice(st, &dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return PBS_ERR_NO_DEVICE;
    const CrcTables* tab = device_tables(dev);
    if (!tab) return PBS_ERR_NOMEM;
    (void)hipGetLastError();
    const unsigned grid = (unsigned)std::min<uint64_t>(n, (uint64_t)ncu * kCrcGroupsPerCu);
    const char* e = std::getenv("PBS_CRC_DYN");  // A/B knob
    unsigned long long* ctr = nullptr;
    if (n > grid && !(e && e[0] == '0')) {
        ctr = stream_counter(st, dev);
        if (!ctr) return PBS_ERR_NOMEM;
        if (hipMemsetAsync(ctr, 0, sizeof(unsigned long long), st) != hipSuccess) return PBS_ERR_HIP;
    }
    hipLaunchKernelGGL(crc32_chunks_kernel, dim3(grid), dim3(kCrcThreads), 0, (hipStream_t)hip_stream,
                       dev_data, base, bounds_dev, order_dev, (uint64_t)n, tab, crcs_dev, ctr, (uint64_t)0);
    return hipGetLastError() == hipSuccess ? PBS_OK : PBS_ERR_HIP;
}

extern "C" int pbs_crc32_chunks_device(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                       const uint64_t* bounds, size_t n, uint32_t* crcs, void* hip_stream) {
    if (n == 0) return PBS_OK;
    if (!bounds || !crcs) return PBS_ERR_INVALID;
    for (size_t i = 0; i < n; ++i)  // every chunk inside the device range, ascending
        if (bounds[i] > bounds[i + 1] || bounds[i] < base || bounds[i + 1] - base > data_len)
            return PBS_ERR_INVALID;
    std::vector<uint32_t> order(n);  // longest first: the strided workgroups finish together
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return bounds[a + 1] - bounds[a] > bounds[b + 1] - bounds[b];
    });
    hipStream_t st = (hipStream_t)hip_stream;
    int sdev = 0;
    if (hipStreamGetDevice(st, &sdev) != hipSuccess) return PBS_ERR_NO_DEVICE;
    DeviceGuard dg(sdev);  // the work area belongs on the stream's device
    if (!dg.ok) return PBS_ERR_NO_DEVICE;
    ArenaLease ar(crc_pool(), sdev);
    uint64_t* d_bounds = ar->get<uint64_t>(0, (n + 1) * 8);
    uint32_t* d_order = ar->get<uint32_t>(1, n * 4);
    uint32_t* d_crc = ar->get<uint32_t>(2, n * 4);
    int rc = PBS_OK;
    if (!d_bounds || !d_order || !d_crc) {
        rc = PBS_ERR_NOMEM;
    } else if (hipMemcpyAsync(d_bounds, bounds, (n + 1) * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
               hipMemcpyAsync(d_order, order.data(), n * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = PBS_ERR_HIP;
    } else {
        rc = pbs_crc32_chunks_async(dev_data, data_len, base, d_bounds, d_order, n, d_crc, hip_stream);
        if (rc == PBS_OK && hipMemcpyAsync(crcs, d_crc, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
            rc = PBS_ERR_HIP;
    }
    if (hipStreamSynchronize(st) != hipSuccess && rc == PBS_OK) rc = PBS_ERR_HIP;  // (before the arena goes back)
    return rc;
}

extern "C" uint64_t pbs_debug_arena_allocs(void) { return g_arena_allocs.load(); }

extern "C" uint32_t pbs_crc32(uint32_t crc, const uint8_t* data, size_t len) {
    static CrcTables tb;
    static std::once_flag once;
    std::call_once(once, [] { make_tables(tb); });
    uint32_t r = ~crc;
    for (size_t i = 0; i < len; ++i) r = (r >> 8) ^ tb.t[(r ^ data[i]) & 0xFFu];
    return ~r;
}

extern "C" size_t pbs_blob_encode_uncompressed(const uint8_t* data, size_t len, uint32_t crc, uint8_t* out,
                                               size_t cap) {
    // UNCOMPRESSED_BLOB_MAGIC_1_0, pbs-datastore/src/file_formats.rs:9
    static const uint8_t kMagic[8] = {66, 171, 56, 7, 190, 131, 112, 161};
    if (len > (128u << 20) || !out || cap < len + PBS_BLOB_HEADER_SIZE || (len && !data)) return 0;
    std::memcpy(out, kMagic, 8);
    for (int i = 0; i < 4; ++i) out[8 + i] = (uint8_t)(crc >> (8 * i));
    if (len) std::memcpy(out + PBS_BLOB_HEADER_SIZE, data, len);
    return len + PBS_BLOB_HEADER_SIZE;
}
