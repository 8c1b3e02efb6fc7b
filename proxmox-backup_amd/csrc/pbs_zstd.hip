// Compressed DataBlob images of every chunk on the GPU (second
// half): `DataBlob::encode(data, None, compress = true)` (pbs-datastore/src/data_blob.rs:
// 139-176) -- a zstd frame of the chunk (`zstd::stream::copy_encode(data, .., 1)`, :151)
// behind the 12-byte header {COMPRESSED_BLOB_MAGIC_1_0, CRC} when it is shorter than the
// chunk, else the uncompressed blob {UNCOMPRESSED_BLOB_MAGIC_1_0, CRC, bytes}; the CRC
// (`compute_crc`, :70-75) covers everything after the header.  C ABI: include/pbs_blob.h.
//
// The frame is built from 64 KiB zstd blocks, one 512-thread workgroup per block at a
// time (one per CU: 154 KiB of LDS).  Per block:
//   stage   the block and up to 16 KiB of the chunk before it (the match window of its
//           first sub-blocks) in LDS -- every later byte read is LDS;
//   RLE     every byte equal: a 4-byte RLE block (the zero pages of a VM image);
//   parse   each of the 8 waves parses one ~8 KiB sub-block (8 KiB + 384 bytes for waves
//           0-3, - 384 for waves 4-7: see kZSubA) with its own 4096-entry table
//           of 16-bit window positions: the 12 KiB before the sub-block first enter the
//           table in accelerated rounds (every 2nd position or sparser), then rounds of
//           256 sampled positions (step 1
//           after a round with a match, doubling to 8 without): candidates = the table
//           (hash of 5 bytes; the last position of an EARLIER round) and the run
//           candidate p - 1, the longer (capped at 32) winning; the wave's greedy walk
//           over the round's match masks (ballots) checks the positions before the next
//           match for a match at the sub-block's last offset (a repeat match, one ballot),
//           extends a taken table match backwards over the literals (one ballot) and every
//           match forwards to its end (256 bytes per step);
//   literals the literal bytes (a bitmap of the matched bytes, per-thread popcounts and a
//           block scan give each literal its index): RLE, raw, or Huffman-coded (RFC 8878
//           4.2) -- histogram, a two-queue Huffman merge limited to 11 bits, canonical
//           codes, weights direct or FSE-coded, then every thread ORs the codes of its
//           literals into 4 streams staged in LDS at offsets from a block scan of the
//           code lengths (the streams are written backwards: bit offsets from the end of
//           the literal's stream);
//   sequences repeat-offset codes per sub-block (one lane each), code histograms, per
//           stream (LL / OF / ML) the cheapest of predefined / RLE / own FSE table (three
//           waves), then one lane writes the FSE bit stream;
//   raw     when the compressed block is not shorter than its bytes.
// Then per chunk: frame size, compressed-or-not (the reference's "only if shorter",
// :153), blob offsets by an exclusive scan, the blocks gathered into the blob images,
// and the blob CRC by the CRC kernel of pbs_blob.hip (12-byte header skipped).
//
// Every decision is integer-only and restated serially by the host twin
// (oracle/zstd_twin.cpp, written separately), so the bytes are compared exactly; libzstd
// decodes every frame back to the chunk (tests).  The bytes are not libzstd's level 1
// (parity unpinned); their size is within a few per cent of it on
// text, pxar-like and VM-image data (tests/test_zstd_cpu.py).
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
#include "dev_arena.h"
#include "zstd_enc.h"

namespace pbs {
namespace {

using namespace zstd;

constexpr int kZThreads = 512;
constexpr int kZWaves = kZThreads / 64;
// One wave's sub-block: waves 0-3 take 8 KiB + 768, waves 4-7 8 KiB - 768.  Waves w and
// w + 4 share a SIMD and the issue arbiter favours the older one: with equal sub-blocks
// waves 4-7 parsed ~9 % longer (text: 692 vs 756 us per block) whichever sub-blocks they
// got (profiles/r04/zstd_swap/), and then ran alone on their SIMDs.  Round 4 moved 384
// bytes; in the round-6 parse kernel waves 4-7 still took ~10 % longer per block (221 vs
// 242-246 us, 25.8 vs 31 ns per byte: profiles/r06/zsplit/probe.log), so 768 now.
#ifndef PBS_ZSUB_DELTA
#define PBS_ZSUB_DELTA 768  // (A/B builds only: the twin's kSubA / kSubB must follow)
#endif
constexpr uint32_t kZSubA = 8192 + PBS_ZSUB_DELTA, kZSubB = 8192 - PBS_ZSUB_DELTA;
__device__ __host__ constexpr uint32_t zsub_start(int w) {  // block position of sub-block w (0..8)
    return w <= 4 ? (uint32_t)w * kZSubA : 4 * kZSubA + (uint32_t)(w - 4) * kZSubB;
}
constexpr uint32_t kZHist = 16384;   // window before a sub-block
constexpr uint32_t kZRound = 256, kZHashLog = 12, kZCap = 32, kZMin = 5, kZMaxStep = 8, kZBack = 8;
// Since round 6 the history rounds step at least 2 bytes (1 before) and a sub-block's match
// window reaches 12 KiB back (16 KiB before): text 38.0 -> 40.4, pxar 39.1 -> 41.5 GiB/s for
// payloads 1.075 -> 1.092 x (text) and 1.034 -> 1.045 x (pxar) libzstd level 1
// (profiles/r06/zwindow/; the twin's kHistMinStep / kWin follow).  The macros are for A/B
// builds only.
#ifndef PBS_ZHIST_MIN
#define PBS_ZHIST_MIN 2
#endif
#ifndef PBS_ZWIN
#define PBS_ZWIN 12288
#endif
constexpr uint32_t kZHistRound = 512, kZHistStep0 = PBS_ZHIST_MIN, kZHistMaxStep = 8;  // history rounds (see parse_subblock)
constexpr uint32_t kZHistMinStep = PBS_ZHIST_MIN, kZWin = PBS_ZWIN;
constexpr int kZPer = kZRound / 64;        // positions per lane and round
constexpr int kZPerH = kZHistRound / 64;   // history positions per lane and round
constexpr uint32_t kZTab = 1u << kZHashLog;
constexpr uint32_t kZStageWords = (kZHist + kEncBlock) / 16 + 3;  // 16-byte words at any alignment + 2 zero words
constexpr uint32_t kZSubSeq = kZSubA / kZMin + 2;                 // sequences one sub-block can emit
constexpr uint32_t kZBlockSeq = kZWaves * kZSubSeq;
// (the per-block chain scratch: 3 x u32 chains, 3 x u16 states, 3 x (kZBlockSeq + 16) code
// bytes inside 6 x kZBlockSeq words, the 16-byte batch accesses aligned)
static_assert(kZBlockSeq % 8 == 0, "chain scratch alignment");
static_assert(3 * kZBlockSeq + 3 * kZBlockSeq / 2 + (3 * (kZBlockSeq + 16) + 3) / 4 <= 6 * kZBlockSeq, "chain scratch size");
constexpr uint64_t kSlot = kEncBlock + 1024;  // block header + up to 64 KiB + slack (section headers, flushes)
constexpr uint32_t kHufStreams = 48 * 1024;  // Huffman streams staged in LDS (longer: raw literals)
constexpr uint32_t kHufMax = 11;
constexpr uint32_t kZRuns = 64;  // blocks with fewer sequences copy raw literals run by run
static_assert(zsub_start(kZWaves) == kEncBlock && kZWaves == 8, "eight sub-blocks cover the block");
static_assert(kZTab * 2 * kZWaves == 64 * 1024, "the tables fill the work area");

// pbs-datastore/src/file_formats.rs:9, :12
constexpr uint8_t kUncompressedMagic[8] = {66, 171, 56, 7, 190, 131, 112, 161};
constexpr uint8_t kCompressedMagic[8] = {49, 185, 88, 66, 111, 182, 163, 127};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

struct Seq {
    uint32_t pos, ml, off;  // match start (block position), length, offset
};
struct Coded {
    uint32_t ll, ml, ofv, codes;  // offset value: repeat code 1-3 or offset + 3; codes llc | mlc << 8 | ofc << 16
};

// The staged window in LDS: window byte P (P = 0 at the chunk byte `hist` before the
// block) is LDS byte P + r.
// (the LDS address space spelled out in the type: with a generic pointer every access
// leans on the compiler inferring LDS through the noinline stages)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
struct Win {
    const lds_u32* w;
    uint32_t r;
    __device__ __forceinline__ uint32_t byte(uint32_t P) const {
        return reinterpret_cast<const lds_u8*>(w)[P + r];
    }
    __device__ __forceinline__ uint32_t word(uint32_t P) const {  // 4 bytes little-endian
        const uint32_t o = P + r;
        return __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], o & 3);
    }
    // the 4 bytes at P and (b4) the byte after them: one pair of LDS words
    __device__ __forceinline__ uint32_t word5(uint32_t P, uint32_t& b4) const {
        const uint32_t o = P + r;
        const uint32_t lo = w[o >> 2], hi = w[(o >> 2) + 1];
        b4 = (hi >> (8 * (o & 3))) & 0xFF;
        return __builtin_amdgcn_alignbyte(hi, lo, o & 3);
    }
};

__device__ __forceinline__ uint32_t hash5(uint32_t w, uint32_t b4) {
    return ((w * 2654435761u) ^ (b4 * 2246822519u)) >> (32 - kZHashLog);
}

// table[h] = max(table[h], v) for this wave's lanes: write, read back, repeat while a
// smaller value of another lane of the same instruction landed (lockstep: the survivors
// only ever raise it)
// (the LDS address space spelled out: a volatile generic access is not narrowed to LDS by
// the compiler and would go out as flat loads and stores, waiting on the memory counter)
typedef __attribute__((address_space(3))) uint16_t lds_u16;
__device__ __forceinline__ void tab_max(lds_u16* e, uint32_t v) {
    volatile lds_u16* ve = e;
    for (;;) {
        *ve = (uint16_t)v;
        if (*ve >= v) break;
    }
}

// tab_max over a lane's K positions: all writes, then all read-backs (in order: LDS ops of
// a wave complete in issue order), then the rare retries
template <int K>
__device__ __forceinline__ void tab_max_batch(lds_u16* tw, const uint32_t* h, const uint32_t* v, const bool* ok) {
#if PBS_ZV_SERIALTAB
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (ok[i]) tab_max(&tw[h[i]], v[i]);
    return;
#endif
    volatile lds_u16* const base = tw;
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (ok[i]) base[h[i]] = (uint16_t)v[i];
    uint32_t rb[K];
#pragma unroll
    for (int i = 0; i < K; ++i) rb[i] = ok[i] ? (uint32_t)base[h[i]] : 0xFFFFu;
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (rb[i] < v[i]) tab_max(&tw[h[i]], v[i]);
}

// a wave-uniform value, provably so (SGPR)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// inclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_incl(uint32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
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

// cnt bytes of an LDS buffer (4-byte aligned) to global dst at any alignment: head bytes
// up to a 4-aligned dst, then dword stores (each built from two LDS dwords), then the tail
__device__ __forceinline__ void lds_to_global(uint8_t* dst, const uint32_t* src, uint32_t cnt, uint32_t t,
                                              uint32_t nt) {
    const uint8_t* const sb = reinterpret_cast<const uint8_t*>(src);
    uint32_t head = (uint32_t)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);
    if (head > cnt) head = cnt;
    if (t < head) dst[t] = sb[t];
    const uint32_t nwd = (cnt - head) >> 2;
    uint32_t* const dw = reinterpret_cast<uint32_t*>(dst + head);
    for (uint32_t w = t; w < nwd; w += nt) {
        const uint32_t o = head + 4 * w;
        dw[w] = __builtin_amdgcn_alignbyte(src[(o >> 2) + 1], src[o >> 2], o & 3);
    }
    for (uint32_t i = head + 4 * nwd + t; i < cnt; i += nt) dst[i] = sb[i];
}

// cnt bytes of the staged window from position `from` to global dst at any alignment: head
// bytes up to a 4-aligned dst, then dword stores (W.word), then the tail; threads t of nt
__device__ __forceinline__ void stage_to_global(uint8_t* dst, const Win& W, uint32_t from, uint32_t cnt, uint32_t t,
                                                uint32_t nt) {
    uint32_t head = (uint32_t)((4 - (reinterpret_cast<uintptr_t>(dst) & 3)) & 3);
    if (head > cnt) head = cnt;
    if (t < head) dst[t] = (uint8_t)W.byte(from + t);
    const uint32_t nwd = (cnt - head) >> 2;
    uint32_t* const dw = reinterpret_cast<uint32_t*>(dst + head);
    // four dwords per thread and step, their LDS reads issued together (one dword a step
    // waited an LDS round trip per store: a VM block's ~40 KB of raw literals took 4.5 us)
    for (uint32_t w0 = t; w0 < nwd; w0 += 4 * nt) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w = w0 + (uint32_t)k * nt;
            v[k] = W.word(from + head + 4 * (w < nwd ? w : 0u));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w = w0 + (uint32_t)k * nt;
            if (w < nwd) dw[w] = v[k];
        }
    }
    for (uint32_t i = head + 4 * nwd + t; i < cnt; i += nt) dst[i] = (uint8_t)W.byte(from + i);
}

// ---------------------------------------------------------------- bit writers
// Backward bit stream of RFC 8878 4.1 as an encoder writes it (fields at increasing bit
// positions, bytes little-endian), one lane, to global memory.
struct GBits {
    uint64_t acc;
    uint32_t n;
    uint8_t* p;
    __device__ void init(uint8_t* dst) {
        acc = 0;
        n = 0;
        p = dst;
    }
    __device__ void put(uint64_t v, uint32_t nb) {
        acc |= (v & ((1ull << nb) - 1ull)) << n;  // nb <= 32
        n += nb;
        if (n >= 32) {
            p[0] = (uint8_t)acc;
            p[1] = (uint8_t)(acc >> 8);
            p[2] = (uint8_t)(acc >> 16);
            p[3] = (uint8_t)(acc >> 24);
            p += 4;
            acc >>= 32;
            n -= 32;
        }
    }
    __device__ void close() {
        put(1, 1);
        while (n > 0) {
            *p++ = (uint8_t)acc;
            acc >>= 8;
            n = n > 8 ? n - 8 : 0;
        }
    }
};

// the same into an LDS byte buffer (weights description)
struct LBits {
    uint64_t acc;
    uint32_t n;
    uint8_t* p;
    __device__ void init(uint8_t* dst) {
        acc = 0;
        n = 0;
        p = dst;
    }
    __device__ void put(uint64_t v, uint32_t nb) {
        acc |= (v & ((1ull << nb) - 1ull)) << n;
        n += nb;
        while (n >= 8) {
            *p++ = (uint8_t)acc;
            acc >>= 8;
            n -= 8;
        }
    }
    __device__ void close() {
        put(1, 1);
        if (n) *p++ = (uint8_t)acc;
        n = 0;
    }
};

// ---------------------------------------------------------------- FSE (one lane)
constexpr int kFseCells = 512;
struct FseT {
    uint16_t next[kFseCells];
    int32_t dnb[53];
    int32_t dfs[53];
    int32_t log;
    uint32_t mode;  // 0 predefined, 1 RLE, 2 FSE-compressed
    uint32_t desc_len;
    uint8_t desc[128];
    uint8_t sym_at[kFseCells];  // construction scratch (LDS: no private arrays on the serial paths)
    int16_t norm[64];
    int32_t cum[64];
};
// a predefined table (RFC 8878 3.1.1.3.2.2), built once per launch
struct PreT {
    uint16_t next[64];
    int32_t dnb[53];
    int32_t dfs[53];
    int32_t log;
};
// Address spaces spelled out where a noinline function receives LDS or global pointers:
// the compiler cannot always narrow a generic pointer and would emit flat accesses, which
// wait on both counters (an LDS lookup then waits for every outstanding global load).
typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
typedef __attribute__((address_space(3))) const int32_t lds_ci32;
#define PBS_GLOBAL __attribute__((address_space(1)))
struct FseView {
    lds_cu16* next;
    lds_ci32* dnb;
    lds_ci32* dfs;
    uint32_t log;
};

// (norm: the predefined counts in global memory, or a table's own counts in LDS)
__device__ __noinline__ void fse_build(FseT& t_g, const int16_t* norm, int nsym, int log) {
    __attribute__((address_space(3))) FseT& t = *(__attribute__((address_space(3))) FseT*)&t_g;
    const int size = 1 << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    int high = size - 1;
    __attribute__((address_space(3))) int32_t* const cum = t.cum;
    cum[0] = 0;
    for (int s = 0; s < nsym; ++s) {
        if (norm[s] == -1) {
            cum[s + 1] = cum[s] + 1;
            t.sym_at[high--] = (uint8_t)s;
        } else {
            cum[s + 1] = cum[s] + norm[s];
        }
    }
    int pos = 0;
    for (int s = 0; s < nsym; ++s)
        for (int k = 0; k < norm[s]; ++k) {
            t.sym_at[pos] = (uint8_t)s;
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    for (int u = 0; u < size; ++u) t.next[cum[t.sym_at[u]]++] = (uint16_t)(size + u);
    int total = 0;
    for (int s = 0; s < nsym; ++s) {
        const int c = norm[s];
        if (c == 0) {
            t.dnb[s] = ((log + 1) << 16) - size;
            t.dfs[s] = 0;
        } else if (c == -1 || c == 1) {
            t.dnb[s] = (log << 16) - size;
            t.dfs[s] = total - 1;
            ++total;
        } else {
            const int maxbits = log - (int)highbit((uint32_t)(c - 1));
            t.dnb[s] = (maxbits << 16) - (c << maxbits);
            t.dfs[s] = total - c;
            total += c;
        }
    }
    t.log = log;
}

// fse_build by ONE WAVE (nsym <= 64), same table: symbol s's cells are the (cs_s + i)-th
// positions of the spread sequence (j * step) & mask that are <= high (cs = exclusive
// prefix of the positive counts); next[] takes, per symbol, its cells in increasing order
// (rank among the same symbol by ballots, 64 cells at a time).
__device__ __noinline__ void fse_build_wave(FseT& t_g, const int16_t* norm_g, int nsym, int log, int lane) {
    __attribute__((address_space(3))) FseT& t = *(__attribute__((address_space(3))) FseT*)&t_g;
    const __attribute__((address_space(3))) int16_t* const norm = (const __attribute__((address_space(3))) int16_t*)norm_g;
    const uint32_t size = 1u << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    const int c = lane < nsym ? norm[lane] : 0;
    const uint32_t cells = c == -1 ? 1u : (c > 0 ? (uint32_t)c : 0u);
    const uint32_t spread = c > 0 ? (uint32_t)c : 0u, low = c == -1 ? 1u : 0u;
    const uint32_t ci = wave_incl(cells, lane), si = wave_incl(spread, lane), li = wave_incl(low, lane);
    const uint32_t nlow = (uint32_t)__builtin_amdgcn_readlane((int)li, 63);
    const uint32_t high = size - 1 - nlow;
    __attribute__((address_space(3))) uint16_t* const spc = t.next;  // (scratch until next[] is written below)
    if (lane < nsym) {
        t.cum[lane] = (int32_t)(ci - cells);
        spc[lane] = (uint16_t)(si - spread);
        if (low) t.sym_at[size - 1 - (li - low)] = (uint8_t)lane;
    }
    __builtin_amdgcn_wave_barrier();
    // spread: placement k at the k-th position <= high
    const uint32_t nspread = (uint32_t)__builtin_amdgcn_readlane((int)si, 63);
    uint32_t kb = 0;
    for (uint32_t j0 = 0; j0 < size; j0 += 64) {
        const uint32_t j = j0 + (uint32_t)lane;
        const uint32_t P = (j * step) & mask;
        const bool ok = j < size && P <= high;
        const unsigned long long b = __ballot(ok);
        const uint32_t k = kb + (uint32_t)__builtin_popcountll(b & ((1ull << lane) - 1ull));
        if (ok && k < nspread) {
            int lo = 0, hi = nsym - 1;  // the last symbol with spc <= k (and a positive count)
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (spc[mid] <= k) lo = mid; else hi = mid - 1;
            }
            while (norm[lo] <= 0) --lo;  // (symbols without spread cells share its spc)
            t.sym_at[P] = (uint8_t)lo;
        }
        kb += (uint32_t)__builtin_popcountll(b);
    }
    __builtin_amdgcn_wave_barrier();
    // next: the cells of each symbol in increasing order; the running slot of symbol s in
    // lane s of `run` (a readlane and a writelane a symbol: no LDS round trip in the loop)
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t run = lane < nsym ? ci - cells : 0u;
    for (uint32_t u0 = 0; u0 < size; u0 += 64) {
        const uint32_t u = u0 + (uint32_t)lane;
        const uint32_t sy = u < size ? t.sym_at[u] : 0xFFFFu;
        unsigned long long rem = __ballot(u < size);
        uint32_t slot = 0;
        while (rem) {
            const int f = __builtin_ctzll(rem);
            const uint32_t s0 = uni((uint32_t)__builtin_amdgcn_readlane((int)sy, f));
            const unsigned long long mm = __ballot(sy == s0) & rem;
            const uint32_t base = uni((uint32_t)__builtin_amdgcn_readlane((int)run, (int)s0));
            if (sy == s0) slot = base + (uint32_t)__builtin_popcountll(mm & lt);
            const uint32_t nb = uni(base + (uint32_t)__builtin_popcountll(mm));
            asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(run) : "s"(nb), "{m0}"(s0));
            rem &= ~mm;
        }
        if (u < size) t.next[slot] = (uint16_t)(size + u);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < nsym) {
        const uint32_t total = ci - cells;
        if (c == 0) {
            t.dnb[lane] = (int32_t)(((uint32_t)log + 1) << 16) - (int32_t)size;
            t.dfs[lane] = 0;
        } else if (c == -1 || c == 1) {
            t.dnb[lane] = (int32_t)((uint32_t)log << 16) - (int32_t)size;
            t.dfs[lane] = (int32_t)total - 1;
        } else {
            const int maxbits = log - (int)highbit((uint32_t)(c - 1));
            t.dnb[lane] = (maxbits << 16) - (c << maxbits);
            t.dfs[lane] = (int32_t)total - c;
        }
    }
    if (lane == 0) t.log = log;
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ FseView view(const FseT& t) {
    return FseView{(lds_cu16*)t.next, (lds_ci32*)t.dnb, (lds_ci32*)t.dfs, (uint32_t)t.log};
}
__device__ __forceinline__ FseView view(const PreT& t) {
    return FseView{(lds_cu16*)t.next, (lds_ci32*)t.dnb, (lds_ci32*)t.dfs, (uint32_t)t.log};
}

__device__ __forceinline__ uint32_t fse_init(const FseView& t, uint32_t s) {
    const uint32_t nb = (uint32_t)((t.dnb[s] + (1 << 15)) >> 16);
    const uint32_t v0 = (nb << 16) - (uint32_t)t.dnb[s];
    return t.next[(v0 >> nb) + t.dfs[s]];
}
template <typename B>
__device__ __forceinline__ void fse_enc(B& b, const FseView& t, uint32_t& v, uint32_t s) {
    const uint32_t nb = (v + (uint32_t)t.dnb[s]) >> 16;
    b.put(v, nb);
    v = t.next[(v >> nb) + t.dfs[s]];
}

__device__ __noinline__ int fse_log(uint32_t total, uint32_t max_sym, int max_log) {
    int log = max_log;
    const int src = (int)highbit(total - 1) - 2;
    const int minb = (int)min(highbit(total) + 1, highbit(max_sym) + 2);
    if (src < log) log = src;
    if (minb > log) log = minb;
    return max(5, min(log, max_log));
}

__device__ __noinline__ void fse_normalize(int16_t* norm, const uint32_t* cnt, int nsym, uint32_t total, int log) {
    const int64_t scale = 1ll << log;
    int64_t sum = 0;
    for (int s = 0; s < nsym; ++s) {
        if (!cnt[s]) {
            norm[s] = 0;
            continue;
        }
        int64_t v = ((int64_t)cnt[s] * scale + total / 2) / total;
        if (v < 1) v = 1;
        norm[s] = (int16_t)v;
        sum += v;
    }
    while (sum != scale) {
        int big = -1;
        for (int s = 0; s < nsym; ++s)
            if (norm[s] > 0 && (big < 0 || norm[s] > norm[big])) big = s;
        if (sum < scale) {
            norm[big] = (int16_t)(norm[big] + (scale - sum));
            sum = scale;
        } else {
            const int64_t take = min(sum - scale, (int64_t)norm[big] - 1);
            norm[big] = (int16_t)(norm[big] - take);
            sum -= take;
        }
    }
}

// RFC 8878 4.1.1 table description; returns its bytes
__device__ __noinline__ uint32_t fse_ncount(uint8_t* o, const int16_t* norm, int nsym, int log) {
    uint8_t* const o0 = o;
    const int size = 1 << log;
    uint64_t bs = (uint64_t)(log - 5);
    int nb = 4;
    int remaining = size + 1, threshold = size, nbits = log + 1, s = 0;
    bool prev0 = false;
    while (s < nsym && remaining > 1) {
        if (prev0) {
            int start = s;
            while (s < nsym && !norm[s]) ++s;
            while (s >= start + 24) {
                start += 24;
                bs |= 0xFFFFull << nb;
                nb += 16;
                while (nb >= 8) {
                    *o++ = (uint8_t)bs;
                    bs >>= 8;
                    nb -= 8;
                }
            }
            while (s >= start + 3) {
                start += 3;
                bs |= 3ull << nb;
                nb += 2;
            }
            bs |= (uint64_t)(s - start) << nb;
            nb += 2;
            while (nb >= 8) {
                *o++ = (uint8_t)bs;
                bs >>= 8;
                nb -= 8;
            }
        }
        int count = norm[s++];
        const int mx = (2 * threshold - 1) - remaining;
        remaining -= count < 0 ? -count : count;
        ++count;
        if (count >= threshold) count += mx;
        bs |= (uint64_t)count << nb;
        nb += nbits;
        nb -= count < mx;
        prev0 = count == 1;
        while (remaining < threshold) {
            --nbits;
            threshold >>= 1;
        }
        while (nb >= 8) {
            *o++ = (uint8_t)bs;
            bs >>= 8;
            nb -= 8;
        }
    }
    while (nb > 0) {
        *o++ = (uint8_t)bs;
        bs >>= 8;
        nb -= 8;
    }
    return (uint32_t)(o - o0);
}

// Table of one sequence symbol stream: the cheapest of predefined (0), RLE (1) and own
// FSE table (2) by the integer estimate (ties keep the earlier mode).  Mode 0 leaves the
// table to the launch's predefined one.  ONE WAVE, a lane per symbol (nsym <= 64): the
// normalisation's rounding, its fix-up (the largest count, first on ties), the estimate;
// lane 0 writes the description, the wave builds the table.
__device__ __noinline__ void seq_table_wave(FseT& t, const uint32_t* cnt, int nsym, uint32_t nseq, const int16_t* pre,
                                            int pre_log, int max_log, int lane) {
    const uint32_t c = lane < nsym ? cnt[lane] : 0u;
    const unsigned long long present = __ballot(c != 0);
    const int distinct = __builtin_popcountll(present);
    const int maxs = present ? 63 - __builtin_clzll(present) : 0;
    uint64_t cp = c ? (uint64_t)c * (256u * pre_log - lg256(pre[lane] < 1 ? 1 : pre[lane])) : 0ull;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cp += __shfl_xor(cp, d, 64);
    if (lane == 0) {
        t.desc_len = 0;
        t.mode = 0;
    }
    if (distinct == 1 && nseq > 2) {
        if (lane == 0) {
            t.mode = 1;
            t.desc[0] = (uint8_t)maxs;
            t.desc_len = 1;
        }
        __builtin_amdgcn_wave_barrier();
        return;
    }
    if (nseq >= 16) {
        const int log = fse_log(nseq, (uint32_t)maxs, max_log);
        const int64_t scale = 1ll << log;
        int64_t v = 0;
        if (c) {
            v = ((int64_t)c * scale + nseq / 2) / nseq;
            if (v < 1) v = 1;
        }
        int64_t sum = v;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
        while (sum != scale) {  // wave-uniform
            uint32_t key = v > 0 ? (uint32_t)v << 8 | (255u - (uint32_t)lane) : 0u;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) key = max(key, (uint32_t)__shfl_xor((int)key, d, 64));
            const int big = 255 - (int)(key & 255u);
            const int64_t vb = (int64_t)(key >> 8);
            int64_t nv = vb;
            if (sum < scale) {
                nv = vb + (scale - sum);
                sum = scale;
            } else {
                const int64_t take = min(sum - scale, vb - 1);
                nv = vb - take;
                sum -= take;
            }
            if (lane == big) v = nv;
        }
        if (lane < nsym) t.norm[lane] = (int16_t)(lane <= maxs ? v : 0);
        __builtin_amdgcn_wave_barrier();
        uint32_t d = 0;
        if (lane == 0) d = fse_ncount(t.desc, t.norm, maxs + 1, log);
        d = uni(d);
        uint64_t cc = c ? (uint64_t)c * (256u * log - lg256((uint32_t)v)) : 0ull;
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) cc += __shfl_xor(cc, k, 64);
        cc += 2048ull * d;
        if (cc < cp) {
            if (lane == 0) {
                t.mode = 2;
                t.desc_len = d;
            }
            fse_build_wave(t, t.norm, maxs + 1, log, lane);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------- LDS layout
// work area (64 KiB): the parse's tables, then the entropy stage's buffers
struct EntropyArea {
    uint32_t streams[kHufStreams / 4 + 4];  // Huffman streams (and, before them, per-wave literal histograms)
    uint32_t bitmap[kEncBlock / 32];        // literal bytes of the block
    uint32_t hist[256];
    uint32_t keys[256];   // symbols sorted by (count, symbol)
    uint32_t tw[512];     // Huffman merge: node weights
    uint16_t par[512];    // ... and parents
    uint8_t lens[256];    // code length per sorted index
    uint8_t len[256];     // code length per symbol
    uint16_t code[256];
    uint32_t shist[36 + 53 + 32];  // sequence code histograms: LL, ML, OF
};
static_assert(sizeof(EntropyArea) <= 64 * 1024, "entropy buffers fit the work area");

struct Ctl {
    uint32_t nseq[kZWaves];     // sequences per sub-block
    uint32_t lastend[kZWaves];  // end of the sub-block's last match (block position), 0 if none
    uint32_t wsum[kZWaves];     // block-scan partials
    uint32_t wsum2[kZWaves];
    uint32_t segP[5];           // Huffman: bits before each segment boundary
    uint32_t lit_mode, lit_size, huf_c, huf_hs, desc_len, need_full;
    uint32_t run_start[kZRuns], run_len[kZRuns], run_out[kZRuns];  // literal runs of a block with few sequences
    uint32_t seq_size, seq_ok, seq_hdr, seq_last[3];  // sequences: body size, fits, header bytes, final states
    int32_t root;               // Huffman merge: the root node
    uint8_t desc[264];          // Huffman tree description (FSE form: <= ~210 bytes before the 128 check)
};

// Wave-uniform element i of a lane-distributed array (element i in lane i & 63 of register
// i >> 6): read and write.
__device__ __forceinline__ uint32_t rd_q(const uint32_t (&r)[4], uint32_t i) {  // i: wave-uniform
    const int l = (int)(i & 63);
    const uint32_t k = i >> 6;
    const uint32_t v = k == 0   ? (uint32_t)__builtin_amdgcn_readlane((int)r[0], l)
                       : k == 1 ? (uint32_t)__builtin_amdgcn_readlane((int)r[1], l)
                       : k == 2 ? (uint32_t)__builtin_amdgcn_readlane((int)r[2], l)
                                : (uint32_t)__builtin_amdgcn_readlane((int)r[3], l);
    return uni(v);
}
__device__ __forceinline__ void wr_q(uint32_t (&r)[4], uint32_t i, uint32_t v) {  // i, v: wave-uniform
    const int l = (int)(i & 63);
    switch (i >> 6) {
        case 0: asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(r[0]) : "s"(v), "{m0}"(l)); break;
        case 1: asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(r[1]) : "s"(v), "{m0}"(l)); break;
        case 2: asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(r[2]) : "s"(v), "{m0}"(l)); break;
        default: asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(r[3]) : "s"(v), "{m0}"(l)); break;
    }
}
// Huffman tree description (RFC 8878 4.2.1), by ONE WAVE: the weights of symbols 0 ..
// last-1 (the last one is implied), FSE-compressed (two interleaved states) when that is
// shorter, else in the direct 4-bit form; false when neither applies (raw literals).  The
// weights, the table (log <= 6: one cell per lane) and the output bytes live in registers,
// so the serial encode is readlanes and scalar arithmetic (round 4's one-lane version
// waited on LDS at every weight: ~40-60 us a block); counts and the direct form by lanes.
template <class EA>
__device__ __noinline__ bool huf_describe(EA& E, Ctl& ctl, FseT& t_scratch, uint32_t mb, uint32_t lastsym,
                                          int lane) {
    const uint32_t nwt = uni(lastsym);
    uint32_t wreg[4], wmax = 0;  // weight of symbol lane + 64 j
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t sy = (uint32_t)lane + 64u * (uint32_t)j;
        const uint32_t ln = sy < nwt ? (uint32_t)E.len[sy] : 0u;
        wreg[j] = ln ? mb + 1 - ln : 0u;
        wmax = max(wmax, wreg[j]);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, d, 64));
    const uint32_t maxw = uni(wmax);
    // weight counts: lane v < 16 holds the count of weight v
    uint32_t wcnt = 0;
    bool single = false;
#pragma unroll
    for (uint32_t v = 0; v < 16; ++v) {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            c += (uint32_t)__builtin_popcountll(__ballot((uint32_t)lane + 64u * (uint32_t)j < nwt && wreg[j] == v));
        if ((uint32_t)lane == v) wcnt = c;
        single |= c == nwt;
    }
    uint32_t* const wc = reinterpret_cast<uint32_t*>(t_scratch.cum);  // weight counts (LDS)
    if (lane < 16) wc[lane] = wcnt;
    __builtin_amdgcn_wave_barrier();
    bool fse_ok = false;
    uint32_t fl = 0;
    if (nwt > 2 && !single) {
        const int lg = fse_log(nwt, maxw, 6);
        FseT& t = t_scratch;
        uint32_t f0 = 0;
        if (lane == 0) {
            fse_normalize(t.norm, wc, (int)maxw + 1, nwt, lg);
            f0 = fse_ncount(ctl.desc + 1, t.norm, (int)maxw + 1, lg);
        }
        f0 = uni((uint32_t)__builtin_amdgcn_readlane((int)f0, 0));
        __builtin_amdgcn_wave_barrier();
        fse_build_wave(t, t.norm, (int)maxw + 1, lg, lane);  // (overwrites wc: no longer needed)
        const uint32_t size = 1u << lg;
        const uint32_t nxr = (uint32_t)lane < size ? (uint32_t)t.next[lane] : 0u;
        const uint32_t dnr = (uint32_t)lane <= maxw ? (uint32_t)t.dnb[lane] : 0u;
        const uint32_t dfr = (uint32_t)lane <= maxw ? (uint32_t)t.dfs[lane] : 0u;
        auto dnb = [&](uint32_t sy) { return uni((uint32_t)__builtin_amdgcn_readlane((int)dnr, (int)sy)); };
        auto dfs = [&](uint32_t sy) { return uni((uint32_t)__builtin_amdgcn_readlane((int)dfr, (int)sy)); };
        auto nxt = [&](uint32_t u) { return uni((uint32_t)__builtin_amdgcn_readlane((int)nxr, (int)u)); };
        auto init = [&](uint32_t sy) {
            const uint32_t nb = (dnb(sy) + (1u << 15)) >> 16;
            const uint32_t v0 = (nb << 16) - dnb(sy);
            return nxt((v0 >> nb) + dfs(sy));
        };
        // the bit stream: bytes into lane k of ob[k >> 6] (bytes past 127 are not kept: the
        // description must stay under 128 bytes anyway)
        uint32_t ob[4] = {0, 0, 0, 0};
        uint64_t acc = 0;
        uint32_t n = 0, nbytes = 0;
        auto put = [&](uint32_t v, uint32_t nb) {
            acc |= (uint64_t)(v & ((1u << nb) - 1u)) << n;
            n += nb;
            while (n >= 8) {
                if (nbytes < 128) wr_q(ob, nbytes, uni((uint32_t)acc & 0xFFu));
                ++nbytes;
                acc >>= 8;
                n -= 8;
            }
        };
        auto enc = [&](uint32_t& v, uint32_t sy) {
            const uint32_t nb = (v + dnb(sy)) >> 16;
            put(v, nb);
            v = nxt((v >> nb) + dfs(sy));
        };
        uint32_t v1, v2, i = nwt;
        if (nwt & 1) {
            v1 = init(rd_q(wreg, --i));
            v2 = init(rd_q(wreg, --i));
            enc(v1, rd_q(wreg, --i));
        } else {
            v2 = init(rd_q(wreg, --i));
            v1 = init(rd_q(wreg, --i));
        }
        while (i > 0) {
            enc(v2, rd_q(wreg, --i));
            enc(v1, rd_q(wreg, --i));
        }
        put(v2, (uint32_t)lg);
        put(v1, (uint32_t)lg);
        put(1, 1);  // close
        if (n) {
            if (nbytes < 128) wr_q(ob, nbytes, uni((uint32_t)acc & 0xFFu));
            ++nbytes;
        }
        fl = f0 + nbytes;
        fse_ok = fl < 128;
        if (fse_ok) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t k = (uint32_t)lane + 64u * (uint32_t)j;
                if (k < nbytes) ctl.desc[1 + f0 + k] = (uint8_t)ob[j];
            }
        }
    }
    const uint32_t direct = nwt <= 128 ? 1 + (nwt + 1) / 2 : 0xFFFFFFFFu;
    bool ok = true;
    if (fse_ok && fl + 1 < direct) {
        if (lane == 0) {
            ctl.desc[0] = (uint8_t)fl;
            ctl.desc_len = fl + 1;
        }
    } else if (direct != 0xFFFFFFFFu) {
        // byte k: the weights of symbols 2k and 2k + 1 (lane k: symbols 2 lane, 2 lane + 1)
        const uint32_t s0 = 2u * (uint32_t)lane, s1 = s0 + 1;
        const uint32_t w0 = (uint32_t)__shfl((int)wreg[0], (int)(s0 & 63), 64);
        const uint32_t w0b = (uint32_t)__shfl((int)wreg[1], (int)(s0 & 63), 64);
        const uint32_t w1 = (uint32_t)__shfl((int)wreg[0], (int)(s1 & 63), 64);
        const uint32_t w1b = (uint32_t)__shfl((int)wreg[1], (int)(s1 & 63), 64);
        const uint32_t a = s0 < 64 ? w0 : w0b;
        const uint32_t b = s1 < nwt ? (s1 < 64 ? w1 : w1b) : 0u;
        if (s0 < nwt) ctl.desc[1 + lane] = (uint8_t)(a << 4 | b);
        if (lane == 0) {
            ctl.desc[0] = (uint8_t)(127 + nwt);
            ctl.desc_len = direct;
        }
    } else {
        ok = false;  // no description fits: raw literals
    }
    __builtin_amdgcn_wave_barrier();
    return ok;
}

// One FSE state chain of the sequences bit stream, by ONE WAVE: the state is initialised
// from the last sequence's code and then encodes sequences ns-2 .. 0 (steps j = 0 .. m-1,
// sequence ns-2-j); chain[j] = the bits step j emits, i.e. for sequence ns-2-j (value |
// count << 16, in step order so a lane's batch of steps is one run of words),
// *last = the final state (flushed after sequence 0).  `shift` picks the code byte (0 LL,
// 8 ML, 16 OF).  The chain is serial, but tANS states forget their past quickly (every
// encode maps many states to one), so lane l runs steps [l seg, (l+1) seg) from a guessed
// state, recording the state before each step; then, in rounds, a lane whose start state
// differs from its left neighbour's end re-runs from that end until its state meets the
// recorded one (the rest of its record is then already right).  Lane 0 starts from the
// true state, so after r rounds lanes 0..r are exact; usually one round settles all.
__device__ __noinline__ void seq_chain_wave(FseView t, const Coded* __restrict__ coded_g, uint32_t ns,
                                            uint32_t shift, uint32_t* __restrict__ chain_g,
                                            uint16_t* __restrict__ states_g, uint8_t* __restrict__ codes_g,
                                            uint32_t* last, int lane, unsigned long long* probe) {
    const PBS_GLOBAL Coded* const coded = (const PBS_GLOBAL Coded*)coded_g;
    PBS_GLOBAL uint32_t* const chain = (PBS_GLOBAL uint32_t*)chain_g;
    PBS_GLOBAL uint16_t* const states = (PBS_GLOBAL uint16_t*)states_g;
    const uint32_t m = ns - 1;
    if (m < 128) {  // short: one lane, serially (the rounds would cost more than they save)
        // the wave loads 64 codes at a time, lane 0 takes them by readlane
        uint32_t x = 0;
        for (uint32_t j0 = 0; j0 < m; j0 += 64) {
            const uint32_t jl = j0 + (uint32_t)lane;
            const uint32_t mine = jl < m ? (coded[ns - 2 - jl].codes >> shift) & 0xFF : 0u;
            if (j0 == 0) x = fse_init(t, (uni(coded[ns - 1].codes) >> shift) & 0xFF);
            uint32_t mine_bits = 0;
            const uint32_t nj = min(64u, m - j0);
            for (uint32_t u = 0; u < nj; ++u) {
                const uint32_t sym = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)u);
                const uint32_t nb = (x + (uint32_t)t.dnb[sym]) >> 16;
                if ((uint32_t)lane == u) mine_bits = (x & ((1u << nb) - 1u)) | nb << 16;
                x = t.next[(x >> nb) + t.dfs[sym]];
            }
            if (jl < m) chain[jl] = mine_bits;
        }
        if (lane == 0) *last = m ? x : fse_init(t, (coded[ns - 1].codes >> shift) & 0xFF);
        return;
    }
    // kB steps a batch; segments are whole batches, so a batch starts kB-aligned and its
    // records go out as 16-byte stores (a store per lane per step, 64 lanes in 64 segments,
    // was a cache line per lane and store: 2 x 64 line requests per step)
    constexpr uint32_t kB = 8;
    const uint32_t seg = ((m + 63) / 64 + kB - 1) / kB * kB;
    const uint32_t a = min(m, (uint32_t)lane * seg), b = min(m, a + seg);
    const uint32_t x0 = fse_init(t, (coded[ns - 1].codes >> shift) & 0xFF);
    // the next batch's codes (and recorded states) are loaded before this batch's stores:
    // loads and stores share one in-order counter, so loads issued after the stores would
    // wait for them.  Loads past the segment read its last step (unused), so the loads are
    // unconditional and the counter waits exact.
    // the stream's codes in step order, a byte per step, so a lane's batch is one 8-byte load
    // (its recorded states one 16-byte load) instead of 2 x 8 loads of 64 cache lines each
    PBS_GLOBAL uint8_t* const cs = (PBS_GLOBAL uint8_t*)codes_g;
    // (8 records in flight per lane: the entropy kernel reads them from HBM, written by the
    // parse kernel, not from this workgroup's L2)
    for (uint32_t j0 = (uint32_t)lane; j0 < m; j0 += 8 * 64) {
        uint32_t cv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t j = j0 + 64u * (uint32_t)u;
            cv[u] = j < m ? coded[ns - 2 - j].codes : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t j = j0 + 64u * (uint32_t)u;
            if (j < m) cs[j] = (uint8_t)((cv[u] >> shift) & 0xFF);
        }
    }
    __threadfence_block();  // (the other lanes' bytes before the batch loads)
    auto run = [&](uint32_t x, bool stop_on_meet) -> uint32_t {  // returns the end state, ~0u: met
        if (a >= b) return x;
        // (a batch starts kB-aligned; its bytes past the segment or the stream are read, not used)
        auto load = [&](uint32_t j, uint32_t (&c)[kB], uint32_t (&sv)[kB]) {
            const uint64_t w = *reinterpret_cast<const PBS_GLOBAL uint64_t*>(cs + j);
#pragma unroll
            for (int u = 0; u < (int)kB; ++u) c[u] = (uint32_t)(w >> (8 * u)) & 0xFFu;
            if (stop_on_meet) {
                const v4u q = *reinterpret_cast<const PBS_GLOBAL v4u*>(states + j);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    sv[2 * u] = q[u] & 0xFFFFu;
                    sv[2 * u + 1] = q[u] >> 16;
                }
            } else {
#pragma unroll
                for (int u = 0; u < (int)kB; ++u) sv[u] = 0u;
            }
        };
        uint32_t cA[kB], sA[kB];
        load(a, cA, sA);
        for (uint32_t j = a;;) {
            uint32_t cB[kB], sB[kB];
            const uint32_t jn = j + kB;
            const bool more = jn < b;
            if (more) load(jn, cB, sB);
            uint32_t cv[kB], st[kB];
            uint32_t meet = kB;  // the step whose recorded state equals the running one
            const uint32_t nj = min(kB, b - j);
            // the batch's symbol entries first (they do not depend on the state): a step then
            // waits for one LDS read, its next[] cell
            uint32_t dn[kB], df[kB];
#pragma unroll
            for (int u = 0; u < (int)kB; ++u) {
                dn[u] = (uint32_t)t.dnb[cA[u]];
                df[u] = (uint32_t)t.dfs[cA[u]];
            }
#pragma unroll
            for (int u = 0; u < (int)kB; ++u)
                if ((uint32_t)u < nj && meet == kB) {
                    if (stop_on_meet && sA[u] == x) {
                        meet = (uint32_t)u;
                    } else {
                        st[u] = x;
                        const uint32_t nb = (x + dn[u]) >> 16;
                        cv[u] = (x & ((1u << nb) - 1u)) | nb << 16;
                        x = t.next[(x >> nb) + df[u]];
                    }
                }
            if (nj == kB && meet == kB) {
                *reinterpret_cast<PBS_GLOBAL v4u*>(states + j) =
                    v4u{st[0] | st[1] << 16, st[2] | st[3] << 16, st[4] | st[5] << 16, st[6] | st[7] << 16};
                *reinterpret_cast<PBS_GLOBAL v4u*>(chain + j) = v4u{cv[0], cv[1], cv[2], cv[3]};
                *reinterpret_cast<PBS_GLOBAL v4u*>(chain + j + 4) = v4u{cv[4], cv[5], cv[6], cv[7]};
            } else {
                const uint32_t nd = min(nj, meet);
#pragma unroll
                for (int u = 0; u < (int)kB; ++u)
                    if ((uint32_t)u < nd) {
                        states[j + u] = (uint16_t)st[u];
                        chain[j + u] = cv[u];
                    }
            }
            if (meet != kB) return ~0u;
            if (!more) break;
#pragma unroll
            for (int u = 0; u < (int)kB; ++u) {
                cA[u] = cB[u];
                sA[u] = sB[u];
            }
            j = jn;
        }
        return x;
    };
    // pass 1: lane 0 from the true state, the others from the table's first state
    uint32_t start = lane == 0 ? x0 : (1u << t.log);
    const uint64_t tp0 = probe ? wall_clock64() : 0;
    uint32_t end = run(start, false);
    const uint64_t tp1 = probe ? wall_clock64() : 0;
    int round = 0;
    for (; round < 64; ++round) {
        // the true start of lane l is lane l-1's end (lane 0: x0)
        const uint32_t left = (uint32_t)__shfl_up((int)end, 1, 64);
        const uint32_t want = lane == 0 ? x0 : left;
        const bool redo = want != start && a < b;
        if (!__ballot(redo)) break;
        if (redo) {
            start = want;
            const uint32_t e = run(start, true);
            if (e != ~0u) end = e;  // never met: the whole segment changed, so does its end
        } else if (a >= b) {
            end = want;  // an empty segment passes its start through
            start = want;
        }
    }
    if (probe && lane == 0) {
        probe[22] += tp1 - tp0;
        probe[23] += wall_clock64() - tp1;
        probe[24] += (unsigned long long)round;
        probe[25] += 1;
    }
    // the final state: the end of the last non-empty segment
    const uint32_t lastlane = m ? (m - 1) / seg : 0;
    const uint32_t fin = (uint32_t)__shfl((int)end, (int)lastlane, 64);
    if (lane == 0) *last = m ? fin : x0;
}

// bits of sequence q in the stream: its three state fields (none for the last sequence,
// nor for an RLE-mode stream) and its extra bits
__device__ __forceinline__ uint32_t seq_bits(const Coded& x, uint32_t q, uint32_t ns, const uint32_t* chains,
                                             uint32_t stride, const uint32_t* mode) {
    const uint32_t llc = x.codes & 0xFF, mlc = (x.codes >> 8) & 0xFF, ofc = x.codes >> 16;
    uint32_t b = ll_bits(llc) + ml_bits(mlc) + ofc;
    if (q + 1 < ns) {
        const uint32_t j = ns - 2 - q;  // the chains are in step order
        if (mode[0] != 1) b += chains[j] >> 16;
        if (mode[1] != 1) b += chains[stride + j] >> 16;
        if (mode[2] != 1) b += chains[2 * stride + j] >> 16;
    }
    return b;
}

// a thread's bits into the zeroed stream words (atomicOr: its first and last words are
// shared with its neighbours)
struct OrBits {
    PBS_GLOBAL uint32_t* w;
    uint32_t wi;
    uint64_t acc;
    uint32_t n;
    __device__ __forceinline__ void init(uint32_t* words, uint32_t bit) {
        w = (PBS_GLOBAL uint32_t*)words;
        wi = bit >> 5;
        n = bit & 31;
        acc = 0;
    }
    __device__ __forceinline__ void put(uint64_t v, uint32_t nb) {
        acc |= (v & ((1ull << nb) - 1ull)) << n;  // nb <= 31
        n += nb;
        if (n >= 32) {
            if ((uint32_t)acc) __hip_atomic_fetch_or(&w[wi], (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ++wi;
            acc >>= 32;
            n -= 32;
        }
    }
    __device__ __forceinline__ void done() {
        if (n && (uint32_t)acc) __hip_atomic_fetch_or(&w[wi], (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

// The same into words staged in LDS (ds_or: no global atomics, whose completion later loads
// of the thread would wait for on the in-order memory counter)
struct OrBitsL {
    lds_u32* w;  // (typed: a generic pointer made these flat atomics)
    uint32_t wi;
    uint64_t acc;
    uint32_t n;
    __device__ __forceinline__ void init(uint32_t* words, uint32_t bit) {
        w = (lds_u32*)words;
        wi = bit >> 5;
        n = bit & 31;
        acc = 0;
    }
    __device__ __forceinline__ void put(uint64_t v, uint32_t nb) {
        acc |= (v & ((1ull << nb) - 1ull)) << n;  // nb <= 31
        n += nb;
        if (n >= 32) {
            if ((uint32_t)acc) __hip_atomic_fetch_or(&w[wi], (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            ++wi;
            acc >>= 32;
            n -= 32;
        }
    }
    __device__ __forceinline__ void done() {
        if (n && (uint32_t)acc) __hip_atomic_fetch_or(&w[wi], (uint32_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

// The parse of one ~8 KiB sub-block by ONE WAVE (wave w: window positions [s0, se)), the
// twin's `parse` (oracle/zstd_twin.cpp) step for step:
//   history  every position of [wlo, s0) enters the table, 8 per lane a step (insert only:
//            the table keeps the last position per hash, whatever the order);
//   rounds   of kZRound positions (lane l, slot i: r0 + (l + 64 i) step): the table lookups
//            before this round's inserts, then per position -- from the walk's position `cur`
//            and repeat offset `rep` at the round start only -- the candidate (the repeat
//            offset when it matches kZMin bytes, else the longer of the table's and the run
//            candidate p - 1), its length capped at kZCap and how far it extends backwards
//            (<= kZBack bytes), packed into one VGPR per slot;
//   walk     wave-uniform scalar steps over the round's match masks: the first match at or
//            after cur is taken (started up to its backward extension earlier, never before
//            cur), a capped one extended forwards to its end, cur moved to the end.  A step
//            is a few scalar instructions and one readlane -- no LDS round trip, no ballot --
//            except for a capped match.  (Round 4's walk measured every length, repeat match
//            and backward extension inside the step: ~280 instructions and two LDS round trips
//            per sequence, ~0.75 us.)
// The sequences go to wseq (block positions, 64 at a time from lane registers); returns
// their count | the end of the last match (block position) << 32.
__device__ __noinline__ uint64_t parse_subblock(const Win W, lds_u16* __restrict__ tabs, Seq* __restrict__ wseq_g,
                                                uint32_t hist, uint32_t N, int wave, int lane,
                                                unsigned long long* probe) {
    PBS_GLOBAL uint32_t* const wseq_w = (PBS_GLOBAL uint32_t*)(wseq_g + (uint64_t)wave * kZSubSeq);
    const uint64_t t_in = probe ? wall_clock64() : 0;
    uint64_t t_hist = t_in;
    const uint32_t s0 = uni(hist + zsub_start(wave));
    uint32_t ns = 0, lastend = 0;
    if (s0 < N) {
        const uint32_t se = uni(min(hist + zsub_start(wave + 1), N));
        const uint32_t wlo = uni(s0 - min(s0, kZWin));
        lds_u16* const tw = tabs + wave * kZTab;
#pragma unroll
        for (int i = 0; i < (int)(kZTab / 2 / 64); ++i) reinterpret_cast<lds_u32*>(tw)[lane + 64 * i] = 0;
        // history: [wlo, s0) in rounds of kZHistRound positions every hs bytes (inserts only);
        // slot 0 (the round's first 64 positions) also looks up its candidates first: a
        // kZMin-byte match (not a run of one byte) sets the next round's step to
        // kZHistMinStep, else it doubles up to kZHistMaxStep (random bytes need no dense
        // history)
        uint32_t hs = kZHistStep0;
        for (uint32_t r0 = wlo, rn; r0 < s0; r0 = rn) {
            rn = r0 + kZHistRound * hs;
            uint32_t h[kZPerH], v[kZPerH], lo[kZPerH], hi[kZPerH], o3[kZPerH];
            bool ok[kZPerH];
#pragma unroll
            for (int i = 0; i < kZPerH; ++i) {
                const uint32_t p = r0 + ((uint32_t)lane + 64u * (uint32_t)i) * hs;
                ok[i] = p < s0 && p + kZMin <= N;
                const uint32_t o = (ok[i] ? p : wlo) + W.r;
                lo[i] = W.w[o >> 2];
                hi[i] = W.w[(o >> 2) + 1];
                o3[i] = o & 3;
                v[i] = p - wlo + 1;
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * kZPerH, 0);  // the DS reads first
#pragma unroll
            for (int i = 0; i < kZPerH; ++i)
                h[i] = hash5(__builtin_amdgcn_alignbyte(hi[i], lo[i], o3[i]), (hi[i] >> (8 * o3[i])) & 0xFF);
            const uint32_t w0 = __builtin_amdgcn_alignbyte(hi[0], lo[0], o3[0]), b40 = (hi[0] >> (8 * o3[0])) & 0xFF;
            const uint32_t t0 = ok[0] ? (uint32_t)tw[h[0]] : 0u;  // slot 0: before the inserts
            tab_max_batch<kZPerH>(tw, h, v, ok);
            uint32_t c4;
            const uint32_t cw = W.word5(t0 ? wlo + t0 - 1 : wlo, c4);
            const uint32_t b = w0 & 0xFF;
            const bool run = w0 == b * 0x01010101u && b40 == b;
            const bool hit = t0 && !run && cw == w0 && c4 == b40;
            hs = uni(__ballot(hit) ? kZHistMinStep : min(2 * hs, kZHistMaxStep));
        }
        if (probe) t_hist = wall_clock64();
        uint64_t t_walk = 0;
        uint32_t cur = s0, step = min(hs, kZMaxStep), lstep = 31 - __builtin_clz(step), rep = 0;
        for (uint32_t r0 = s0, rn; r0 < se; r0 = rn) {
            uint64_t tq = probe ? wall_clock64() : 0;
            auto qmark = [&](int idx) {  // (probe: the round's parts)
                if (probe) {
                    const uint64_t t2 = wall_clock64();
                    probe[idx] += t2 - tq;
                    tq = t2;
                }
            };
            rn = r0 + kZRound * step;
            uint32_t P[kZPer], h[kZPer], t[kZPer], wp[kZPer], b4[kZPer], lo[kZPer], hi[kZPer], o3[kZPer], pm1[kZPer];
            bool okp[kZPer];
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                P[i] = r0 + ((uint32_t)lane + 64u * (uint32_t)i) * step;
                okp[i] = P[i] < se && P[i] + kZMin <= N;
                const uint32_t o = (okp[i] ? P[i] : s0) + W.r;
                lo[i] = W.w[o >> 2];
                hi[i] = W.w[(o >> 2) + 1];
                o3[i] = o & 3;
                pm1[i] = W.byte(P[i] > wlo && okp[i] ? P[i] - 1 : s0);  // (the run candidate's first byte)
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 3 * kZPer, 0);
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                b4[i] = (hi[i] >> (8 * o3[i])) & 0xFF;
                wp[i] = __builtin_amdgcn_alignbyte(hi[i], lo[i], o3[i]);
                h[i] = hash5(wp[i], b4[i]);
                t[i] = okp[i] ? (uint32_t)tw[h[i]] : 0u;
            }
            {
                uint32_t v[kZPer];
#pragma unroll
                for (int i = 0; i < kZPer; ++i) v[i] = P[i] - wlo + 1;
                tab_max_batch<kZPer>(tw, h, v, okp);
            }
            qmark(43);
            // the table's and the repeat offset's candidate words: all reads first
            uint32_t clo[kZPer], chi[kZPer], co3[kZPer], rlo[kZPer], rhi[kZPer], ro3[kZPer];
            bool rok[kZPer];
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                const uint32_t oc = (t[i] ? wlo + t[i] - 1 : s0) + W.r;
                clo[i] = W.w[oc >> 2];
                chi[i] = W.w[(oc >> 2) + 1];
                co3[i] = oc & 3;
                rok[i] = rep && okp[i] && P[i] >= wlo + rep;
                const uint32_t orp = (rok[i] ? P[i] - rep : s0) + W.r;
                rlo[i] = W.w[orp >> 2];
                rhi[i] = W.w[(orp >> 2) + 1];
                ro3[i] = orp & 3;
            }
            // per position: the candidate S (+ the run candidate as the alternative when the
            // table's and the run's both match), from the round-start cur and rep only
            uint32_t S[kZPer], lim[kZPer], L[kZPer], La[kZPer];
            bool go[kZPer], goA[kZPer], both[kZPer], has[kZPer], isrep[kZPer];
            bool anyA = false;
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                const bool live = okp[i] && P[i] >= cur && P[i] + kZMin <= se;
                const uint32_t c4 = (chi[i] >> (8 * co3[i])) & 0xFF;
                const uint32_t cw = __builtin_amdgcn_alignbyte(chi[i], clo[i], co3[i]);
                const bool mt = live && t[i] && cw == wp[i] && c4 == b4[i];
                const uint32_t b = wp[i] & 0xFF;
                const bool mr = live && P[i] > wlo && wp[i] == b * 0x01010101u && b4[i] == b && pm1[i] == b;
                const uint32_t r4 = (rhi[i] >> (8 * ro3[i])) & 0xFF;
                const uint32_t rw = __builtin_amdgcn_alignbyte(rhi[i], rlo[i], ro3[i]);
                const bool mrep = live && rok[i] && rw == wp[i] && r4 == b4[i];
                S[i] = mrep ? P[i] - rep : mt ? wlo + t[i] - 1 : P[i] - 1;
                has[i] = mrep || mt || mr;
                isrep[i] = mrep;
                go[i] = has[i];
                both[i] = !mrep && mt && mr;
                goA[i] = both[i];
                anyA |= goA[i];
                lim[i] = has[i] ? min(se - P[i], kZCap) : 0u;
                L[i] = lim[i];
                La[i] = lim[i];
            }
            qmark(44);
            // lengths: the common prefix from byte 4 on (bytes 0-4 are equal), 8 bytes a step
            // (a lane done, or not matching, reads the sub-block start on both sides: one
            // address for all of them, a broadcast, where its own position cost the LDS a
            // bank access per lane), a slot only while one of its lanes goes on
            const bool alt = __ballot(anyA) != 0;
            for (uint32_t k = 4; k < kZCap; k += 8) {
                bool more = false;
                // every slot's words read together (one wait for all of them), the alternative's
                // too when any lane has one
                uint32_t xd0[kZPer], xd1[kZPer], xa0[kZPer], xa1[kZPer];
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    const bool g = go[i] && k < lim[i];
                    const uint32_t sa = g ? S[i] + k : s0, pa = g ? P[i] + k : s0;
                    xd0[i] = W.word(sa) ^ W.word(pa);
                    xd1[i] = W.word(sa + 4) ^ W.word(pa + 4);
                }
                if (alt) {
#pragma unroll
                    for (int i = 0; i < kZPer; ++i) {
                        const bool ga = goA[i] && k < lim[i];
                        const uint32_t sb2 = ga ? P[i] - 1 + k : s0, pb2 = ga ? P[i] + k : s0;
                        xa0[i] = W.word(sb2) ^ W.word(pb2);
                        xa1[i] = W.word(sb2 + 4) ^ W.word(pb2 + 4);
                    }
                }
#pragma unroll
                for (int i = 0; i < kZPer; ++i) {
                    const uint32_t d0 = xd0[i], d1 = xd1[i];
                    if (go[i]) {
                        if (k >= lim[i]) {
                            go[i] = false;
                        } else if (d0 | d1) {
                            const uint32_t f = d0 ? (uint32_t)__builtin_ctz(d0) >> 3 : 4u + ((uint32_t)__builtin_ctz(d1) >> 3);
                            L[i] = min(lim[i], k + f);
                            go[i] = false;
                        }
                    }
                    if (alt && goA[i]) {
                        const uint32_t a0 = xa0[i], a1 = xa1[i];
                        if (k >= lim[i]) {
                            goA[i] = false;
                        } else if (a0 | a1) {
                            const uint32_t f = a0 ? (uint32_t)__builtin_ctz(a0) >> 3 : 4u + ((uint32_t)__builtin_ctz(a1) >> 3);
                            La[i] = min(lim[i], k + f);
                            goA[i] = false;
                        }
                    }
                    more |= go[i] || goA[i];
                }
                if (!__ballot(more)) break;
            }
            qmark(45);
            // the choice, the backward extension (table and run candidates, at most kZBack
            // bytes, never before the window) and the packed record per slot
            uint32_t D[kZPer];
            unsigned long long m[kZPer];
            // the backward extension's words, every slot's read together (a slot without a
            // table or run candidate, or too near the window start, reads position 8: one
            // address for all such lanes, a broadcast)
            uint32_t bx1[kZPer], bx2[kZPer];
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                if (both[i] && La[i] > L[i]) {  // the run's is longer (ties: the table's)
                    S[i] = P[i] - 1;
                    L[i] = La[i];
                }
                const bool ok = has[i] && !isrep[i] && S[i] >= 8;
                const uint32_t pp = ok ? P[i] : 8u, ss = ok ? S[i] : 8u;
                bx1[i] = W.word(pp - 4) ^ W.word(ss - 4);
                bx2[i] = W.word(pp - 8) ^ W.word(ss - 8);
            }
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                uint32_t e = 0;
                if (has[i] && !isrep[i]) {
                    const uint32_t emax = min(kZBack, S[i] - wlo);
                    if (S[i] >= 8) {
                        const uint32_t x1 = bx1[i], x2 = bx2[i];
                        e = x1 ? (uint32_t)__builtin_clz(x1) >> 3 : 4u + (x2 ? (uint32_t)__builtin_clz(x2) >> 3 : 4u);
                    } else {
                        while (e < emax && W.byte(P[i] - 1 - e) == W.byte(S[i] - 1 - e)) ++e;
                    }
                    e = min(e, emax);
                }
                D[i] = has[i] ? (S[i] - wlo) | L[i] << 16 | e << 24 : 0u;
            }
#pragma unroll
            for (int i = 0; i < kZPer; ++i) m[i] = __ballot(has[i]);
            // each match position's successor on the chain: the first match position at or
            // after its end (index q + ceil(L / step); a length under kZCap is at most 31, so
            // the end lies in this slot or the next), 256 when the chain leaves the round,
            // kZCapped when the length is capped (the walk extends it and looks itself)
            constexpr uint32_t kZNone = 256, kZCapped = 512;
            uint32_t first_from[kZPer + 2];  // first match index in slots >= i (uniform)
            first_from[kZPer] = first_from[kZPer + 1] = kZNone;
#pragma unroll
            for (int i = kZPer - 1; i >= 0; --i)
                first_from[i] = m[i] ? 64u * (uint32_t)i + (uint32_t)__builtin_ctzll(m[i]) : first_from[i + 1];
            uint32_t Sx[kZPer];
#pragma unroll
            for (int i = 0; i < kZPer; ++i) {
                const uint32_t q = 64u * (uint32_t)i + (uint32_t)lane;
                const uint32_t Lh = (D[i] >> 16) & 0xFF;
                const uint32_t b = (uint32_t)lane + ((Lh + step - 1) >> lstep);  // the end, from slot i's start
                const unsigned long long mi = b < 64 ? m[i] & (~0ull << b) : 0ull;
                const unsigned long long mn = i + 1 < kZPer ? (b < 64 ? m[i + 1 < kZPer ? i + 1 : i]
                                                                     : m[i + 1 < kZPer ? i + 1 : i] & (~0ull << (b - 64)))
                                                            : 0ull;
                const uint32_t next = mi ? 64u * (uint32_t)i + (uint32_t)__builtin_ctzll(mi)
                                         : mn ? 64u * (uint32_t)(i + 1) + (uint32_t)__builtin_ctzll(mn) : first_from[i + 2];
                Sx[i] = Lh == kZCap ? kZCapped : q + ((Lh + step - 1) >> lstep) >= kZRound ? kZNone : next;
            }
            qmark(46);
            if (probe) {
                t_walk = wall_clock64();
                probe[33] += 1;  // rounds
            }
            // the walk: wave-uniform scalar steps along the chain -- read the successor of the
            // position taken, append the position to the path (lane k of `path`; a capped
            // match's full length to `pathL`).  Slot by slot, so each slot's successor register
            // is named directly.  Every 64 positions (and at the end) the path's records are
            // written by the lanes in parallel (flush).
            const uint32_t cur0 = cur;
            uint32_t path = 0, pathL = 0, k = 0;
            uint32_t carry = cur0;  // the previous match's end
            bool found = false;
            auto flush = [&](uint32_t K) {
                // lane j < K: path position q; its packed record from its slot and lane
                const uint32_t q = path & 0x3FF, l4 = (q & 63) * 4;
                const uint32_t d0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l4, (int)D[0]),
                               d1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l4, (int)D[1]),
                               d2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l4, (int)D[2]),
                               d3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l4, (int)D[3]);
                const uint32_t sl = q >> 6;
                const uint32_t d = sl == 0 ? d0 : sl == 1 ? d1 : sl == 2 ? d2 : d3;
                const uint32_t pq = r0 + (q << lstep);
                const uint32_t Lq = (path & 0x400) ? pathL : (d >> 16) & 0xFF;
                const uint32_t end = pq + Lq;
                const uint32_t up = (uint32_t)__shfl_up((int)end, 1, 64);
                const uint32_t prev_end = lane ? up : carry;
                const uint32_t e = min(d >> 24, pq - prev_end);
                const uint32_t Sq = wlo + (d & 0xFFFF);
                if ((uint32_t)lane < K && ns + (uint32_t)lane < kZSubSeq) {
                    PBS_GLOBAL uint32_t* const rec = wseq_w + 3 * (ns + (uint32_t)lane);
                    rec[0] = pq - e - hist;
                    rec[1] = Lq + e;
                    rec[2] = pq - Sq;
                }
                carry = uni((uint32_t)__builtin_amdgcn_readlane((int)end, (int)K - 1));
                rep = uni((uint32_t)__builtin_amdgcn_readlane((int)(pq - Sq), (int)K - 1));
                ns = uni(ns + K);
                found = true;
            };
            // the first match at or after the round-start position
            uint32_t q = uni(cur > r0 ? (cur - r0 + step - 1) >> lstep : 0);
            {
                const uint32_t w0 = q >> 6;
                uint32_t f = kZNone;
                if (q < kZRound) {
                    const unsigned long long mm =
                        (w0 == 0 ? m[0] : w0 == 1 ? m[1] : w0 == 2 ? m[2] : m[3]) & (~0ull << (q & 63));
                    f = mm ? 64u * w0 + (uint32_t)__builtin_ctzll(mm)
                           : (w0 == 0 ? first_from[1] : w0 == 1 ? first_from[2] : w0 == 2 ? first_from[3] : kZNone);
                }
                q = uni(f);
            }
#pragma unroll
            for (int wi = 0; wi < kZPer; ++wi) {
                while (q < 64u * (uint32_t)(wi + 1)) {
                    const uint32_t l = q & 63;
                    uint32_t nxt = (uint32_t)__builtin_amdgcn_readlane((int)Sx[wi], (int)l);
                    uint32_t tag = q;
                    if (__builtin_expect(nxt == kZCapped, 0)) {
                        // forwards to the end (within the sub-block): 16 bytes per lane a step,
                        // their word reads issued together
                        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)D[wi], (int)l);
                        const uint32_t p = uni(r0 + (q << lstep)), S0 = wlo + (d & 0xFFFF);
                        uint32_t Lc = kZCap;
                        const uint32_t kk = (uint32_t)lane;
                        for (;;) {
                            const uint32_t xf = p + Lc + 16 * kk, xs = S0 + Lc + 16 * kk;
                            uint32_t mis = 16;
                            if (xf + 16 <= se) {
                                uint32_t dd[4];
#pragma unroll
                                for (int k2 = 0; k2 < 4; ++k2) dd[k2] = W.word(xs + 4 * k2) ^ W.word(xf + 4 * k2);
#pragma unroll
                                for (int k2 = 3; k2 >= 0; --k2)
                                    if (dd[k2]) mis = 4 * (uint32_t)k2 + ((uint32_t)__builtin_ctz(dd[k2]) >> 3);
                            } else {
                                mis = 0;
                                while (xf + mis < se && W.byte(xs + mis) == W.byte(xf + mis)) ++mis;
                            }
                            const unsigned long long bad = __ballot(mis < 16);
                            if (bad) {
                                const int f = __builtin_ctzll(bad);
                                Lc += 16 * (uint32_t)f + (uint32_t)__builtin_amdgcn_readlane((int)mis, f);
                                break;
                            }
                            Lc += 1024;
                        }
                        Lc = uni(Lc);
                        asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(pathL) : "s"(Lc), "{m0}"(k));
                        tag = q | 0x400;
                        // the first match at or after its end
                        const uint32_t x = uni(q + ((Lc + step - 1) >> lstep));
                        uint32_t f = kZNone;
                        if (x < kZRound) {
                            const uint32_t w0 = x >> 6;
                            const unsigned long long mm =
                                (w0 == 0 ? m[0] : w0 == 1 ? m[1] : w0 == 2 ? m[2] : m[3]) & (~0ull << (x & 63));
                            f = mm ? 64u * w0 + (uint32_t)__builtin_ctzll(mm)
                                   : (w0 == 0 ? first_from[1] : w0 == 1 ? first_from[2] : w0 == 2 ? first_from[3] : kZNone);
                        }
                        nxt = uni(f);
                    }
                    asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(path) : "s"(tag), "{m0}"(k));
                    ++k;
                    if (k == 64) {
                        flush(64);
                        k = 0;
                    }
                    q = nxt;
                }
            }
            if (k) flush(k);
            if (probe) {
                const uint64_t t2 = wall_clock64();
                probe[32] += t2 - t_walk;  // walk time (records inside)
                t_walk = t2;
            }
            if (found) {
                cur = carry;  // the last match's end
                lastend = cur - hist;
            }
            if (probe) probe[42] += wall_clock64() - t_walk;  // sequence records
            step = found ? 1 : min(2 * step, kZMaxStep);
            lstep = 31 - __builtin_clz(step);
            if (cur > rn) rn = cur;  // positions inside a match that ran past the round: not searched
        }
    }
    if (probe && lane == 0 && s0 < N) {  // wave 0 of workgroup 0: history / rounds + walk
        probe[13] += t_hist - t_in;
        probe[14] += wall_clock64() - t_hist;
    }
    return (uint64_t)ns | (uint64_t)lastend << 32;
}

// Two-queue Huffman merge (one lane): leaves 0..m-1 = the symbols sorted by (count,
// symbol) (E.tw holds their weights on entry, E.keys the symbols), internal nodes m.. in
// creation order, ties taking the leaf; parents in E.par, the root in ctl.root.  A step reads
// the two heads of both queues at once (one LDS wait, not one per pop): the second pop
// takes from these four; a head past its queue is read but not used.
template <class EA>
__device__ __noinline__ void huf_merge(EA& E, Ctl& ctl, uint32_t dist) {
        const int m = (int)dist;
        int li = 0, ii = m, nn = m;
        while (nn < 2 * m - 1) {
            const uint32_t l0 = E.tw[li], l1 = E.tw[li + 1], i0 = E.tw[ii], i1 = E.tw[ii + 1];
            int a, b;
            uint32_t wa, wb;
            if (li < m && (ii >= nn || l0 <= i0)) {
                a = li++;
                wa = l0;
                if (li < m && (ii >= nn || l1 <= i0)) { b = li++; wb = l1; } else { b = ii++; wb = i0; }
            } else {
                a = ii++;
                wa = i0;
                if (li < m && (ii >= nn || l0 <= i1)) { b = li++; wb = l0; } else { b = ii++; wb = i1; }
            }
            E.tw[nn] = wa + wb;
            E.par[a] = (uint16_t)nn;
            E.par[b] = (uint16_t)nn;
            ++nn;
        }
        ctl.root = nn - 1;
}


// Literal section mode of a block (ONE WAVE): RLE (one distinct byte), raw, or Huffman
// when the entropy estimate says it may pay -- then the code lengths (two-queue merge,
// limited to 11 bits), canonical codes and the tree description.  ctl.lit_mode = lane 0's.
template <class EA>
__device__ __noinline__ void literal_mode_wave(EA& E, Ctl& ctl, FseT& fsc, uint32_t nlit, int lane,
                                               unsigned long long* probe) {
    uint64_t tq = probe ? wall_clock64() : 0;
    auto mark = [&](int idx) {
        if (probe && lane == 0) {
            const uint64_t t2 = wall_clock64();
            probe[idx] += t2 - tq;
            tq = t2;
        }
    };
    uint32_t c4[4], dist = 0, lastsym = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        c4[i] = E.hist[lane + 64 * i];
        const unsigned long long b = __ballot(c4[i] != 0);
        dist += (uint32_t)__builtin_popcountll(b);
        if (b) lastsym = 64 * i + 63 - (uint32_t)__builtin_clzll(b);
    }
    // 0 raw, 1 RLE, 2 Huffman (if its exact size wins below)
    uint32_t mode = 0;
    if (nlit > 0 && dist == 1) {
        mode = 1;
    } else if (nlit >= 32) {
        uint64_t est = 0;
        const uint32_t ln = lg256(nlit);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (c4[i]) est += (uint64_t)c4[i] * (ln - lg256(c4[i]));
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) est += __shfl_xor(est, d, 64);
        if (est / 2048 + 64 < (uint64_t)nlit - nlit / 64) mode = 2;
    }
    if (mode == 2) {
        // symbols sorted by (count, symbol): rank of each key among the present ones
        uint32_t key[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            key[i] = c4[i] << 8 | (uint32_t)(lane + 64 * i);
            E.keys[lane + 64 * i] = c4[i] ? key[i] : 0xFFFFFFFFu;
        }
        __builtin_amdgcn_wave_barrier();  // one wave: LDS ops run in order; no code motion across
        uint32_t rk[4] = {0, 0, 0, 0};
        for (int s2 = 0; s2 < 256; ++s2) {
            const uint32_t o = E.keys[s2];
#pragma unroll
            for (int i = 0; i < 4; ++i) rk[i] += o < key[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (c4[i]) E.tw[rk[i]] = key[i];  // sorted keys (temporarily in tw)
        mark(26);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // sorted symbols and leaf weights, by lane
            const uint32_t q = (uint32_t)lane + 64u * (uint32_t)i;
            if (q < dist) {
                const uint32_t kv = E.tw[q];
                E.keys[q] = kv & 0xFF;
                E.tw[q] = kv >> 8;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) huf_merge(E, ctl, dist);
        __builtin_amdgcn_wave_barrier();
        mark(27);
        const int m = (int)dist, root = ctl.root;
        // depth of each leaf (sorted index i = 4 lane + j: contiguous per lane)
        int32_t kr = 0;
        uint32_t L4[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int i = 4 * lane + jj;
            uint32_t d = 0;
            if (i < m)
                for (int nd = i; nd != root; nd = E.par[nd]) ++d;
            L4[jj] = i < m ? min(d, kHufMax) : 0u;
            if (i < m) kr += 1 << (kHufMax - L4[jj]);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) kr += __shfl_xor(kr, d, 64);
        kr -= 1 << kHufMax;
        while (kr > 0) {  // lengthen the longest code under the limit, least frequent first
            uint32_t best = 0;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const uint32_t i = 4 * lane + jj;
                if ((int)i < m && L4[jj] < kHufMax) best = max(best, L4[jj] << 16 | (0xFFFFu - i));
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, d, 64));
            const uint32_t bi = 0xFFFFu - (best & 0xFFFFu), bl = best >> 16;
            kr -= 1 << (kHufMax - bl - 1);
            if ((bi >> 2) == (uint32_t)lane) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if ((bi & 3) == (uint32_t)jj) ++L4[jj];
            }
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) E.lens[4 * lane + jj] = (uint8_t)L4[jj];
        if (lane == 0 && kr < 0) {  // shorten: most frequent first, while the deficit allows
            while (kr < 0)
                for (int i = m - 1; i >= 0 && kr < 0; --i) {
                    uint32_t L = E.lens[i];
                    while (L > 1 && (1 << (kHufMax - L)) <= -kr) {
                        kr += 1 << (kHufMax - L);
                        --L;
                    }
                    E.lens[i] = (uint8_t)L;
                }
        }
        __builtin_amdgcn_wave_barrier();
        mark(28);
        // per symbol lengths
#pragma unroll
        for (int i = 0; i < 4; ++i) E.len[lane + 64 * i] = 0;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int i = 4 * lane + jj;
            if (i < m) E.len[E.keys[i]] = E.lens[i];
        }
        __builtin_amdgcn_wave_barrier();
        // canonical codes: by (length descending, symbol ascending), increasing
        uint32_t ls[4], mb = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ls[i] = E.len[lane + 64 * i];
            mb = max(mb, ls[i]);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) mb = max(mb, (uint32_t)__shfl_xor((int)mb, d, 64));
        uint32_t start[kHufMax + 2];
        {
            uint32_t cntL[kHufMax + 2];
            for (uint32_t L = 0; L <= kHufMax + 1; ++L) cntL[L] = 0;
            for (uint32_t L = 1; L <= kHufMax; ++L) {
                uint32_t c = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) c += (uint32_t)__builtin_popcountll(__ballot(ls[i] == L));
                cntL[L] = c;
            }
            uint32_t prevL = 0, s = 0;
            for (uint32_t L = mb; L >= 1; --L) {
                if (!cntL[L]) continue;
                start[L] = prevL ? (s >> (prevL - L)) : 0u;
                s = start[L] + cntL[L];
                prevL = L;
            }
        }
        // rank among the same length by symbol (symbols lane + 64 i): per length, the
        // ballots of the four symbol groups in order
        {
            uint32_t rk[4] = {0, 0, 0, 0};
            const unsigned long long lt = (1ull << lane) - 1ull;
            for (uint32_t L = 1; L <= mb; ++L) {
                uint32_t acc = 0;
#pragma unroll
                for (int i2 = 0; i2 < 4; ++i2) {
                    const unsigned long long b = __ballot(ls[i2] == L);
                    if (ls[i2] == L) rk[i2] = acc + (uint32_t)__builtin_popcountll(b & lt);
                    acc += (uint32_t)__builtin_popcountll(b);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (ls[i]) E.code[lane + 64 * i] = (uint16_t)(start[ls[i]] + rk[i]);
        }
        mark(29);
        if (!huf_describe(E, ctl, fsc, mb, lastsym, lane)) mode = 0;
        mark(30);
    }
    if (lane == 0) ctl.lit_mode = mode;  // (lane 0's: it may have fallen back to raw)
}

// The literal section (all threads): Huffman streams ORed into LDS at offsets from the
// block scan of code lengths and copied out, or raw bytes compacted through LDS, or the
// RLE byte.  Thread t's literals are the set bits of bm (block positions 128 t ..).
__device__ __noinline__ void write_literals(EntropyArea& E, const Ctl& ctl, const Win W, uint32_t hist, uint4 bm4,
                                            uint32_t litbase, uint32_t bbase, uint32_t nlit, uint32_t lm, bool four,
                                            uint32_t seg, uint8_t* lit_out, int tid, uint32_t nruns) {
    const uint32_t bmw[4] = {bm4.x, bm4.y, bm4.z, bm4.w};
    if (lm == 2) {
        const uint32_t words = kHufStreams / 4 + 4;
        for (uint32_t i = tid; i < words; i += kZThreads) E.streams[i] = 0;
        __syncthreads();
        // stream s starts at byte S_s of the LDS buffer
        // (scalars, not an array: a dynamically indexed array would live in scratch memory)
        const uint32_t S0 = 0;
        const uint32_t S1 = four ? (ctl.segP[1] - ctl.segP[0] + 8) / 8 : (ctl.segP[4] - ctl.segP[0] + 8) / 8;
        const uint32_t S2 = four ? S1 + (ctl.segP[2] - ctl.segP[1] + 8) / 8 : S1;
        const uint32_t S3 = four ? S2 + (ctl.segP[3] - ctl.segP[2] + 8) / 8 : S1;
        const uint32_t S4 = four ? S3 + (ctl.segP[4] - ctl.segP[3] + 8) / 8 : S1;
        auto Sat = [&](uint32_t g) { return g == 0 ? S0 : g == 1 ? S1 : g == 2 ? S2 : g == 3 ? S3 : S4; };
        uint32_t idx = litbase, pb = bbase;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1) {
                const uint32_t sym = W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2));
                const uint32_t L = E.len[sym], cv = E.code[sym];
                const uint32_t sg = four ? min(idx / seg, 3u) : 0u;
                const uint32_t endP = four ? ctl.segP[sg + 1] : ctl.segP[4];
                const uint32_t o = 8 * Sat(sg) + (endP - pb - L);
                const uint64_t v = (uint64_t)cv << (o & 31);
                atomicOr(&E.streams[o >> 5], (uint32_t)v);
                if ((o & 31) + L > 32) atomicOr(&E.streams[(o >> 5) + 1], (uint32_t)(v >> 32));
                pb += L;
                ++idx;
            }
        if (tid < (four ? 4 : 1)) {  // end marks
            const uint32_t bits = ctl.segP[four ? tid + 1 : 4] - ctl.segP[tid];
            const uint32_t o = 8 * Sat((uint32_t)tid) + bits;
            atomicOr(&E.streams[o >> 5], 1u << (o & 31));
        }
        __syncthreads();
        const uint32_t hs = ctl.huf_hs, c = ctl.huf_c;
        const uint32_t dl = ctl.desc_len;
        uint8_t* const body = lit_out + hs;
        if (tid == 0) {
            if (hs == 3) {
                const uint32_t v = 2u | (four ? 1u : 0u) << 2 | nlit << 4 | c << 14;
                lit_out[0] = (uint8_t)v;
                lit_out[1] = (uint8_t)(v >> 8);
                lit_out[2] = (uint8_t)(v >> 16);
            } else if (hs == 4) {
                const uint32_t v = 2u | 2u << 2 | nlit << 4 | c << 18;
                for (int i = 0; i < 4; ++i) lit_out[i] = (uint8_t)(v >> (8 * i));
            } else {
                const uint64_t v = 2u | 3u << 2 | (uint64_t)nlit << 4 | (uint64_t)c << 22;
                for (int i = 0; i < 5; ++i) lit_out[i] = (uint8_t)(v >> (8 * i));
            }
            if (four)
                for (int s = 0; s < 3; ++s) {
                    const uint32_t sz = Sat((uint32_t)s + 1) - Sat((uint32_t)s);
                    body[dl + 2 * s] = (uint8_t)sz;
                    body[dl + 2 * s + 1] = (uint8_t)(sz >> 8);
                }
        }
        for (uint32_t i = tid; i < dl; i += kZThreads) body[i] = ctl.desc[i];
        const uint32_t tot = four ? S4 : S1;
        lds_to_global(body + dl + (four ? 6 : 0), E.streams, tot, (uint32_t)tid, kZThreads);
    } else {
        const uint32_t rawh = nlit < 32 ? 1u : nlit < 4096 ? 2u : 3u;
        if (tid == 0) {
            const uint32_t t = lm;  // 0 raw, 1 RLE
            if (rawh == 1) {
                lit_out[0] = (uint8_t)(t | nlit << 3);
            } else if (rawh == 2) {
                lit_out[0] = (uint8_t)(t | 1u << 2 | nlit << 4);
                lit_out[1] = (uint8_t)(nlit >> 4);
            } else {
                lit_out[0] = (uint8_t)(t | 3u << 2 | nlit << 4);
                lit_out[1] = (uint8_t)(nlit >> 4);
                lit_out[2] = (uint8_t)(nlit >> 12);
            }
        }
        if (lm == 1) {
            if (tid == 0) {  // the one distinct byte
                uint32_t s = 0;
                while (!E.hist[s]) ++s;
                lit_out[rawh] = (uint8_t)s;
            }
        } else if (nruns) {
            // few sequences: run by run, every thread on each run (coalesced dword stores)
            for (uint32_t r = 0; r < nruns; ++r)
                stage_to_global(lit_out + rawh + ctl.run_out[r], W, hist + ctl.run_start[r], ctl.run_len[r],
                                (uint32_t)tid, kZThreads);
        } else {
            // compacted through LDS (the stream buffer, free here) in pieces of 48 KiB, then
            // copied out with dword stores: scattered global byte stores cost a line each
            uint8_t* const lb = reinterpret_cast<uint8_t*>(E.streams);
            for (uint32_t pb = 0; pb < nlit; pb += kHufStreams) {
                const uint32_t pe = min(nlit, pb + kHufStreams);
                uint32_t idx = litbase;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1, ++idx)
                        if (idx >= pb && idx < pe)
                            lb[idx - pb] = (uint8_t)W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2));
                __syncthreads();
                lds_to_global(lit_out + rawh + pb, E.streams, pe - pb, (uint32_t)tid, kZThreads);
                __syncthreads();
            }
        }
    }
}

// Repeat-offset coding of sub-block w2 by ONE WAVE (the repeat offsets are tracked per
// sub-block): literal lengths, offset values, codes.  The offsets are a serial state
// machine, but its state is the last three offsets, so it forgets its past: lane l codes
// the sequences [l seg, (l+1) seg) from the state reached by running the machine over the
// 8 sequences before them from empty (lane 0: the true start); then, in rounds, a lane
// whose start differs from its left neighbour's end re-codes from that end.
__device__ __forceinline__ void rep_step(uint32_t& ra, uint32_t& rb, uint32_t& rc3, uint32_t o, bool ll0,
                                         uint32_t& ofv) {
    ofv = o + 3;
    if (!ll0 && ra == o) ofv = 1;
    else if (rb && rb == o) ofv = ll0 ? 1 : 2;
    else if (rc3 && rc3 == o) ofv = ll0 ? 2 : 3;
    else if (ll0 && ra > 1 && ra - 1 == o) ofv = 3;
    if (ofv > 3) {
        rc3 = rb;
        rb = ra;
        ra = o;
    } else {
        const uint32_t rcode = ofv - 1 + (ll0 ? 1u : 0u);
        if (rcode > 0) {
            const uint32_t cu = rcode == 3 ? ra - 1 : rcode == 1 ? rb : rc3;
            if (rcode >= 2) rc3 = rb;
            rb = ra;
            ra = cu;
        }
    }
}

__device__ __forceinline__ Seq ld_seq(const PBS_GLOBAL Seq* p) {
    const PBS_GLOBAL uint32_t* q = (const PBS_GLOBAL uint32_t*)p;
    return Seq{q[0], q[1], q[2]};
}
__device__ __forceinline__ void st_coded(PBS_GLOBAL Coded* p, const Coded& c) {
    *(PBS_GLOBAL v4u*)p = v4u{c.ll, c.ml, c.ofv, c.codes};
}

__device__ __noinline__ void rep_code_wave(const uint32_t* nseq, const uint32_t* lastend, const Seq* __restrict__ wseq_g,
                                           Coded* __restrict__ coded_g, uint32_t w2, int lane) {
    const PBS_GLOBAL Seq* const wseq_all = (const PBS_GLOBAL Seq*)wseq_g;
    PBS_GLOBAL Coded* const coded = (PBS_GLOBAL Coded*)coded_g;
    uint32_t first = 0, lit_end = 0;
    for (uint32_t v = 0; v < w2; ++v) {
        first += min(nseq[v], kZSubSeq);
        if (nseq[v]) lit_end = lastend[v];
    }
    const PBS_GLOBAL Seq* const ws = wseq_all + (uint64_t)w2 * kZSubSeq;
    const uint32_t cnt = min(nseq[w2], kZSubSeq);
    if (!cnt) return;
    const uint32_t seg = (cnt + 63) / 64;
    const uint32_t a = min(cnt, (uint32_t)lane * seg), b = min(cnt, a + seg);
    constexpr uint32_t kWarm = 8;
    // codes [from, to) from state (ra, rb, rc3); write: store the Coded entries
    auto run = [&](uint32_t from, uint32_t to, uint32_t& ra, uint32_t& rb, uint32_t& rc3, bool write) {
        uint32_t prev_end = from == 0 ? lit_end : 0u;
        if (from > 0) {
            const Seq p = ld_seq(ws + from - 1);
            prev_end = p.pos + p.ml;
        }
        for (uint32_t q0 = from; q0 < to; q0 += 8) {
            Seq e8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)  // 8 loads in flight
                if (q0 + u < to) e8[u] = ld_seq(ws + q0 + u);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (q0 + u >= to) break;
                const Seq e = e8[u];
                Coded c;
                c.ll = e.pos - prev_end;
                c.ml = e.ml;
                rep_step(ra, rb, rc3, e.off, c.ll == 0, c.ofv);
                if (write) {
                    c.codes = ll_code(c.ll) | ml_code(c.ml) << 8 | highbit(c.ofv) << 16;
                    st_coded(coded + first + q0 + u, c);
                }
                prev_end = e.pos + e.ml;
            }
        }
    };
    uint32_t sa = 0, sb = 0, sc = 0;  // the start state
    if (a < b && a > 0) run(a > kWarm ? a - kWarm : 0u, a, sa, sb, sc, false);
    uint32_t ea = sa, eb = sb, ec = sc;  // the end state
    if (a < b) run(a, b, ea, eb, ec, true);
    for (int round = 0; round < 64; ++round) {
        // the true start of lane l is lane l-1's end (lane 0: empty); empty segments pass it on
        const uint32_t la = (uint32_t)__shfl_up((int)ea, 1, 64), lb = (uint32_t)__shfl_up((int)eb, 1, 64),
                       lc = (uint32_t)__shfl_up((int)ec, 1, 64);
        const uint32_t wa = lane == 0 ? 0u : la, wb = lane == 0 ? 0u : lb, wc = lane == 0 ? 0u : lc;
        const bool differ = a < b && (wa != sa || wb != sb || wc != sc);  // (empty segments: trailing)
        if (!__ballot(differ)) break;
        if (differ) {
            sa = wa;
            sb = wb;
            sc = wc;
            ea = sa;
            eb = sb;
            ec = sc;
            run(a, b, ea, eb, ec, true);
        }
    }
}

// PBS_ZSTD_PROBE=1 (diagnostics): workgroup 0, thread 0 adds the wall-clock ticks (100 MHz)
// of each phase into g_zprobe: 0 stage + RLE, 1 parse, 2 literal bitmap + histogram,
// 3 literal mode / Huffman code + repeat codes, 4 code histograms + Huffman sizes,
// 5 sequence tables, 6 state chains + literal size, 7 literal section, 8 sequence bit
// stream, 9 block end; 10 blocks, 11 sequences, 12 literals; 13/14 wave 0's history and
// rounds + walk; 15 literal bitmap, 16 sampled histogram (both inside 2); per role (lane 0
// of the wave doing it): 17 literal mode (wave 0), 18 repeat coding (wave 1), 19 LL table
// (wave 1), 20 LL state chain (wave 1), 21 literal section (wave 0); long LL chains: 22 pass
// 1, 23 rounds (ticks), 24 rounds, 25 chains; Huffman (wave 0): 26 rank, 27 merge, 28
// lengths, 29 canonical codes, 30 description; 32/33 wave 0's walk ticks / rounds, 34 + w
// wave w's parse.
__device__ unsigned long long g_zprobe[64];  // (48..56: the split entropy kernel's phases)
// PBS_ZSTD_DEBUG_ITEM=k (diagnostics): the parse's sequences of item k -- per sub-block its
// count, then its kZSubSeq {pos, ml, off} records -- copied out for a diff with the twin's
// (zstd_twin_parse)
__device__ uint32_t g_zdbg[kZWaves * (1 + 3 * kZSubSeq)];
#define ZMARK(ph)                                  \
    do {                                           \
        if (probe) {                               \
            const uint64_t t_ = wall_clock64();    \
            g_zprobe[ph] += t_ - tp;               \
            tp = t_;                               \
        }                                          \
    } while (0)

__global__ __launch_bounds__(kZThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void zstd_block_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint64_t* __restrict__ items, uint64_t nitems, uint8_t* __restrict__ slots,
    uint64_t* __restrict__ sizes, Seq* __restrict__ seq_scratch, Coded* __restrict__ coded_scratch,
    uint32_t* __restrict__ chain_scratch, int probe_on, int64_t dbg_item) {
    __shared__ uint4 stage[kZStageWords];
    __shared__ __attribute__((aligned(16))) uint8_t work[64 * 1024];
    __shared__ FseT fse[3];  // LL, OF, ML
    __shared__ FseT fse_huf;  // the Huffman description's scratch (beside the sequence tables)
    __shared__ PreT pre[3];  // the predefined tables, same order
    __shared__ Ctl ctl;
    // (the wave index as a provably uniform value: everything derived from it -- a sub-block's
    // bounds, the parse's walk state -- then lives in SGPRs and branches on the scalar unit)
    const int tid = threadIdx.x, lane = tid & 63, wave = (int)uni((uint32_t)tid >> 6);
    const bool probe = probe_on && blockIdx.x == 0 && tid == 0;
    uint64_t tp = probe ? wall_clock64() : 0;
    uint16_t* const tabs = reinterpret_cast<uint16_t*>(work);
    EntropyArea& E = *reinterpret_cast<EntropyArea*>(work);
    Seq* const wseq_all = seq_scratch + (uint64_t)blockIdx.x * kZBlockSeq;
    Coded* const coded = coded_scratch + (uint64_t)blockIdx.x * kZBlockSeq;
    // per stream, per sequence: the emitted bits, then (as u16) the state before each step,
    // then (as bytes) the stream's codes in step order
    uint32_t* const chains = chain_scratch + (uint64_t)blockIdx.x * 6 * kZBlockSeq;
    if (wave == 0 && lane < 3) {  // the predefined tables, once per launch (fse[] as scratch)
        FseT& t = fse[lane];
        if (lane == 0) fse_build(t, kLLNorm, 36, kLLLog);
        if (lane == 1) fse_build(t, kOFNorm, 29, kOFLog);
        if (lane == 2) fse_build(t, kMLNorm, 53, kMLLog);
        PreT& q = pre[lane];
        for (int i = 0; i < 64; ++i) q.next[i] = t.next[i];
        for (int i = 0; i < 53; ++i) {
            q.dnb[i] = t.dnb[i];
            q.dfs[i] = t.dfs[i];
        }
        q.log = t.log;
    }

    for (uint64_t k = blockIdx.x; k < nitems; k += gridDim.x) {
        __syncthreads();  // LDS of the previous item
        ZMARK(9);
        const uint64_t it = items[k];
        const uint64_t ci = it >> 32, j = (uint32_t)it;
        const uint64_t c0 = bounds[2 * ci], c1 = bounds[2 * ci + 1];  // (chunk spans {start, end})
        const uint64_t len = c1 - c0, off = j * (uint64_t)kEncBlock;
        const uint32_t n = (uint32_t)(len > off ? (len - off < kEncBlock ? len - off : kEncBlock) : 0);
        const bool last = off + n == len;
        uint8_t* const out = slots + k * kSlot;
        if (n == 0) {  // the empty chunk's frame: one empty raw block
            if (tid == 0) {
                write_block_header(out, true, 0, 0);
                sizes[k] = 3;
            }
            continue;
        }
        const uint32_t hist = (uint32_t)(off < kZHist ? off : kZHist);  // window bytes before the block
        const uint32_t N = hist + n;
        // stage the aligned 16-byte words holding [src - hist, src + n)
        const uint8_t* const wsrc = data + (c0 - base) + off - hist;
        const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(wsrc) & 15);
        const uint8_t* const a0 = wsrc - r;
        const uint32_t nw = (N + r + 15) >> 4;
        // (with the RLE test: every block byte, LDS bytes [r + hist, r + N), equal to the first)
        const uint32_t b0 = data[(c0 - base) + off];
        const uint32_t bb = b0 * 0x01010101u, blo = r + hist, bhi = r + N;
        auto same_dw = [&](uint32_t a, uint32_t val) {  // the dword at LDS byte a
            if (a + 4 <= blo || a >= bhi) return true;
            uint32_t mk = 0xFFFFFFFFu;
            if (a < blo) mk &= 0xFFFFFFFFu << (8 * (blo - a));
            if (a + 4 > bhi) mk &= 0xFFFFFFFFu >> (8 * (a + 4 - bhi));
            return ((val ^ bb) & mk) == 0;
        };
        bool same = true;
        for (uint32_t i0 = tid; i0 < nw; i0 += 4 * kZThreads) {
            v4u v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = i0 + kZThreads * q;
                if (i < nw) v[q] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a0) + i);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = i0 + kZThreads * q;
                if (i < nw) {
                    stage[i] = make_uint4(v[q].x, v[q].y, v[q].z, v[q].w);
                    same = same && same_dw(16 * i, v[q].x) && same_dw(16 * i + 4, v[q].y) &&
                           same_dw(16 * i + 8, v[q].z) && same_dw(16 * i + 12, v[q].w);
                }
            }
        }
        if (tid < 2) stage[nw + tid] = make_uint4(0, 0, 0, 0);  // word reads past the end stay defined
        // ---- RLE block: every byte equal
        if (__syncthreads_and(same)) {
            ZMARK(0);
            if (tid == 0) {
                write_block_header(out, last, 1, n);
                out[3] = (uint8_t)b0;
                sizes[k] = 4;
            }
            continue;
        }
        ZMARK(0);
        const Win W{(const lds_u32*)stage, r};

        // ---- parse: wave w owns the sub-block [s0, se) (window positions)
        {
            const uint64_t tw0 = probe_on && blockIdx.x == 0 ? wall_clock64() : 0;
            const uint64_t pr = parse_subblock(W, (lds_u16*)tabs, wseq_all, hist, N, wave, lane,
                                               probe_on && blockIdx.x == 0 && wave == 0 ? g_zprobe : nullptr);
            const uint32_t ns = (uint32_t)pr, lastend = (uint32_t)(pr >> 32);
            if (probe_on && blockIdx.x == 0 && lane == 0) atomicAdd(&g_zprobe[34 + wave], wall_clock64() - tw0);
            if (lane == 0) {
                ctl.nseq[wave] = ns;
                ctl.lastend[wave] = lastend;
            }
            __threadfence_block();  // the sequence list (global) before the other waves read it (workgroup scope: an agent-scope fence writes back L2)
        }
        __syncthreads();
        ZMARK(1);
        if ((int64_t)k == dbg_item) {
            for (uint32_t i = tid; i < kZWaves * (1 + 3 * kZSubSeq); i += kZThreads) {
                const uint32_t w2 = i / (1 + 3 * kZSubSeq), r2 = i % (1 + 3 * kZSubSeq);
                g_zdbg[i] = r2 == 0 ? ctl.nseq[w2]
                                    : reinterpret_cast<const uint32_t*>(wseq_all + (uint64_t)w2 * kZSubSeq)[r2 - 1];
            }
        }

        // ---- literals: bitmap of the unmatched bytes, literal index per thread range
        for (uint32_t i = tid; i < kEncBlock / 32; i += kZThreads) {
            const uint32_t b = 32 * i;
            E.bitmap[i] = b + 32 <= n ? 0xFFFFFFFFu : (b >= n ? 0u : (0xFFFFFFFFu >> (32 - (n - b))));
        }
        for (uint32_t i = tid; i < kZWaves * 256; i += kZThreads) E.streams[i] = 0;  // per-wave histograms
        __syncthreads();
        {
            // lane per match: its partial end words by atomics, up to 4 whole words by
            // stores (no other match touches them); longer runs of whole words by the wave
            const Seq* const wseq = wseq_all + (uint64_t)wave * kZSubSeq;
            const uint32_t nsw = min(ctl.nseq[wave], kZSubSeq);
            for (uint32_t q0 = 0; q0 < nsw; q0 += 64) {
                uint32_t a = 0, b = 0;
                if (q0 + lane < nsw) {
                    const Seq e = wseq[q0 + lane];
                    a = e.pos;
                    b = e.pos + e.ml;
                }
                uint32_t wa = 0, wb = 0;
                if (a < b) {
                    if ((a >> 5) == ((b - 1) >> 5)) {
                        const uint32_t cnt = b - a;
                        const uint32_t mask = (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << (a & 31);
                        if (cnt == 32)
                            E.bitmap[a >> 5] = 0;
                        else
                            atomicAnd(&E.bitmap[a >> 5], ~mask);
                    } else {
                        if (a & 31) atomicAnd(&E.bitmap[a >> 5], (1u << (a & 31)) - 1u);
                        if (b & 31) atomicAnd(&E.bitmap[b >> 5], ~((1u << (b & 31)) - 1u));
                        wa = (a + 31) >> 5;
                        wb = b >> 5;
                        if (wb - wa <= 4) {
                            for (uint32_t w = wa; w < wb; ++w) E.bitmap[w] = 0;
                            wb = wa;
                        }
                    }
                }
                for (unsigned long long lg = __ballot(wb > wa); lg; lg &= lg - 1) {
                    const int l = __builtin_ctzll(lg);
                    const uint32_t la = (uint32_t)__builtin_amdgcn_readlane((int)wa, l);
                    const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane((int)wb, l);
                    for (uint32_t w = la + lane; w < lb; w += 64) E.bitmap[w] = 0;
                }
            }
        }
        __syncthreads();
        ZMARK(15);
        // thread t owns block positions [128 t, 128 t + 128): bitmap words 4t .. 4t + 3
        uint32_t bmw[4], cnt_t = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bmw[i] = E.bitmap[4 * tid + i];
            cnt_t += __builtin_popcount(bmw[i]);
        }
        // the sampled histogram first: literals at block positions divisible by 16 (one
        // predicated LDS atomic per 16 positions); the full one only when the sample says
        // Huffman may pay (random literals never need it)
        uint32_t* const wh = E.streams + wave * 256;
        uint32_t samp_t = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if ((bmw[k >> 1] >> ((16 * k) & 31)) & 1u) {
                atomicAdd(&wh[W.byte(hist + 128 * tid + 16 * k)], 1u);
                ++samp_t;
            }
        }
        const uint32_t incl = wave_incl(cnt_t, lane);
        const uint32_t sincl = wave_incl(samp_t, lane);
        if (lane == 63) {
            ctl.wsum[wave] = incl;
            ctl.wsum2[wave] = sincl;
        }
        __syncthreads();
        uint32_t litbase = incl - cnt_t, nlit = 0, nsamp = 0;
        for (int w2 = 0; w2 < kZWaves; ++w2) {
            litbase += w2 < wave ? ctl.wsum[w2] : 0u;
            nlit += ctl.wsum[w2];
            nsamp += ctl.wsum2[w2];
        }
        if (tid < 256) {
            uint32_t c = 0;
            for (int w2 = 0; w2 < kZWaves; ++w2) c += E.streams[w2 * 256 + tid];
            E.hist[tid] = c;
        }
        __syncthreads();
        ZMARK(16);
        if (wave == 0) {  // 1: the full histogram is needed; 0: raw literals
            uint32_t need = nlit > 0;
            if (nlit >= 32 && nsamp > 0) {
                uint64_t es = 0;
                const uint32_t lm = lg256(nsamp);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t c = E.hist[lane + 64 * i];
                    if (c) es += (uint64_t)c * (lm - lg256(c));
                }
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) es += __shfl_xor(es, d, 64);
                if (es * nlit / nsamp / 2048 + 64 >= (uint64_t)nlit - nlit / 64) need = 0;
            }
            if (lane == 0) {
                ctl.need_full = need;
                ctl.lit_mode = 0;
            }
        }
        __syncthreads();
        if (ctl.need_full) {
            for (uint32_t i = tid; i < kZWaves * 256; i += kZThreads) E.streams[i] = 0;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; ++i)
                for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1)
                    atomicAdd(&wh[W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2))], 1u);
            __syncthreads();
            if (tid < 256) {
                uint32_t c = 0;
                for (int w2 = 0; w2 < kZWaves; ++w2) c += E.streams[w2 * 256 + tid];
                E.hist[tid] = c;
            }
            __syncthreads();
        }
        ZMARK(2);

        // ---- repeat-offset coding (every wave its sub-block), then two independent halves at
        // once: the literal mode (Huffman code, wave 0) and the sequence side -- per stream (LL
        // on wave 1, OF on 2, ML on 3) its code histogram, its table and its FSE state chain.
        // (Round 3 ran them one after the other: the chains waited for the literal mode and the
        // literal section for the chains -- ~80 us of a ~1.25 ms text block.)
        const bool role_probe = probe_on && blockIdx.x == 0;
        uint64_t zt = role_probe ? wall_clock64() : 0;
        auto role_end = [&](int idx) {
            if (role_probe && lane == 0) {
                const uint64_t t2 = wall_clock64();
                atomicAdd(&g_zprobe[idx], t2 - zt);
                zt = t2;
            }
        };
        rep_code_wave(ctl.nseq, ctl.lastend, wseq_all, coded, (uint32_t)wave, lane);
        __threadfence_block();
        {
            // this sub-block's code histograms (LL | ML | OF, 121 bins) into the wave's own copy
            // in the stream buffer (free until the literal section); the stream's wave sums them
            uint32_t* const wc = E.streams + wave * 128;
            for (uint32_t i = (uint32_t)lane; i < 128; i += 64) wc[i] = 0;
            __builtin_amdgcn_wave_barrier();
            uint32_t first = 0;
            for (int w2 = 0; w2 < wave; ++w2) first += min(ctl.nseq[w2], kZSubSeq);
            const uint32_t cnt = min(ctl.nseq[wave], kZSubSeq);
            for (uint32_t q0 = 0; q0 < cnt; q0 += 64 * 4) {
                uint32_t cv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t q = q0 + 64 * (uint32_t)u + (uint32_t)lane;
                    cv[u] = q < cnt ? coded[first + q].codes : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (cv[u] != 0xFFFFFFFFu) {
                        atomicAdd(&wc[cv[u] & 0xFF], 1u);
                        atomicAdd(&wc[36 + ((cv[u] >> 8) & 0xFF)], 1u);
                        atomicAdd(&wc[36 + 53 + (cv[u] >> 16)], 1u);
                    }
            }
        }
        if (wave == 1) role_end(18);
        __syncthreads();
        ZMARK(3);
        uint32_t nseq = 0;
        for (int w2 = 0; w2 < kZWaves; ++w2) nseq += min(ctl.nseq[w2], kZSubSeq);
        if (wave == 0) {
            if (ctl.need_full) literal_mode_wave(E, ctl, fse_huf, nlit, lane, role_probe ? g_zprobe : nullptr);
            role_end(17);
        } else if (wave <= 3) {
            const int k = wave - 1;  // 0 LL, 1 OF, 2 ML
            const uint32_t sh = k == 0 ? 0u : k == 1 ? 16u : 8u;
            uint32_t* const hk = E.shist + (k == 0 ? 0 : k == 1 ? 36 + 53 : 36);  // (the histogram layout: LL, ML, OF)
            const uint32_t nbin = k == 0 ? 36u : k == 1 ? 32u : 53u;
            const uint32_t boff = k == 0 ? 0u : k == 1 ? 36u + 53u : 36u;
            uint32_t tot = 0;
#pragma unroll
            for (int w2 = 0; w2 < kZWaves; ++w2) tot += (uint32_t)lane < nbin ? E.streams[w2 * 128 + boff + lane] : 0u;
            if ((uint32_t)lane < nbin) hk[lane] = tot;
            __builtin_amdgcn_wave_barrier();
            if (nseq > 0) {
                if (k == 0) seq_table_wave(fse[0], hk, 36, nseq, kLLNorm, kLLLog, kLLMaxLog, lane);
                if (k == 1) seq_table_wave(fse[1], hk, 29, nseq, kOFNorm, kOFLog, kOFMaxLog, lane);
                if (k == 2) seq_table_wave(fse[2], hk, 53, nseq, kMLNorm, kMLLog, kMLMaxLog, lane);
            }
            if (wave == 1) role_end(19);
            if (nseq >= 2 && fse[k].mode != 1) {
                const FseView tv = fse[k].mode == 2 ? view(fse[k]) : view(pre[k]);
                seq_chain_wave(tv, coded, nseq, sh, chains + (uint64_t)k * kZBlockSeq,
                               reinterpret_cast<uint16_t*>(chains + 3ull * kZBlockSeq) + (uint64_t)k * kZBlockSeq,
                               reinterpret_cast<uint8_t*>(chains + 3ull * kZBlockSeq + 3ull * kZBlockSeq / 2) +
                                   (uint64_t)k * (kZBlockSeq + 16),
                               &ctl.seq_last[k], lane, role_probe && k == 0 ? g_zprobe : nullptr);
                __threadfence_block();
            }
            if (wave == 1) role_end(20);
        }
        __syncthreads();
        ZMARK(5);
        // literal runs (few sequences: the raw literals are copied run by run, coalesced)
        if (wave == 0 && nseq < kZRuns) {
            const Coded x = (uint32_t)lane < nseq ? coded[lane] : Coded{0, 0, 0, 0};
            const uint32_t span = x.ll + x.ml, lit = x.ll;
            const uint32_t si = wave_incl(span, lane), li = wave_incl(lit, lane);
            if ((uint32_t)lane <= nseq) {
                ctl.run_start[lane] = si - span;
                ctl.run_out[lane] = li - lit;
                ctl.run_len[lane] = (uint32_t)lane < nseq ? lit : (n > si - span ? n - (si - span) : 0u);  // (never a wrapped length)
            }
        }
        // ---- Huffman sizes: per-thread code-length sums, block scan, segment totals
        const uint32_t lit_mode = ctl.lit_mode;
        uint32_t bits_t = 0;
        if (lit_mode == 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1)
                    bits_t += E.len[W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2))];
        }
        const uint32_t bincl = wave_incl(bits_t, lane);
        if (lane == 63) ctl.wsum2[wave] = bincl;
        const bool four = nlit >= 256;
        const uint32_t seg = four ? (nlit + 3) / 4 : nlit;
        __syncthreads();
        ZMARK(4);
        uint32_t bbase = bincl - bits_t;
        for (int w2 = 0; w2 < wave; ++w2) bbase += ctl.wsum2[w2];
        if (lit_mode == 2) {
            // the thread holding literal index seg * s records the bits before it
            if (tid == 0) {
                ctl.segP[0] = 0;
                uint32_t tot = 0;
                for (int w2 = 0; w2 < kZWaves; ++w2) tot += ctl.wsum2[w2];
                ctl.segP[4] = tot;
                if (!four) ctl.segP[1] = tot;
            }
            if (four) {
                uint32_t idx = litbase, pb = bbase;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1) {
                        if (idx == seg || idx == 2 * seg || idx == 3 * seg) ctl.segP[idx / seg] = pb;
                        pb += E.len[W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2))];
                        ++idx;
                    }
            }
        }
        __syncthreads();
        // literal section: size decision (thread 0)
        if (tid == 0) {
            uint32_t lm = lit_mode, sz = 0;
            const uint32_t rawh = nlit < 32 ? 1u : nlit < 4096 ? 2u : 3u;
            if (lm == 2) {
                uint32_t sb = 0;
                const int ns4 = four ? 4 : 1;
                for (int s = 0; s < ns4; ++s) sb += (ctl.segP[four ? s + 1 : 4] - ctl.segP[s] + 8) / 8;
                const uint32_t c = ctl.desc_len + (four ? 6u : 0u) + sb;
                const uint32_t mx = max(nlit, c);
                const uint32_t hs = mx < 1024 ? 3u : mx < 16384 ? 4u : 5u;
                if (sb > kHufStreams || hs + c >= rawh + nlit) {
                    lm = 0;
                } else {
                    sz = hs + c;
                    ctl.huf_c = c;   // the header's compressed size
                    ctl.huf_hs = hs; // header bytes
                }
            }
            if (lm == 0) sz = rawh + nlit;
            if (lm == 1) sz = rawh + 1;
            ctl.lit_mode = lm;
            ctl.lit_size = sz;
        }
        __syncthreads();
        ZMARK(6);
        const uint32_t lm = ctl.lit_mode, lsz = ctl.lit_size;
        uint8_t* const lit_out = out + 3;
        if (probe) {
            g_zprobe[10] += 1;
            g_zprobe[11] += nseq;
            g_zprobe[12] += nlit;
        }
        // ---- the sequence section header (count, modes, table descriptions; thread 0)
        if (wave == 0 && role_probe) zt = wall_clock64();
        if (tid == 0) {
            uint8_t* o = lit_out + lsz;
            uint8_t* const o0 = o;
            const uint32_t ns = nseq;
            if (ns < 128) {
                *o++ = (uint8_t)ns;
            } else if (ns < 0x7F00) {
                *o++ = (uint8_t)((ns >> 8) + 0x80);
                *o++ = (uint8_t)ns;
            } else {
                *o++ = 0xFF;
                *o++ = (uint8_t)(ns - 0x7F00);
                *o++ = (uint8_t)((ns - 0x7F00) >> 8);
            }
            if (ns) {
                *o++ = (uint8_t)(fse[0].mode << 6 | fse[1].mode << 4 | fse[2].mode << 2);
                for (int k = 0; k < 3; ++k)
                    for (uint32_t i = 0; i < fse[k].desc_len; ++i) *o++ = fse[k].desc[i];
            }
            ctl.seq_hdr = (uint32_t)(o - o0);
            if (ns >= 1)  // a single sequence's states come from its own codes
                for (int k = 0; k < 3; ++k)
                    if (fse[k].mode != 1 && ns == 1) {
                        const uint32_t sh = k == 0 ? 0u : k == 1 ? 16u : 8u;
                        const FseView tv = fse[k].mode == 2 ? view(fse[k]) : view(pre[k]);
                        ctl.seq_last[k] = fse_init(tv, (coded[0].codes >> sh) & 0xFF);
                    }
        }
        // ---- the literal section
        write_literals(E, ctl, W, hist, make_uint4(bmw[0], bmw[1], bmw[2], bmw[3]), litbase, bbase, nlit, lm, four, seg,
                       lit_out, tid, nseq < kZRuns ? nseq + 1 : 0u);
        if (wave == 0) role_end(21);
        // ---- sequences bit stream: per-sequence bit counts, a block scan, then every
        // thread writes its range of sequences (the last sequence first in the stream) with
        // atomicOr into the zeroed words
        __syncthreads();
        ZMARK(7);
        {
            const uint32_t ns = nseq, hdr = ctl.seq_hdr;
            const uint32_t mode[3] = {fse[0].mode, fse[1].mode, fse[2].mode};
            const uint32_t per = (ns + kZThreads - 1) / kZThreads;
            const uint32_t q0 = min(ns, (uint32_t)tid * per), q1 = min(ns, q0 + per);
            uint32_t st = 0;
            for (uint32_t q = q0; q < q1; ++q) st += seq_bits(coded[q], q, ns, chains, kZBlockSeq, mode);
            const uint32_t si = wave_incl(st, lane);
            if (lane == 63) ctl.wsum[wave] = si;
            __syncthreads();
            uint32_t pt = si - st, T = 0;
            for (int w2 = 0; w2 < kZWaves; ++w2) {
                pt += w2 < wave ? ctl.wsum[w2] : 0u;
                T += ctl.wsum[w2];
            }
            uint32_t flushb = 0;
            for (int k = 0; k < 3; ++k)
                if (ns && mode[k] != 1) flushb += (uint32_t)(mode[k] == 2 ? fse[k].log : pre[k].log);
            const uint32_t sbytes = ns ? (T + flushb + 1 + 7) / 8 : 0u;
            const uint32_t body = lsz + hdr + sbytes;
            const bool ok = body < n;
            const uint32_t lastw_l = ns ? (8u * (uint32_t)((uintptr_t)(lit_out + lsz + hdr) & 3u) + T + flushb) >> 5 : 0u;
            if (ok && ns && lastw_l + 1 <= (uint32_t)(sizeof(E.streams) / 4)) {
                // staged in LDS (the Huffman streams' buffer, free since the literal section was
                // written), then stored as whole words; word 0 keeps the bytes before S0
                uint8_t* const S0 = lit_out + lsz + hdr;
                uint32_t* const A = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(S0) & ~(uintptr_t)3);
                const uint32_t off0 = 8u * (uint32_t)(S0 - reinterpret_cast<uint8_t*>(A));
                const uint32_t lastw = lastw_l;
                uint32_t* const L = E.streams;
                for (uint32_t wdx = tid; wdx <= lastw; wdx += kZThreads) L[wdx] = 0;
                __syncthreads();
                OrBitsL ob;
                ob.init(L, off0 + (T - pt - st));
                for (uint32_t q = q1; q-- > q0;) {
                    const Coded x = coded[q];
                    const uint32_t llc = x.codes & 0xFF, mlc = (x.codes >> 8) & 0xFF, ofc = x.codes >> 16;
                    if (q + 1 < ns) {
                        const uint32_t j = ns - 2 - q;  // (step order)
                        if (mode[1] != 1) {
                            const uint32_t c = chains[kZBlockSeq + j];
                            ob.put(c & 0xFFFF, c >> 16);
                        }
                        if (mode[2] != 1) {
                            const uint32_t c = chains[2 * kZBlockSeq + j];
                            ob.put(c & 0xFFFF, c >> 16);
                        }
                        if (mode[0] != 1) {
                            const uint32_t c = chains[j];
                            ob.put(c & 0xFFFF, c >> 16);
                        }
                    }
                    ob.put(x.ll - ll_base(llc), ll_bits(llc));
                    ob.put(x.ml - ml_base(mlc), ml_bits(mlc));
                    ob.put(x.ofv - (1u << ofc), ofc);
                }
                ob.done();
                if (tid == kZThreads - 1) {  // the final states (ML, OF, LL) and the end mark
                    OrBitsL fb;
                    fb.init(L, off0 + T);
                    if (mode[2] != 1) fb.put(ctl.seq_last[2], (uint32_t)(mode[2] == 2 ? fse[2].log : pre[2].log));
                    if (mode[1] != 1) fb.put(ctl.seq_last[1], (uint32_t)(mode[1] == 2 ? fse[1].log : pre[1].log));
                    if (mode[0] != 1) fb.put(ctl.seq_last[0], (uint32_t)(mode[0] == 2 ? fse[0].log : pre[0].log));
                    fb.put(1, 1);
                    fb.done();
                }
                __syncthreads();
                for (uint32_t wdx = tid; wdx <= lastw; wdx += kZThreads)
                    A[wdx] = wdx ? L[wdx] : (off0 ? A[0] & ((1u << off0) - 1u) : 0u) | L[0];
            } else if (ok && ns) {
                uint8_t* const S0 = lit_out + lsz + hdr;
                uint32_t* const A = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(S0) & ~(uintptr_t)3);
                const uint32_t off0 = 8u * (uint32_t)(S0 - reinterpret_cast<uint8_t*>(A));
                const uint32_t lastw = (off0 + T + flushb + 1 - 1) >> 5;
                if (tid == 0)
                    for (uint8_t* b = S0; b < reinterpret_cast<uint8_t*>(A + 1); ++b) *b = 0;
                for (uint32_t wdx = 1 + tid; wdx <= lastw; wdx += kZThreads) A[wdx] = 0;
                __threadfence_block();  // the zeros (and the section header) stored before any atomicOr
                __syncthreads();
                OrBits ob;
                ob.init(A, off0 + (T - pt - st));
                for (uint32_t q = q1; q-- > q0;) {
                    const Coded x = coded[q];
                    const uint32_t llc = x.codes & 0xFF, mlc = (x.codes >> 8) & 0xFF, ofc = x.codes >> 16;
                    if (q + 1 < ns) {
                        const uint32_t j = ns - 2 - q;  // (step order)
                        if (mode[1] != 1) {
                            const uint32_t c = chains[kZBlockSeq + j];
                            ob.put(c & 0xFFFF, c >> 16);
                        }
                        if (mode[2] != 1) {
                            const uint32_t c = chains[2 * kZBlockSeq + j];
                            ob.put(c & 0xFFFF, c >> 16);
                        }
                        if (mode[0] != 1) {
                            const uint32_t c = chains[j];
                            ob.put(c & 0xFFFF, c >> 16);
                        }
                    }
                    ob.put(x.ll - ll_base(llc), ll_bits(llc));
                    ob.put(x.ml - ml_base(mlc), ml_bits(mlc));
                    ob.put(x.ofv - (1u << ofc), ofc);
                }
                ob.done();
                if (tid == kZThreads - 1) {  // the final states (ML, OF, LL) and the end mark
                    OrBits fb;
                    fb.init(A, off0 + T);
                    if (mode[2] != 1) fb.put(ctl.seq_last[2], (uint32_t)(mode[2] == 2 ? fse[2].log : pre[2].log));
                    if (mode[1] != 1) fb.put(ctl.seq_last[1], (uint32_t)(mode[1] == 2 ? fse[1].log : pre[1].log));
                    if (mode[0] != 1) fb.put(ctl.seq_last[0], (uint32_t)(mode[0] == 2 ? fse[0].log : pre[0].log));
                    fb.put(1, 1);
                    fb.done();
                }
            }
            if (tid == 0) {
                ctl.seq_ok = ok;
                ctl.seq_size = body;
            }
        }
        __syncthreads();
        ZMARK(8);
        if (!ctl.seq_ok) {  // raw block (dword stores: byte stores cost a 64 KiB block 128 rounds)
            stage_to_global(out + 3, W, hist, n, (uint32_t)tid, kZThreads);
            if (tid == 0) {
                write_block_header(out, last, 0, n);
                sizes[k] = 3 + (uint64_t)n;
            }
        } else if (tid == 0) {
            write_block_header(out, last, 2, ctl.seq_size);
            sizes[k] = 3 + (uint64_t)ctl.seq_size;
        }
    }
}

// ---------------------------------------------------------------- split form (round 6)
// The same blocks in two kernels, byte for byte: zstd_parse_kernel (one 512-thread workgroup
// per CU: stage, RLE test, parse, then per sub-block the repeat coding and code histograms,
// the literal bitmap, the literal histogram and the literals compacted to global memory) and
// zstd_entropy_kernel (256-thread workgroups, three per CU: literal mode on wave 0 beside the
// LL / OF / ML tables and state chains on waves 1-3, then the literal section and the
// sequence bit stream from the compacted literals and the coded sequences).  In the fused
// kernel the entropy half ran on 4 of the block's 8 waves while the others waited at a
// barrier and no other block could use the CU's LDS; here a CU runs three blocks' entropy
// halves at once (52 KiB of LDS, 168 VGPRs each) and the parse kernel's waves never wait for one.
// The batch of items between the two kernels lives in global memory (ZItem, the coded
// sequences, the literals).
constexpr int kEThreads = 256;
constexpr int kEWaves = kEThreads / 64;
struct ZItem {
    uint32_t kind;  // 0: the entropy kernel encodes the block; 1: complete (empty or RLE)
    uint32_t nlit, need_full, pad;
    uint32_t nseq[kZWaves];
    uint32_t shist[36 + 53 + 32];  // LL | ML | OF code histograms
    uint32_t pad2[3];
    uint32_t hist[256];  // literal histogram (need_full)
};
// the parse kernel's work area after the parse (the tables are dead then)
struct PArea {
    uint32_t bitmap[kEncBlock / 32];
    uint32_t wh[kZWaves * 256];  // per-wave literal histograms
    uint32_t wc[kZWaves * 128];  // per-wave code histograms (LL | ML | OF)
    uint32_t hist[256];
    uint8_t lit[32 * 1024];  // literals compacted in pieces, then copied out
};
static_assert(sizeof(PArea) <= 64 * 1024, "the parse kernel's buffers fit the work area");
struct PCtl {
    uint32_t nseq[kZWaves], lastend[kZWaves], wsum[kZWaves], wsum2[kZWaves], need_full;
    uint32_t run_start[kZRuns], run_len[kZRuns], run_out[kZRuns];  // literal runs of a block with few sequences
};
// the entropy kernel's area: the fused kernel's EntropyArea without the literal bitmap (the
// parse kernel's) and with a 36.5 KiB stream buffer -- Huffman streams up to kHufStreams
// (48 KiB) longer than it are ORed into the output in global memory instead (same bytes),
// and so is a sequence bit stream longer than it; with it three workgroups fit a CU's LDS
constexpr uint32_t kEStreams = 36 * 1024 + 512;  // (3 x the LDS of a workgroup must stay under 160 KiB after the allocation granule)
struct EArea {
    // the Huffman merge's scratch (keys, tw, par: literal_mode_wave only) shares the stream
    // buffer, which is free until the literal section
    union {
        uint32_t streams[kEStreams / 4 + 4];
        struct {
            uint32_t keys[256];
            uint32_t tw[512];
            uint16_t par[512];
        };
    };
    uint32_t hist[256];
    uint8_t lens[256];
    uint8_t len[256];
    uint16_t code[256];
    uint32_t shist[36 + 53 + 32];
};

// The split kernels' item dealing.  deal == nullptr: static, item k, k + grid, ... (the
// stride passed in); otherwise the next unclaimed item of the launch's counter (zeroed
// before the launch), so a workgroup that drew cheap items (RLE zero pages, raw blocks the
// entropy kernel skips) takes more: the VM image's blocks are that uneven.  Every thread
// of the workgroup calls it (it has two barriers).
__device__ __forceinline__ uint64_t deal_item(uint32_t* deal, uint32_t& s_next, uint64_t stride_next) {
    if (!deal) return stride_next;
    __syncthreads();
    if (threadIdx.x == 0) s_next = atomicAdd(deal, 1u);
    __syncthreads();
    return s_next;
}

__global__ __launch_bounds__(kZThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void zstd_parse_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint64_t* __restrict__ items, uint64_t nitems, uint64_t item_base, uint8_t* __restrict__ slots,
    uint64_t* __restrict__ sizes, Seq* __restrict__ seq_scratch, Coded* __restrict__ coded_items,
    uint8_t* __restrict__ lit_items, ZItem* __restrict__ zitems, uint32_t* __restrict__ deal,
    uint32_t* __restrict__ elist, int probe_on, int64_t dbg_item) {
    __shared__ uint4 stage[kZStageWords];
    __shared__ __attribute__((aligned(16))) uint8_t work[64 * 1024];
    __shared__ PCtl pc;
    __shared__ uint32_t s_next;
    const int tid = threadIdx.x, lane = tid & 63, wave = (int)uni((uint32_t)tid >> 6);
    const bool probe = probe_on && blockIdx.x == 0 && tid == 0;
    uint64_t tp = probe ? wall_clock64() : 0;
    uint16_t* const tabs = reinterpret_cast<uint16_t*>(work);
    PArea& A = *reinterpret_cast<PArea*>(work);
    Seq* const wseq_all = seq_scratch + (uint64_t)blockIdx.x * kZBlockSeq;
    for (uint64_t k = deal_item(deal, s_next, blockIdx.x); k < nitems; k = deal_item(deal, s_next, k + gridDim.x)) {
        __syncthreads();  // LDS of the previous item
        ZMARK(9);
        ZItem* const zi = zitems + k;
        const uint64_t it = items[k];
        const uint64_t ci = it >> 32, j = (uint32_t)it;
        const uint64_t c0 = bounds[2 * ci], c1 = bounds[2 * ci + 1];
        const uint64_t len = c1 - c0, off = j * (uint64_t)kEncBlock;
        const uint32_t n = (uint32_t)(len > off ? (len - off < kEncBlock ? len - off : kEncBlock) : 0);
        const bool last = off + n == len;
        uint8_t* const out = slots + k * kSlot;
        if (n == 0) {  // the empty chunk's frame: one empty raw block
            if (tid == 0) {
                write_block_header(out, true, 0, 0);
                sizes[k] = 3;
                zi->kind = 1;
            }
            continue;
        }
        const uint32_t hist = (uint32_t)(off < kZHist ? off : kZHist);
        const uint32_t N = hist + n;
        const uint8_t* const wsrc = data + (c0 - base) + off - hist;
        const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(wsrc) & 15);
        const uint8_t* const a0 = wsrc - r;
        const uint32_t nw = (N + r + 15) >> 4;
        const uint32_t b0 = data[(c0 - base) + off];
        const uint32_t bb = b0 * 0x01010101u, blo = r + hist, bhi = r + N;
        auto same_dw = [&](uint32_t a, uint32_t val) {
            if (a + 4 <= blo || a >= bhi) return true;
            uint32_t mk = 0xFFFFFFFFu;
            if (a < blo) mk &= 0xFFFFFFFFu << (8 * (blo - a));
            if (a + 4 > bhi) mk &= 0xFFFFFFFFu >> (8 * (a + 4 - bhi));
            return ((val ^ bb) & mk) == 0;
        };
        bool same = true;
        for (uint32_t i0 = tid; i0 < nw; i0 += 4 * kZThreads) {
            v4u v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = i0 + kZThreads * q;
                if (i < nw) v[q] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a0) + i);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = i0 + kZThreads * q;
                if (i < nw) {
                    stage[i] = make_uint4(v[q].x, v[q].y, v[q].z, v[q].w);
                    same = same && same_dw(16 * i, v[q].x) && same_dw(16 * i + 4, v[q].y) &&
                           same_dw(16 * i + 8, v[q].z) && same_dw(16 * i + 12, v[q].w);
                }
            }
        }
        if (tid < 2) stage[nw + tid] = make_uint4(0, 0, 0, 0);
        if (__syncthreads_and(same)) {  // RLE block: every byte equal
            ZMARK(0);
            if (tid == 0) {
                write_block_header(out, last, 1, n);
                out[3] = (uint8_t)b0;
                sizes[k] = 4;
                zi->kind = 1;
            }
            continue;
        }
        ZMARK(0);
        const Win W{(const lds_u32*)stage, r};
        {
            const uint64_t tw0 = probe_on && blockIdx.x == 0 ? wall_clock64() : 0;
            const uint64_t pr = parse_subblock(W, (lds_u16*)tabs, wseq_all, hist, N, wave, lane,
                                               probe_on && blockIdx.x == 0 && wave == 0 ? g_zprobe : nullptr);
            if (probe_on && blockIdx.x == 0 && lane == 0) atomicAdd(&g_zprobe[34 + wave], wall_clock64() - tw0);
            if (lane == 0) {
                pc.nseq[wave] = (uint32_t)pr;
                pc.lastend[wave] = (uint32_t)(pr >> 32);
            }
            __threadfence_block();  // the sequence list (global) before the other waves read it
        }
        __syncthreads();
        ZMARK(1);
        if ((int64_t)(k + item_base) == dbg_item) {
            for (uint32_t i = tid; i < kZWaves * (1 + 3 * kZSubSeq); i += kZThreads) {
                const uint32_t w2 = i / (1 + 3 * kZSubSeq), r2 = i % (1 + 3 * kZSubSeq);
                g_zdbg[i] = r2 == 0 ? pc.nseq[w2]
                                    : reinterpret_cast<const uint32_t*>(wseq_all + (uint64_t)w2 * kZSubSeq)[r2 - 1];
            }
        }
        // ---- per sub-block (its wave): the matches out of the literal bitmap, the repeat
        // coding, the code histogram
        for (uint32_t i = tid; i < kEncBlock / 32; i += kZThreads) {
            const uint32_t b = 32 * i;
            A.bitmap[i] = b + 32 <= n ? 0xFFFFFFFFu : (b >= n ? 0u : (0xFFFFFFFFu >> (32 - (n - b))));
        }
        for (uint32_t i = tid; i < kZWaves * 256; i += kZThreads) A.wh[i] = 0;
        for (uint32_t i = tid; i < kZWaves * 128; i += kZThreads) A.wc[i] = 0;
        __syncthreads();
        Coded* const coded = coded_items + k * (uint64_t)kZBlockSeq;
        {
            const Seq* const wseq = wseq_all + (uint64_t)wave * kZSubSeq;
            const uint32_t nsw = min(pc.nseq[wave], kZSubSeq);
            for (uint32_t q0 = 0; q0 < nsw; q0 += 64) {
                uint32_t a = 0, b = 0;
                if (q0 + lane < nsw) {
                    const Seq e = wseq[q0 + lane];
                    a = e.pos;
                    b = e.pos + e.ml;
                }
                uint32_t wa = 0, wb = 0;
                if (a < b) {
                    if ((a >> 5) == ((b - 1) >> 5)) {
                        const uint32_t cnt = b - a;
                        const uint32_t mask = (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << (a & 31);
                        if (cnt == 32)
                            A.bitmap[a >> 5] = 0;
                        else
                            atomicAnd(&A.bitmap[a >> 5], ~mask);
                    } else {
                        if (a & 31) atomicAnd(&A.bitmap[a >> 5], (1u << (a & 31)) - 1u);
                        if (b & 31) atomicAnd(&A.bitmap[b >> 5], ~((1u << (b & 31)) - 1u));
                        wa = (a + 31) >> 5;
                        wb = b >> 5;
                        if (wb - wa <= 4) {
                            for (uint32_t w = wa; w < wb; ++w) A.bitmap[w] = 0;
                            wb = wa;
                        }
                    }
                }
                for (unsigned long long lg = __ballot(wb > wa); lg; lg &= lg - 1) {
                    const int l = __builtin_ctzll(lg);
                    const uint32_t la = (uint32_t)__builtin_amdgcn_readlane((int)wa, l);
                    const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane((int)wb, l);
                    for (uint32_t w = la + lane; w < lb; w += 64) A.bitmap[w] = 0;
                }
            }
        }
        rep_code_wave(pc.nseq, pc.lastend, wseq_all, coded, (uint32_t)wave, lane);
        __threadfence_block();
        {
            uint32_t* const wc = A.wc + wave * 128;
            uint32_t first = 0;
            for (int w2 = 0; w2 < wave; ++w2) first += min(pc.nseq[w2], kZSubSeq);
            const uint32_t cnt = min(pc.nseq[wave], kZSubSeq);
            for (uint32_t q0 = 0; q0 < cnt; q0 += 64 * 4) {
                uint32_t cv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t q = q0 + 64 * (uint32_t)u + (uint32_t)lane;
                    cv[u] = q < cnt ? coded[first + q].codes : 0xFFFFFFFFu;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (cv[u] != 0xFFFFFFFFu) {
                        atomicAdd(&wc[cv[u] & 0xFF], 1u);
                        atomicAdd(&wc[36 + ((cv[u] >> 8) & 0xFF)], 1u);
                        atomicAdd(&wc[36 + 53 + (cv[u] >> 16)], 1u);
                    }
            }
        }
        __syncthreads();
        ZMARK(3);
        // ---- literals: per thread (block positions [128 t, 128 t + 128)) its count and the
        // sampled histogram; the full histogram only when the sample says Huffman may pay
        uint32_t bmw[4], cnt_t = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bmw[i] = A.bitmap[4 * tid + i];
            cnt_t += __builtin_popcount(bmw[i]);
        }
        uint32_t* const wh = A.wh + wave * 256;
        uint32_t samp_t = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if ((bmw[q >> 1] >> ((16 * q) & 31)) & 1u) {
                atomicAdd(&wh[W.byte(hist + 128 * tid + 16 * q)], 1u);
                ++samp_t;
            }
        }
        const uint32_t incl = wave_incl(cnt_t, lane);
        const uint32_t sincl = wave_incl(samp_t, lane);
        if (lane == 63) {
            pc.wsum[wave] = incl;
            pc.wsum2[wave] = sincl;
        }
        __syncthreads();
        uint32_t litbase = incl - cnt_t, nlit = 0, nsamp = 0;
        for (int w2 = 0; w2 < kZWaves; ++w2) {
            litbase += w2 < wave ? pc.wsum[w2] : 0u;
            nlit += pc.wsum[w2];
            nsamp += pc.wsum2[w2];
        }
        if (tid < 256) {
            uint32_t c = 0;
            for (int w2 = 0; w2 < kZWaves; ++w2) c += A.wh[w2 * 256 + tid];
            A.hist[tid] = c;
        }
        __syncthreads();
        if (wave == 0) {  // 1: the full histogram is needed; 0: raw literals
            uint32_t need = nlit > 0;
            if (nlit >= 32 && nsamp > 0) {
                uint64_t es = 0;
                const uint32_t lm = lg256(nsamp);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t c = A.hist[lane + 64 * i];
                    if (c) es += (uint64_t)c * (lm - lg256(c));
                }
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) es += __shfl_xor(es, d, 64);
                if (es * nlit / nsamp / 2048 + 64 >= (uint64_t)nlit - nlit / 64) need = 0;
            }
            if (lane == 0) pc.need_full = need;
        }
        __syncthreads();
        const uint32_t need_full = pc.need_full;
        const uint32_t rawh = nlit < 32 ? 1u : nlit < 4096 ? 2u : 3u;
        if (!need_full && rawh + nlit + 1 >= n) {
            // raw literals and at least a one-byte sequence section: the compressed block
            // cannot be shorter than the block (the entropy kernel's body < n test), so the raw
            // block goes out here, from the staged window (the entropy kernel skips the item;
            // from global memory it would read the 64 KiB again: a VM image's random pages)
            stage_to_global(out + 3, W, hist, n, (uint32_t)tid, kZThreads);
            if (tid == 0) {
                write_block_header(out, last, 0, n);
                sizes[k] = 3 + (uint64_t)n;
                zi->kind = 1;
            }
            continue;
        }
        if (need_full) {
            for (uint32_t i = tid; i < kZWaves * 256; i += kZThreads) A.wh[i] = 0;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; ++i)
                for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1)
                    atomicAdd(&wh[W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2))], 1u);
            __syncthreads();
            if (tid < 256) {
                uint32_t c = 0;
                for (int w2 = 0; w2 < kZWaves; ++w2) c += A.wh[w2 * 256 + tid];
                zi->hist[tid] = c;
            }
        }
        if (tid < 36 + 53 + 32) {
            uint32_t c = 0;
            for (int w2 = 0; w2 < kZWaves; ++w2) c += A.wc[w2 * 128 + tid];
            zi->shist[tid] = c;
        }
        if (tid < kZWaves) zi->nseq[tid] = pc.nseq[tid];
        if (tid == 0) {
            zi->kind = 0;
            zi->nlit = nlit;
            zi->need_full = need_full;
            if (deal) elist[atomicAdd(deal + 2, 1u)] = (uint32_t)k;  // the entropy kernel's items
        }
        ZMARK(2);
        // ---- the literals compacted in order to global memory (through LDS, dword stores):
        // for the entropy kernel, or -- raw literals for sure (no full histogram) -- straight
        // to their place in the block (behind the raw literal header the entropy kernel writes)
        uint8_t* const lo = need_full ? lit_items + k * (uint64_t)kEncBlock : out + 3 + rawh;
        uint32_t nseq_b = 0;
#pragma unroll
        for (int w2 = 0; w2 < kZWaves; ++w2) nseq_b += min(pc.nseq[w2], kZSubSeq);
        if (nseq_b < kZRuns) {
            // few sequences (a VM image's random pages: ~40 KB of literals in a handful of
            // runs): the runs straight from the staged window with dword stores, as the fused
            // kernel does -- the bitmap compaction below is an LDS byte round trip per literal
            if (wave == 0) {
                const Coded x = (uint32_t)lane < nseq_b ? coded[lane] : Coded{0, 0, 0, 0};
                const uint32_t span = x.ll + x.ml, lit = x.ll;
                const uint32_t si = wave_incl(span, lane), li = wave_incl(lit, lane);
                if ((uint32_t)lane <= nseq_b) {
                    pc.run_start[lane] = si - span;
                    pc.run_out[lane] = li - lit;
                    pc.run_len[lane] = (uint32_t)lane < nseq_b ? lit : (n > si - span ? n - (si - span) : 0u);  // (never a wrapped length)
                }
            }
            __syncthreads();
            for (uint32_t r2 = 0; r2 <= nseq_b; ++r2)
                stage_to_global(lo + pc.run_out[r2], W, hist + pc.run_start[r2], pc.run_len[r2], (uint32_t)tid,
                                kZThreads);
        }
        for (uint32_t pb = 0; pb < (nseq_b < kZRuns ? 0u : nlit); pb += (uint32_t)sizeof(A.lit)) {
            const uint32_t pe = min(nlit, pb + (uint32_t)sizeof(A.lit));
            uint32_t idx = litbase;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                for (uint32_t m2 = bmw[i]; m2; m2 &= m2 - 1, ++idx)
                    if (idx >= pb && idx < pe) A.lit[idx - pb] = (uint8_t)W.byte(hist + 128 * tid + 32 * i + __builtin_ctz(m2));
            __syncthreads();
            lds_to_global(lo + pb, reinterpret_cast<const uint32_t*>(A.lit), pe - pb, (uint32_t)tid, kZThreads);
            __syncthreads();
        }
        if (probe) {
            g_zprobe[10] += 1;
            g_zprobe[11] += min(pc.nseq[0], kZSubSeq) + min(pc.nseq[1], kZSubSeq) + min(pc.nseq[2], kZSubSeq) +
                            min(pc.nseq[3], kZSubSeq) + min(pc.nseq[4], kZSubSeq) + min(pc.nseq[5], kZSubSeq) +
                            min(pc.nseq[6], kZSubSeq) + min(pc.nseq[7], kZSubSeq);
            g_zprobe[12] += nlit;
        }
        ZMARK(15);
    }
}

// thread t of nt: the compacted literals [i0, i1) of `lits` (16-byte aligned) in order,
// fn(index, byte); 64 bytes (four 16-byte loads) in flight at a time -- the parse kernel
// wrote them, so they come from HBM
template <typename F>
__device__ __forceinline__ void for_literals(const uint8_t* __restrict__ lits, uint32_t i0, uint32_t i1, F&& fn) {
    if (i0 >= i1) return;
    const v4u* const q = reinterpret_cast<const v4u*>(lits);
    const uint32_t wl = (i1 - 1) >> 4;
    for (uint32_t w0 = i0 >> 4; w0 <= wl; w0 += 4) {
        v4u c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = q[w0 + (uint32_t)k <= wl ? w0 + (uint32_t)k : wl];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (w0 + (uint32_t)k > wl) break;
            const uint32_t d[4] = {c[k].x, c[k].y, c[k].z, c[k].w};
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                const uint32_t i = 16 * (w0 + (uint32_t)k) + (uint32_t)b;
                if (i >= i0 && i < i1) fn(i, (d[b >> 2] >> (8 * (b & 3))) & 0xFFu);
            }
        }
    }
}

__global__ __launch_bounds__(kEThreads) __attribute__((amdgpu_waves_per_eu(3, 3))) void zstd_entropy_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint64_t* __restrict__ items, uint64_t nitems, uint8_t* __restrict__ slots, uint64_t* __restrict__ sizes,
    const Coded* __restrict__ coded_items, const uint8_t* __restrict__ lit_items, const ZItem* __restrict__ zitems,
    uint32_t* __restrict__ chain_scratch, uint32_t* __restrict__ deal, const uint32_t* __restrict__ elist,
    int probe_on) {
    __shared__ __attribute__((aligned(16))) EArea E;
    __shared__ uint32_t s_next;
    __shared__ FseT fse[3];   // LL, OF, ML
    __shared__ FseT fse_huf;  // the Huffman description's scratch
    __shared__ PreT pre[3];
    __shared__ Ctl ctl;
    const int tid = threadIdx.x, lane = tid & 63, wave = (int)uni((uint32_t)tid >> 6);
    const bool probe = probe_on && blockIdx.x == 0 && tid == 0;
    uint64_t tp = probe ? wall_clock64() : 0;
    uint32_t* const chains = chain_scratch + (uint64_t)blockIdx.x * 6 * kZBlockSeq;
    if (wave == 0 && lane < 3) {  // the predefined tables, once per launch
        FseT& t = fse[lane];
        if (lane == 0) fse_build(t, kLLNorm, 36, kLLLog);
        if (lane == 1) fse_build(t, kOFNorm, 29, kOFLog);
        if (lane == 2) fse_build(t, kMLNorm, 53, kMLLog);
        PreT& q = pre[lane];
        for (int i = 0; i < 64; ++i) q.next[i] = t.next[i];
        for (int i = 0; i < 53; ++i) {
            q.dnb[i] = t.dnb[i];
            q.dfs[i] = t.dfs[i];
        }
        q.log = t.log;
    }
    // dealt: the items the parse kernel listed (the rest are done: RLE, raw, empty);
    // static: every item, skipping those
    const uint64_t ne = deal ? (uint64_t)*reinterpret_cast<volatile const uint32_t*>(deal + 1) : nitems;  // (deal[1]: the parse kernel's deal[2])
    for (uint64_t e = deal_item(deal, s_next, blockIdx.x); e < ne; e = deal_item(deal, s_next, e + gridDim.x)) {
        __syncthreads();  // LDS of the previous item
        ZMARK(54);
        const uint64_t k = deal ? (uint64_t)elist[e] : e;
        const ZItem* const zi = zitems + k;
        if (uni(zi->kind)) continue;
        const uint64_t it = items[k];
        const uint64_t ci = it >> 32, j = (uint32_t)it;
        const uint64_t c0 = bounds[2 * ci], c1 = bounds[2 * ci + 1];
        const uint64_t len = c1 - c0, off = j * (uint64_t)kEncBlock;
        const uint32_t n = (uint32_t)(len - off < kEncBlock ? len - off : kEncBlock);
        const bool last = off + n == len;
        uint8_t* const out = slots + k * kSlot;
        const Coded* const coded = coded_items + k * (uint64_t)kZBlockSeq;
        const uint8_t* const lits = lit_items + k * (uint64_t)kEncBlock;
        const uint32_t nlit = uni(zi->nlit), need_full = uni(zi->need_full);
        uint32_t nseq = 0;
#pragma unroll
        for (int w2 = 0; w2 < kZWaves; ++w2) nseq += min(uni(zi->nseq[w2]), kZSubSeq);
        if (tid < kZWaves) ctl.nseq[tid] = zi->nseq[tid];
        if (tid < 36 + 53 + 32) E.shist[tid] = zi->shist[tid];
        if (need_full) E.hist[tid] = zi->hist[tid];  // (kEThreads == 256)
        if (tid == 0) ctl.lit_mode = 0;
        __syncthreads();
        ZMARK(48);
        // ---- the literal mode (wave 0) beside the sequence tables and chains (waves 1-3)
        const bool role_probe = probe_on && blockIdx.x == 0;
        uint64_t zt = role_probe ? wall_clock64() : 0;
        auto role_end = [&](int idx) {
            if (role_probe && lane == 0) {
                const uint64_t t2 = wall_clock64();
                atomicAdd(&g_zprobe[idx], t2 - zt);
                zt = t2;
            }
        };
        if (wave == 0) {
            if (need_full) literal_mode_wave(E, ctl, fse_huf, nlit, lane, role_probe ? g_zprobe : nullptr);
            role_end(17);
        } else {
            const int kk = wave - 1;  // 0 LL, 1 OF, 2 ML
            const uint32_t sh = kk == 0 ? 0u : kk == 1 ? 16u : 8u;
            uint32_t* const hk = E.shist + (kk == 0 ? 0 : kk == 1 ? 36 + 53 : 36);
            if (nseq > 0) {
                if (kk == 0) seq_table_wave(fse[0], hk, 36, nseq, kLLNorm, kLLLog, kLLMaxLog, lane);
                if (kk == 1) seq_table_wave(fse[1], hk, 29, nseq, kOFNorm, kOFLog, kOFMaxLog, lane);
                if (kk == 2) seq_table_wave(fse[2], hk, 53, nseq, kMLNorm, kMLLog, kMLMaxLog, lane);
            }
            if (wave == 1) role_end(19);
            if (nseq >= 2 && fse[kk].mode != 1) {
                const FseView tv = fse[kk].mode == 2 ? view(fse[kk]) : view(pre[kk]);
                seq_chain_wave(tv, coded, nseq, sh, chains + (uint64_t)kk * kZBlockSeq,
                               reinterpret_cast<uint16_t*>(chains + 3ull * kZBlockSeq) + (uint64_t)kk * kZBlockSeq,
                               reinterpret_cast<uint8_t*>(chains + 3ull * kZBlockSeq + 3ull * kZBlockSeq / 2) +
                                   (uint64_t)kk * (kZBlockSeq + 16),
                               &ctl.seq_last[kk], lane, role_probe && kk == 0 ? g_zprobe : nullptr);
                __threadfence_block();
            }
            if (wave == 1) role_end(20);
        }
        __syncthreads();
        ZMARK(49);
        // ---- Huffman sizes: thread t's literals [i0, i1) of the compacted list, a block scan
        const uint32_t lit_mode = ctl.lit_mode;
        const uint32_t per = ((nlit + kEThreads - 1) / kEThreads + 15) & ~15u;
        const uint32_t i0 = min(nlit, (uint32_t)tid * per), i1 = min(nlit, i0 + per);
        uint32_t bits_t = 0;
        if (lit_mode == 2) for_literals(lits, i0, i1, [&](uint32_t, uint32_t sym) { bits_t += E.len[sym]; });
        const uint32_t bincl = wave_incl(bits_t, lane);
        if (lane == 63) ctl.wsum2[wave] = bincl;
        const bool four = nlit >= 256;
        const uint32_t seg = four ? (nlit + 3) / 4 : nlit;
        __syncthreads();
        ZMARK(50);
        uint32_t bbase = bincl - bits_t;
        for (int w2 = 0; w2 < wave; ++w2) bbase += ctl.wsum2[w2];
        if (lit_mode == 2) {
            if (tid == 0) {
                ctl.segP[0] = 0;
                uint32_t tot = 0;
                for (int w2 = 0; w2 < kEWaves; ++w2) tot += ctl.wsum2[w2];
                ctl.segP[4] = tot;
                if (!four) ctl.segP[1] = tot;
            }
            // the thread holding literal index seg * s records the bits before it
            if (four && i0 < i1 && (i0 / seg != (i1 - 1) / seg || i0 % seg == 0)) {
                uint32_t pb = bbase;
                for_literals(lits, i0, i1, [&](uint32_t idx, uint32_t sym) {
                    if (idx == seg || idx == 2 * seg || idx == 3 * seg) ctl.segP[idx / seg] = pb;
                    pb += E.len[sym];
                });
            }
        }
        __syncthreads();
        if (tid == 0) {  // literal section: size decision
            uint32_t lm = lit_mode, sz = 0;
            const uint32_t rawh = nlit < 32 ? 1u : nlit < 4096 ? 2u : 3u;
            if (lm == 2) {
                uint32_t sb = 0;
                const int ns4 = four ? 4 : 1;
                for (int s2 = 0; s2 < ns4; ++s2) sb += (ctl.segP[four ? s2 + 1 : 4] - ctl.segP[s2] + 8) / 8;
                const uint32_t c = ctl.desc_len + (four ? 6u : 0u) + sb;
                const uint32_t mx = max(nlit, c);
                const uint32_t hs = mx < 1024 ? 3u : mx < 16384 ? 4u : 5u;
                if (sb > kHufStreams || hs + c >= rawh + nlit) {
                    lm = 0;
                } else {
                    sz = hs + c;
                    ctl.huf_c = c;
                    ctl.huf_hs = hs;
                }
            }
            if (lm == 0) sz = rawh + nlit;
            if (lm == 1) sz = rawh + 1;
            ctl.lit_mode = lm;
            ctl.lit_size = sz;
        }
        __syncthreads();
        ZMARK(51);
        const uint32_t lm = ctl.lit_mode, lsz = ctl.lit_size;
        uint8_t* const lit_out = out + 3;
        if (probe) g_zprobe[55] += 1;
        // ---- the sequence section header (thread 0)
        if (tid == 0) {
            uint8_t* o = lit_out + lsz;
            uint8_t* const o0 = o;
            const uint32_t ns = nseq;
            if (ns < 128) {
                *o++ = (uint8_t)ns;
            } else if (ns < 0x7F00) {
                *o++ = (uint8_t)((ns >> 8) + 0x80);
                *o++ = (uint8_t)ns;
            } else {
                *o++ = 0xFF;
                *o++ = (uint8_t)(ns - 0x7F00);
                *o++ = (uint8_t)((ns - 0x7F00) >> 8);
            }
            if (ns) {
                *o++ = (uint8_t)(fse[0].mode << 6 | fse[1].mode << 4 | fse[2].mode << 2);
                for (int kk = 0; kk < 3; ++kk)
                    for (uint32_t i = 0; i < fse[kk].desc_len; ++i) *o++ = fse[kk].desc[i];
            }
            ctl.seq_hdr = (uint32_t)(o - o0);
            if (ns == 1)  // a single sequence's states come from its own codes
                for (int kk = 0; kk < 3; ++kk)
                    if (fse[kk].mode != 1) {
                        const uint32_t sh = kk == 0 ? 0u : kk == 1 ? 16u : 8u;
                        const FseView tv = fse[kk].mode == 2 ? view(fse[kk]) : view(pre[kk]);
                        ctl.seq_last[kk] = fse_init(tv, (coded[0].codes >> sh) & 0xFF);
                    }
        }
        // ---- the literal section
        if (lm == 2) {
            const uint32_t S0 = 0;
            const uint32_t S1 = four ? (ctl.segP[1] - ctl.segP[0] + 8) / 8 : (ctl.segP[4] - ctl.segP[0] + 8) / 8;
            const uint32_t S2 = four ? S1 + (ctl.segP[2] - ctl.segP[1] + 8) / 8 : S1;
            const uint32_t S3 = four ? S2 + (ctl.segP[3] - ctl.segP[2] + 8) / 8 : S1;
            const uint32_t S4 = four ? S3 + (ctl.segP[4] - ctl.segP[3] + 8) / 8 : S1;
            auto Sat = [&](uint32_t g) { return g == 0 ? S0 : g == 1 ? S1 : g == 2 ? S2 : g == 3 ? S3 : S4; };
            const uint32_t hs = ctl.huf_hs, c = ctl.huf_c;
            const uint32_t dl = ctl.desc_len;
            uint8_t* const body = lit_out + hs;
            const uint32_t tot = four ? S4 : S1;
            // the streams in LDS, or (longer than its buffer) straight into the output: its
            // bytes zeroed, then ORed into the aligned words around them (the bytes before
            // are the section header, ORed with zeros; the ones after are written later)
            uint8_t* const sdst = body + dl + (four ? 6 : 0);
            const bool in_lds = tot + 16 <= (uint32_t)sizeof(E.streams);
            uint32_t* const gw = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(sdst) & ~(uintptr_t)3);
            const uint32_t gsh = 8u * (uint32_t)(sdst - reinterpret_cast<uint8_t*>(gw));
            if (in_lds) {
                for (uint32_t i = tid; i < (tot + 3) / 4 + 2; i += kEThreads) E.streams[i] = 0;
            } else {
                for (uint32_t i = tid; i < tot; i += kEThreads) sdst[i] = 0;
                __threadfence_block();
            }
            __syncthreads();
            // (two loops, each with its address space in the pointer's type: one lambda
            // choosing between the buffers made every OR a flat atomic, LDS ones included)
            lds_u32* const ls = (lds_u32*)E.streams;
            PBS_GLOBAL uint32_t* const gg = (PBS_GLOBAL uint32_t*)gw;
            auto orbits = [&](uint32_t o, uint64_t v, uint32_t L) {
                if (in_lds) {
                    __hip_atomic_fetch_or(&ls[o >> 5], (uint32_t)(v << (o & 31)), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                    if ((o & 31) + L > 32)
                        __hip_atomic_fetch_or(&ls[(o >> 5) + 1], (uint32_t)((v << (o & 31)) >> 32), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    const uint32_t og = o + gsh;
                    const uint64_t w = v << (og & 31);
                    __hip_atomic_fetch_or(&gg[og >> 5], (uint32_t)w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((og & 31) + L > 32)
                        __hip_atomic_fetch_or(&gg[(og >> 5) + 1], (uint32_t)(w >> 32), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                }
            };
            uint32_t pb = bbase;
            auto lit_bits = [&](uint32_t idx, uint32_t sym, auto&& put) {
                const uint32_t L = E.len[sym], cv = E.code[sym];
                const uint32_t sg = four ? min(idx / seg, 3u) : 0u;
                const uint32_t endP = four ? ctl.segP[sg + 1] : ctl.segP[4];
                put(8 * Sat(sg) + (endP - pb - L), (uint64_t)cv, L);
                pb += L;
            };
            if (in_lds)
                for_literals(lits, i0, i1, [&](uint32_t idx, uint32_t sym) {
                    lit_bits(idx, sym, [&](uint32_t o, uint64_t v, uint32_t L) {
                        __hip_atomic_fetch_or(&ls[o >> 5], (uint32_t)(v << (o & 31)), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                        if ((o & 31) + L > 32)
                            __hip_atomic_fetch_or(&ls[(o >> 5) + 1], (uint32_t)((v << (o & 31)) >> 32),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    });
                });
            else
                for_literals(lits, i0, i1, [&](uint32_t idx, uint32_t sym) { lit_bits(idx, sym, orbits); });
            if (tid < (four ? 4 : 1)) {  // end marks
                const uint32_t bits = ctl.segP[four ? tid + 1 : 4] - ctl.segP[tid];
                orbits(8 * Sat((uint32_t)tid) + bits, 1ull, 1);
            }
            if (!in_lds) __threadfence_block();
            __syncthreads();
            if (tid == 0) {
                if (hs == 3) {
                    const uint32_t v = 2u | (four ? 1u : 0u) << 2 | nlit << 4 | c << 14;
                    lit_out[0] = (uint8_t)v;
                    lit_out[1] = (uint8_t)(v >> 8);
                    lit_out[2] = (uint8_t)(v >> 16);
                } else if (hs == 4) {
                    const uint32_t v = 2u | 2u << 2 | nlit << 4 | c << 18;
                    for (int i = 0; i < 4; ++i) lit_out[i] = (uint8_t)(v >> (8 * i));
                } else {
                    const uint64_t v = 2u | 3u << 2 | (uint64_t)nlit << 4 | (uint64_t)c << 22;
                    for (int i = 0; i < 5; ++i) lit_out[i] = (uint8_t)(v >> (8 * i));
                }
                if (four)
                    for (int s2 = 0; s2 < 3; ++s2) {
                        const uint32_t sz = Sat((uint32_t)s2 + 1) - Sat((uint32_t)s2);
                        body[dl + 2 * s2] = (uint8_t)sz;
                        body[dl + 2 * s2 + 1] = (uint8_t)(sz >> 8);
                    }
            }
            for (uint32_t i = tid; i < dl; i += kEThreads) body[i] = ctl.desc[i];
            if (in_lds) lds_to_global(sdst, E.streams, tot, (uint32_t)tid, kEThreads);
        } else {
            const uint32_t rawh = nlit < 32 ? 1u : nlit < 4096 ? 2u : 3u;
            if (tid == 0) {
                const uint32_t t = lm;  // 0 raw, 1 RLE
                if (rawh == 1) {
                    lit_out[0] = (uint8_t)(t | nlit << 3);
                } else if (rawh == 2) {
                    lit_out[0] = (uint8_t)(t | 1u << 2 | nlit << 4);
                    lit_out[1] = (uint8_t)(nlit >> 4);
                } else {
                    lit_out[0] = (uint8_t)(t | 3u << 2 | nlit << 4);
                    lit_out[1] = (uint8_t)(nlit >> 4);
                    lit_out[2] = (uint8_t)(nlit >> 12);
                }
                if (lm == 1) {  // the one distinct byte
                    uint32_t s2 = 0;
                    while (!E.hist[s2]) ++s2;
                    lit_out[rawh] = (uint8_t)s2;
                }
            }
            // (without the full histogram the parse kernel put them in place already)
            if (lm == 0 && need_full) copy_global(lit_out + rawh, lits, nlit, (uint32_t)tid, kEThreads);
        }
        if (wave == 0) role_end(21);
        __syncthreads();
        ZMARK(52);
        // ---- the sequence bit stream (the fused kernel's, over 256 threads)
        {
            const uint32_t ns = nseq, hdr = ctl.seq_hdr;
            const uint32_t mode[3] = {fse[0].mode, fse[1].mode, fse[2].mode};
            const uint32_t pq = (ns + kEThreads - 1) / kEThreads;
            const uint32_t q0 = min(ns, (uint32_t)tid * pq), q1 = min(ns, q0 + pq);
            // (the coded records come from HBM -- the parse kernel wrote them -- so 8 are
            // loaded, with their chain fields, before any is used)
            auto load8 = [&](uint32_t qb, Coded (&x)[8], uint32_t (&cl)[8], uint32_t (&co)[8], uint32_t (&cm)[8]) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t q = qb + (uint32_t)u < q1 ? qb + (uint32_t)u : q1 - 1;
                    const v4u r = *reinterpret_cast<const v4u*>(coded + q);
                    x[u] = Coded{r.x, r.y, r.z, r.w};
                    const uint32_t jj = q + 1 < ns ? ns - 2 - q : 0u;
                    cl[u] = chains[jj];
                    co[u] = chains[kZBlockSeq + jj];
                    cm[u] = chains[2 * kZBlockSeq + jj];
                }
            };
            uint32_t st = 0;
            for (uint32_t qb = q0; qb < q1; qb += 8) {
                Coded x[8];
                uint32_t cl[8], co[8], cm[8];
                load8(qb, x, cl, co, cm);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t q = qb + (uint32_t)u;
                    if (q >= q1) break;
                    const uint32_t llc = x[u].codes & 0xFF, mlc = (x[u].codes >> 8) & 0xFF, ofc = x[u].codes >> 16;
                    uint32_t b = ll_bits(llc) + ml_bits(mlc) + ofc;
                    if (q + 1 < ns) {
                        if (mode[0] != 1) b += cl[u] >> 16;
                        if (mode[1] != 1) b += co[u] >> 16;
                        if (mode[2] != 1) b += cm[u] >> 16;
                    }
                    st += b;
                }
            }
            const uint32_t si = wave_incl(st, lane);
            if (lane == 63) ctl.wsum[wave] = si;
            __syncthreads();
            uint32_t pt = si - st, T = 0;
            for (int w2 = 0; w2 < kEWaves; ++w2) {
                pt += w2 < wave ? ctl.wsum[w2] : 0u;
                T += ctl.wsum[w2];
            }
            uint32_t flushb = 0;
            for (int kk = 0; kk < 3; ++kk)
                if (ns && mode[kk] != 1) flushb += (uint32_t)(mode[kk] == 2 ? fse[kk].log : pre[kk].log);
            // this thread's sequences into a bit writer, last first (the stream is backwards),
            // 8 records loaded before any is written
            auto put_range = [&](auto& ob) {
                for (uint32_t qe = q1; qe > q0;) {
                    const uint32_t qb = qe >= q0 + 8 ? qe - 8 : q0;
                    Coded x[8];
                    uint32_t cl[8], co[8], cm[8];
                    load8(qb, x, cl, co, cm);
#pragma unroll
                    for (int u = 7; u >= 0; --u) {
                        const uint32_t q = qb + (uint32_t)u;
                        if (q >= qe) continue;
                        const uint32_t llc = x[u].codes & 0xFF, mlc = (x[u].codes >> 8) & 0xFF, ofc = x[u].codes >> 16;
                        if (q + 1 < ns) {
                            if (mode[1] != 1) ob.put(co[u] & 0xFFFF, co[u] >> 16);
                            if (mode[2] != 1) ob.put(cm[u] & 0xFFFF, cm[u] >> 16);
                            if (mode[0] != 1) ob.put(cl[u] & 0xFFFF, cl[u] >> 16);
                        }
                        ob.put(x[u].ll - ll_base(llc), ll_bits(llc));
                        ob.put(x[u].ml - ml_base(mlc), ml_bits(mlc));
                        ob.put(x[u].ofv - (1u << ofc), ofc);
                    }
                    qe = qb;
                }
            };
            const uint32_t sbytes = ns ? (T + flushb + 1 + 7) / 8 : 0u;
            const uint32_t body = lsz + hdr + sbytes;
            const bool ok = body < n;
            const uint32_t lastw_l = ns ? (8u * (uint32_t)((uintptr_t)(lit_out + lsz + hdr) & 3u) + T + flushb) >> 5 : 0u;
            if (ok && ns && lastw_l + 1 <= (uint32_t)(sizeof(E.streams) / 4)) {
                uint8_t* const S0 = lit_out + lsz + hdr;
                uint32_t* const Aw = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(S0) & ~(uintptr_t)3);
                const uint32_t off0 = 8u * (uint32_t)(S0 - reinterpret_cast<uint8_t*>(Aw));
                const uint32_t lastw = lastw_l;
                uint32_t* const L = E.streams;
                for (uint32_t wdx = tid; wdx <= lastw; wdx += kEThreads) L[wdx] = 0;
                __syncthreads();
                OrBitsL ob;
                ob.init(L, off0 + (T - pt - st));
                put_range(ob);
                ob.done();
                if (tid == kEThreads - 1) {  // the final states (ML, OF, LL) and the end mark
                    OrBitsL fb;
                    fb.init(L, off0 + T);
                    if (mode[2] != 1) fb.put(ctl.seq_last[2], (uint32_t)(mode[2] == 2 ? fse[2].log : pre[2].log));
                    if (mode[1] != 1) fb.put(ctl.seq_last[1], (uint32_t)(mode[1] == 2 ? fse[1].log : pre[1].log));
                    if (mode[0] != 1) fb.put(ctl.seq_last[0], (uint32_t)(mode[0] == 2 ? fse[0].log : pre[0].log));
                    fb.put(1, 1);
                    fb.done();
                }
                __syncthreads();
                for (uint32_t wdx = tid; wdx <= lastw; wdx += kEThreads)
                    Aw[wdx] = wdx ? L[wdx] : (off0 ? Aw[0] & ((1u << off0) - 1u) : 0u) | L[0];
            } else if (ok && ns) {
                uint8_t* const S0 = lit_out + lsz + hdr;
                uint32_t* const Aw = reinterpret_cast<uint32_t*>(reinterpret_cast<uintptr_t>(S0) & ~(uintptr_t)3);
                const uint32_t off0 = 8u * (uint32_t)(S0 - reinterpret_cast<uint8_t*>(Aw));
                const uint32_t lastw = (off0 + T + flushb + 1 - 1) >> 5;
                if (tid == 0)
                    for (uint8_t* b = S0; b < reinterpret_cast<uint8_t*>(Aw + 1); ++b) *b = 0;
                for (uint32_t wdx = 1 + tid; wdx <= lastw; wdx += kEThreads) Aw[wdx] = 0;
                __threadfence_block();  // the zeros (and the section header) stored before any atomicOr
                __syncthreads();
                OrBits ob;
                ob.init(Aw, off0 + (T - pt - st));
                put_range(ob);
                ob.done();
                if (tid == kEThreads - 1) {
                    OrBits fb;
                    fb.init(Aw, off0 + T);
                    if (mode[2] != 1) fb.put(ctl.seq_last[2], (uint32_t)(mode[2] == 2 ? fse[2].log : pre[2].log));
                    if (mode[1] != 1) fb.put(ctl.seq_last[1], (uint32_t)(mode[1] == 2 ? fse[1].log : pre[1].log));
                    if (mode[0] != 1) fb.put(ctl.seq_last[0], (uint32_t)(mode[0] == 2 ? fse[0].log : pre[0].log));
                    fb.put(1, 1);
                    fb.done();
                }
            }
            if (tid == 0) {
                ctl.seq_ok = ok;
                ctl.seq_size = body;
            }
        }
        __syncthreads();
        ZMARK(53);
        if (!ctl.seq_ok) {  // raw block
            copy_global(out + 3, data + (c0 - base) + off, n, (uint32_t)tid, kEThreads);
            if (tid == 0) {
                write_block_header(out, last, 0, n);
                sizes[k] = 3 + (uint64_t)n;
            }
        } else if (tid == 0) {
            write_block_header(out, last, 2, ctl.seq_size);
            sizes[k] = 3 + (uint64_t)ctl.seq_size;
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
    const uint64_t len = bounds[2 * ci + 1] - bounds[2 * ci];
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
// block, the magic and the frame header); otherwise the item's 64 KiB of chunk bytes.
__global__ __launch_bounds__(kZThreads) void zstd_assemble_kernel(
    const uint8_t* __restrict__ data, uint64_t base, const uint64_t* __restrict__ bounds,
    const uint64_t* __restrict__ items, uint64_t nitems, const uint64_t* __restrict__ first,
    const uint8_t* __restrict__ slots, const uint64_t* __restrict__ sizes, const uint64_t* __restrict__ ipre,
    const uint64_t* __restrict__ boff, const uint8_t* __restrict__ comp, uint8_t* __restrict__ blobs) {
    for (uint64_t k = blockIdx.x; k < nitems; k += gridDim.x) {
        const uint64_t it = items[k];
        const uint64_t ci = it >> 32, j = (uint32_t)it;
        const uint64_t len = bounds[2 * ci + 1] - bounds[2 * ci];
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
            const uint8_t* const src = data + (bounds[2 * ci] - base) + off;
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

// Work areas of pbs_blob_encode_chunks_device, per device (dev_arena.h): the block slots
// (~ the input size), the sequence lists of the resident workgroups and the per-call
// arrays.  Concurrent calls on one device lease different arenas; a call in steady state
// allocates and frees nothing.
ArenaPool& zpool() {
    static ArenaPool* p = new ArenaPool;  // never destroyed (HIP may be torn down first at exit)
    return *p;
}
enum ZSlot : unsigned { kZsBounds, kZsItems, kZsFirst, kZsSizes, kZsIpre, kZsBsz, kZsBoff, kZsComp, kZsCrc, kZsTmp,
                        kZsSlots, kZsSeqs, kZsCoded, kZsChains, kZsZItems, kZsLits, kZsDeal, kZsEList };

}  // namespace
}  // namespace pbs

using namespace pbs;

extern "C" size_t pbs_zstd_frame_bound(size_t len) { return (size_t)zstd::frame_bound(len); }

// Frees the blob encoder's idle device work areas (~ the bytes of the largest call each)
// and the calling thread's CRC counters of the shared streams.
extern "C" void pbs_blob_encode_release(void) {
    zpool().clear();
    release_thread_counters();
}

extern "C" size_t pbs_blob_stream_bound(const uint64_t* bounds, size_t n) {
    if (!bounds || n == 0) return 0;
    return 12 * n + (size_t)(bounds[n] - bounds[0]);
}

// The chunks as spans {start, end} (absolute stream offsets; any order, gaps allowed):
// pbs_blob_encode_spans_device, and pbs_blob_encode_chunks_device through it.
extern "C" int pbs_blob_encode_spans_device(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                            const uint64_t* spans, size_t n, int compress, uint8_t* blobs_dev,
                                            size_t blobs_cap, uint64_t* blob_offsets, uint32_t* crcs,
                                            uint8_t* compressed, pbs_blob_encode_timing* timing,
                                            void* hip_stream) {
    using Clock = std::chrono::steady_clock;
    const Clock::time_point t0 = Clock::now();
    if (timing) std::memset(timing, 0, sizeof(*timing));
    if (!blob_offsets) return PBS_ERR_INVALID;
    blob_offsets[0] = 0;
    if (n == 0) return PBS_OK;
    if (!spans || !blobs_dev || (data_len && !dev_data) || n >= 0xFFFFFFFFull) return PBS_ERR_INVALID;
    uint64_t bytes_in = 0;
    for (size_t i = 0; i < n; ++i) {
        if (spans[2 * i] > spans[2 * i + 1] || spans[2 * i] < base || spans[2 * i + 1] - base > data_len)
            return PBS_ERR_INVALID;
        // the reference refuses blobs over MAX_BLOB_SIZE (data_blob.rs:92, 128 MiB, :13)
        if (spans[2 * i + 1] - spans[2 * i] > (128ull << 20)) return PBS_ERR_INVALID;
        bytes_in += spans[2 * i + 1] - spans[2 * i];
    }
    const uint64_t* const bounds = spans;  // (device copies below: 2 n entries)
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
        const uint64_t len = bounds[2 * i + 1] - bounds[2 * i];
        const uint64_t nb = len ? (len + zstd::kEncBlock - 1) / zstd::kEncBlock : 1;
        for (uint64_t j = 0; j < nb; ++j) items.push_back((uint64_t)i << 32 | j);
    }
    first[n] = items.size();
    const uint64_t ni = items.size();

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
    // one 512-thread workgroup per CU the stream may use (a CU-masked stream, e.g. the upload
    // path's beside the digest queue, gets as many workgroups as its mask has CUs: the items
    // are dealt statically, and a workgroup waiting for a CU would hold the whole kernel)
    int use_cu = ncu;
    {
        uint32_t mask[16] = {};
        if (ncu <= 512 && hipExtStreamGetCUMask(st, 16, mask) == hipSuccess) {
            int bits = 0;
            for (uint32_t w : mask) bits += __builtin_popcount(w);
            if (bits > 0 && bits < use_cu) use_cu = bits;
        }
        (void)hipGetLastError();
    }
    const unsigned grid = (unsigned)std::min<uint64_t>(ni, (uint64_t)use_cu);
    ArenaLease ar(zpool(), dev);
    uint64_t* d_bounds = ar->get<uint64_t>(kZsBounds, 2 * n * 8);
    uint64_t* d_items = ar->get<uint64_t>(kZsItems, ni * 8);
    uint64_t* d_first = ar->get<uint64_t>(kZsFirst, (n + 1) * 8);
    uint64_t* d_sizes = ar->get<uint64_t>(kZsSizes, (ni + 1) * 8);
    uint64_t* d_ipre = ar->get<uint64_t>(kZsIpre, (ni + 1) * 8);
    uint64_t* d_bsz = ar->get<uint64_t>(kZsBsz, (n + 1) * 8);
    uint64_t* d_boff = ar->get<uint64_t>(kZsBoff, (n + 1) * 8);
    uint8_t* d_comp = ar->get<uint8_t>(kZsComp, n);
    uint32_t* d_crc = ar->get<uint32_t>(kZsCrc, n * 4);
    void* d_tmp = ar->get<void>(kZsTmp, std::max<size_t>(tmpb, 256));
    uint8_t* z_slots = nullptr;
    Seq* z_seqs = nullptr;
    Coded* z_coded = nullptr;
    uint32_t* z_chains = nullptr;
    // the split kernels (default; PBS_ZSTD_SPLIT=0: the fused kernel, A/B): the parse kernel on
    // one workgroup per CU, the entropy kernel on three per CU, items in batches of zbatch whose
    // coded sequences, literals and ZItem records wait in global memory between the two
    static const bool split = [] {
        const char* e = std::getenv("PBS_ZSTD_SPLIT");
        return !(e && e[0] == '0');
    }();
    // (read per call, so a test can run many small batches and both dealings in one process)
    const bool zdeal = [] {  // PBS_ZSTD_DEAL=0: items dealt statically (A/B)
        const char* e = std::getenv("PBS_ZSTD_DEAL");
        return !(e && e[0] == '0');
    }();
    const uint64_t zbatch = [] {
        const char* e = std::getenv("PBS_ZSTD_BATCH");
        const uint64_t v = e ? std::strtoull(e, nullptr, 0) : 0;
        // 32768 items (2 GiB of input, ~10 GB of scratch: the coded sequences take the
        // worst case per block): one batch per call up to that, and the tails of the two
        // launches (an entropy workgroup holds ~11 items of a 8192-item batch, the last one
        // alone) amortised -- text 36.9 -> 38.0, pxar 37.3 -> 39.1 GiB/s against 8192
        // (profiles/r06/zbatch/)
        return v ? v : (uint64_t)32768;
    }();
    const uint64_t bmax = std::min<uint64_t>(ni, zbatch);
    const unsigned grid_e = (unsigned)std::min<uint64_t>(bmax, 3ull * (uint64_t)use_cu);  // 3 per CU (52 KiB LDS, 168 VGPRs)
    ZItem* z_items = nullptr;
    uint8_t* z_lits = nullptr;
    uint32_t* z_deal = nullptr;   // per batch: the parse and entropy counters, the entropy list's length
    uint32_t* z_elist = nullptr;  // the batch's items left to the entropy kernel
    const uint64_t nbatch = (ni + bmax - 1) / bmax;
    if (compress) {
        z_slots = ar->get<uint8_t>(kZsSlots, ni * kSlot);
        z_seqs = ar->get<Seq>(kZsSeqs, (size_t)grid * kZBlockSeq * sizeof(Seq));
        if (split) {
            z_coded = ar->get<Coded>(kZsCoded, (size_t)bmax * kZBlockSeq * sizeof(Coded));
            z_chains = ar->get<uint32_t>(kZsChains, (size_t)grid_e * 6 * kZBlockSeq * sizeof(uint32_t));
            z_items = ar->get<ZItem>(kZsZItems, (size_t)bmax * sizeof(ZItem));
            z_lits = ar->get<uint8_t>(kZsLits, (size_t)bmax * kEncBlock);
            if (zdeal && (!(z_deal = ar->get<uint32_t>(kZsDeal, (size_t)nbatch * 4 * sizeof(uint32_t))) ||
                          !(z_elist = ar->get<uint32_t>(kZsEList, (size_t)bmax * sizeof(uint32_t)))))
                fail(PBS_ERR_NOMEM);
            if (!z_items || !z_lits) fail(PBS_ERR_NOMEM);
        } else {
            z_coded = ar->get<Coded>(kZsCoded, (size_t)grid * kZBlockSeq * sizeof(Coded));
            z_chains = ar->get<uint32_t>(kZsChains, (size_t)grid * 6 * kZBlockSeq * sizeof(uint32_t));
        }
        if (!z_slots || !z_seqs || !z_coded || !z_chains) fail(PBS_ERR_NOMEM);
    }
    if (!d_bounds || !d_items || !d_first || !d_sizes || !d_ipre || !d_bsz || !d_boff || !d_comp || !d_crc || !d_tmp)
        fail(PBS_ERR_NOMEM);
    hipEvent_t ev[4] = {};
    for (unsigned i = 0; i < 4 && rc == PBS_OK; ++i)
        if (!(ev[i] = ar->event(i))) fail(PBS_ERR_HIP);
    if (rc == PBS_OK)
        ok(hipMemcpyAsync(d_bounds, bounds, 2 * n * 8, hipMemcpyHostToDevice, st)) &&
            ok(hipMemcpyAsync(d_items, items.data(), ni * 8, hipMemcpyHostToDevice, st)) &&
            ok(hipMemcpyAsync(d_first, first.data(), (n + 1) * 8, hipMemcpyHostToDevice, st)) &&
            ok(hipMemsetAsync(d_sizes, 0, (ni + 1) * 8, st)) &&
            (!z_deal || ok(hipMemsetAsync(z_deal, 0, (size_t)nbatch * 4 * sizeof(uint32_t), st)));
    if (rc == PBS_OK) {
        (void)hipGetLastError();
        ok(hipEventRecord(ev[0], st));
        static const bool zprobe = [] {
            const char* e = std::getenv("PBS_ZSTD_PROBE");
            return e && e[0] == '1';
        }();
        static const int64_t dbg_item = [] {
            const char* e = std::getenv("PBS_ZSTD_DEBUG_ITEM");
            return e ? (int64_t)std::strtoll(e, nullptr, 0) : (int64_t)-1;
        }();
        if (compress && zprobe) {
            const unsigned long long z[64] = {};
            (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_zprobe), z, sizeof z, 0, hipMemcpyHostToDevice, st);
        }
        if (compress && split) {
            for (uint64_t b0 = 0; b0 < ni; b0 += bmax) {
                const uint64_t nb = std::min<uint64_t>(bmax, ni - b0);
                uint32_t* const dl = z_deal ? z_deal + 4 * (b0 / bmax) : nullptr;
                hipLaunchKernelGGL(zstd_parse_kernel, dim3((unsigned)std::min<uint64_t>(nb, (uint64_t)grid)),
                                   dim3(kZThreads), 0, st, dev_data, base, d_bounds, d_items + b0, nb, b0,
                                   z_slots + b0 * kSlot, d_sizes + b0, z_seqs, z_coded, z_lits, z_items, dl,
                                   z_elist, zprobe ? 1 : 0, dbg_item);
                hipLaunchKernelGGL(zstd_entropy_kernel, dim3((unsigned)std::min<uint64_t>(nb, (uint64_t)grid_e)),
                                   dim3(kEThreads), 0, st, dev_data, base, d_bounds, d_items + b0, nb,
                                   z_slots + b0 * kSlot, d_sizes + b0, z_coded, z_lits, z_items, z_chains,
                                   dl ? dl + 1 : nullptr, z_elist, zprobe ? 1 : 0);
            }
        } else if (compress) {
            hipLaunchKernelGGL(zstd_block_kernel, dim3(grid), dim3(kZThreads), 0, st, dev_data, base, d_bounds, d_items,
                               ni, z_slots, d_sizes, z_seqs, z_coded, z_chains, zprobe ? 1 : 0, dbg_item);
        }
        if (compress && dbg_item >= 0) {
            static uint32_t h[kZWaves * (1 + 3 * kZSubSeq)];
            (void)hipMemcpyFromSymbolAsync(h, HIP_SYMBOL(g_zdbg), sizeof h, 0, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            if (const char* path = std::getenv("PBS_ZSTD_DEBUG_OUT"))
                if (FILE* f = std::fopen(path, "wb")) {
                    std::fwrite(h, sizeof h, 1, f);
                    std::fclose(f);
                }
        }
        if (compress && zprobe) {
            unsigned long long h[64] = {};
            (void)hipMemcpyFromSymbolAsync(h, HIP_SYMBOL(g_zprobe), sizeof h, 0, hipMemcpyDeviceToHost, st);
            (void)hipStreamSynchronize(st);
            const double nb = h[10] ? (double)h[10] : 1.0;
            std::fprintf(stderr,
                         "zstd probe (workgroup 0, us per block over %llu blocks, %.0f sequences, %.0f literals per "
                         "block): stage %.1f parse %.1f litmap %.1f repcode %.1f sizes %.1f litmode||seqside %.1f decision %.1f "
                         "literals %.1f seqstream %.1f end %.1f | wave 0: history %.1f rounds+walk %.1f | litmap: bitmap %.1f "
                         "sampled %.1f | roles: litmode %.1f repcode %.1f LLtable %.1f LLchain %.1f litsection %.1f | long LL "
                         "chains %llu: pass 1 %.1f rounds %.1f (%.2f rounds) | Huffman: rank %.1f merge %.1f lengths %.1f codes "
                         "%.1f describe %.1f | wave 0 walk %.1f in %.1f rounds | parse by wave %.1f %.1f %.1f %.1f %.1f %.1f %.1f %.1f "
                         "| wave 0 rounds: table %.1f candidates %.1f lengths %.1f pack %.1f records %.1f\n",
                         h[10], h[11] / nb, h[12] / nb, h[0] / nb / 100, h[1] / nb / 100, h[2] / nb / 100,
                         h[3] / nb / 100, h[4] / nb / 100, h[5] / nb / 100, h[6] / nb / 100, h[7] / nb / 100,
                         h[8] / nb / 100, h[9] / nb / 100, h[13] / nb / 100, h[14] / nb / 100, h[15] / nb / 100,
                         h[16] / nb / 100, h[17] / nb / 100, h[18] / nb / 100, h[19] / nb / 100, h[20] / nb / 100,
                         h[21] / nb / 100, h[25], h[25] ? h[22] / (double)h[25] / 100 : 0.0,
                         h[25] ? h[23] / (double)h[25] / 100 : 0.0, h[25] ? h[24] / (double)h[25] : 0.0,
                         h[26] / nb / 100, h[27] / nb / 100, h[28] / nb / 100, h[29] / nb / 100, h[30] / nb / 100,
                         h[32] / nb / 100, h[33] / nb, h[34] / nb / 100, h[35] / nb / 100, h[36] / nb / 100,
                         h[37] / nb / 100, h[38] / nb / 100, h[39] / nb / 100, h[40] / nb / 100, h[41] / nb / 100,
                         h[43] / nb / 100, h[44] / nb / 100, h[45] / nb / 100, h[46] / nb / 100, h[42] / nb / 100);
            if (split) {
                const double ne = h[55] ? (double)h[55] : 1.0;
                std::fprintf(stderr,
                             "zstd probe, entropy kernel (workgroup 0, us per block over %llu blocks): load %.1f roles %.1f "
                             "sizes %.1f decision %.1f literals %.1f seqstream %.1f end %.1f | roles: litmode %.1f LLtable "
                             "%.1f LLchain %.1f litsection %.1f\n",
                             h[55], h[48] / ne / 100, h[49] / ne / 100, h[50] / ne / 100, h[51] / ne / 100,
                             h[52] / ne / 100, h[53] / ne / 100, h[54] / ne / 100, h[17] / ne / 100, h[19] / ne / 100,
                             h[20] / ne / 100, h[21] / ne / 100);
            }
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
                           dim3(kZThreads), 0, st, dev_data, base, d_bounds, d_items, ni, d_first, z_slots,
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
        timing->bytes_in = bytes_in;
        timing->bytes_out = blob_offsets[n];
        timing->blocks = ni;
        if (compressed)
            for (size_t i = 0; i < n; ++i) timing->compressed_chunks += compressed[i];
    }
    if (rc != PBS_OK) (void)hipStreamSynchronize(st);  // the arena goes back idle
    if (timing) timing->total_ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    return rc;
}

extern "C" int pbs_blob_encode_chunks_device(const uint8_t* dev_data, size_t data_len, uint64_t base,
                                             const uint64_t* bounds, size_t n, int compress, uint8_t* blobs_dev,
                                             size_t blobs_cap, uint64_t* blob_offsets, uint32_t* crcs,
                                             uint8_t* compressed, pbs_blob_encode_timing* timing,
                                             void* hip_stream) {
    if (!blob_offsets) return PBS_ERR_INVALID;
    if (n == 0) {
        if (timing) std::memset(timing, 0, sizeof(*timing));
        blob_offsets[0] = 0;
        return PBS_OK;
    }
    if (!bounds) return PBS_ERR_INVALID;
    std::vector<uint64_t> spans(2 * n);
    for (size_t i = 0; i < n; ++i) {
        spans[2 * i] = bounds[i];
        spans[2 * i + 1] = bounds[i + 1];
    }
    return pbs_blob_encode_spans_device(dev_data, data_len, base, spans.data(), n, compress, blobs_dev, blobs_cap,
                                        blob_offsets, crcs, compressed, timing, hip_stream);
}
