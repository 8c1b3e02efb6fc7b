// zstd format constants and frame-level helpers (RFC 8878) for the GPU blob encoder
// (pbs_zstd.hip).  The block encoder itself -- parse, Huffman literals, FSE sequence
// tables, repeat-offset codes -- lives in pbs_zstd.hip; its serial host restatement is
// oracle/zstd_twin.cpp (test infrastructure, written separately from these sources).
//
// The reference compresses every chunk with `zstd::stream::copy_encode(data, .., 1)`
// (pbs-datastore/src/data_blob.rs:151; `bulk::compress(data, 1)` with a crypt config, :99)
// and reads it back with `zstd::stream::decode_all` (:214), which accepts any valid frame.
// The bytes a compressor emits depend on its match finder, so they are not the
// reference's (libzstd 1.5.x level 1): the frames written here are checked by decoding
// them with the image's libzstd (1.4.8) -- "parity unpinned", DESIGN.md section 10.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define PBS_HD __host__ __device__
#else
#define PBS_HD
#endif

namespace pbs {
namespace zstd {

constexpr uint32_t kMagic = 0xFD2FB528u;
constexpr uint32_t kBlockMax = 128u * 1024u;  // the format's largest block
constexpr uint32_t kEncBlock = 64u * 1024u;   // the blocks this encoder writes
constexpr uint32_t kFrameHeaderMax = 4 + 1 + 8;  // magic, descriptor, content size

// RFC 8878 3.1.1.3.2.1: literal-length and match-length codes (baseline, extra bits)
constexpr uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,    9,     10,    11,
                                  12, 13, 14, 15, 16, 18, 20, 22, 24,   28,    32,    40,
                                  48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
constexpr uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  1,  1,
                                 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  12,  13,   14,   15,   16,
                                  17, 18, 19, 20, 21, 22, 23, 24, 25,  26,  27,   28,   29,   30,
                                  31, 32, 33, 34, 35, 37, 39, 41, 43,  47,  51,   59,   67,   83,
                                  99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
constexpr uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// RFC 8878 3.1.1.3.2.2: predefined distributions
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
constexpr int kLLLog = 6, kMLLog = 6, kOFLog = 5;
constexpr int kLLMaxLog = 9, kMLMaxLog = 9, kOFMaxLog = 8;  // FSE_Compressed_Mode limits

PBS_HD inline uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// The code tables as arithmetic (no table loads: on the GPU an indexed constant table is a
// vector memory load per lookup, and the code search a dependent chain of them).  Equal to
// kLLBase / kLLBits / kMLBase / kMLBits and to the table searches for every value
// (tests/test_zstd_cpu.py::test_code_functions_match_tables).
PBS_HD inline uint32_t ll_code(uint32_t ll) {
    if (ll < 16) return ll;
    if (ll >= 64) return highbit(ll) + 19;
    if (ll < 24) return 16 + ((ll - 16) >> 1);
    if (ll < 32) return 20 + ((ll - 24) >> 2);
    if (ll < 48) return 22 + ((ll - 32) >> 3);
    return 24;
}

PBS_HD inline uint32_t ml_code(uint32_t ml) {  // ml >= 3
    const uint32_t b = ml - 3;
    if (b < 32) return b;
    if (b >= 128) return highbit(b) + 36;
    if (b < 40) return 32 + ((b - 32) >> 1);
    if (b < 48) return 36 + ((b - 40) >> 2);
    if (b < 64) return 38 + ((b - 48) >> 3);
    if (b < 96) return 40 + ((b - 64) >> 4);
    return 42;
}

PBS_HD inline uint32_t ll_bits(uint32_t c) {
    return c < 16 ? 0u : c < 20 ? 1u : c < 22 ? 2u : c < 24 ? 3u : c == 24 ? 4u : c - 19;
}
PBS_HD inline uint32_t ll_base(uint32_t c) {
    return c < 16 ? c : c < 20 ? 16 + 2 * (c - 16) : c < 22 ? 24 + 4 * (c - 20) : c < 24 ? 32 + 8 * (c - 22)
                                                                                         : c == 24 ? 48u : 1u << (c - 19);
}
PBS_HD inline uint32_t ml_bits(uint32_t c) {
    return c < 32 ? 0u : c < 36 ? 1u : c < 38 ? 2u : c < 40 ? 3u : c < 42 ? 4u : c == 42 ? 5u : c - 36;
}
PBS_HD inline uint32_t ml_base(uint32_t c) {
    return c < 32 ? c + 3
                  : c < 36 ? 35 + 2 * (c - 32)
                           : c < 38 ? 43 + 4 * (c - 36)
                                    : c < 40 ? 51 + 8 * (c - 38)
                                             : c < 42 ? 67 + 16 * (c - 40) : c == 42 ? 99u : (1u << (c - 36)) + 3;
}

// floor(256 * log2(x)) for 1 <= x < 2^17, integer only: the cost unit of every entropy
// decision (identical on the GPU and in the host twin)
PBS_HD inline uint32_t lg256(uint32_t x) {
    const uint32_t e = highbit(x);
    uint64_t m = e <= 16 ? (uint64_t)x << (16 - e) : (uint64_t)x >> (e - 16);  // [2^16, 2^17)
    uint32_t f = 0;
    for (int i = 0; i < 8; ++i) {
        m = (m * m) >> 16;
        f <<= 1;
        if (m >= (1u << 17)) {
            f |= 1;
            m >>= 1;
        }
    }
    return e * 256 + f;
}

// Block header: Last_Block, Block_Type (0 raw, 1 RLE, 2 compressed), Block_Size.
PBS_HD inline void write_block_header(uint8_t* o, bool last, uint32_t type, uint32_t size) {
    const uint32_t h = (last ? 1u : 0u) | (type << 1) | (size << 3);
    o[0] = (uint8_t)h;
    o[1] = (uint8_t)(h >> 8);
    o[2] = (uint8_t)(h >> 16);
}

// Frame header for a chunk of `len` bytes: single segment, content size, no checksum.
PBS_HD inline size_t write_frame_header(uint8_t* o, uint64_t len) {
    o[0] = 0x28;
    o[1] = 0xB5;
    o[2] = 0x2F;
    o[3] = 0xFD;
    if (len < 256) {
        o[4] = 0x20;  // FCS flag 0 (1 byte with single segment), single segment
        o[5] = (uint8_t)len;
        return 6;
    }
    if (len < 65536 + 256) {
        o[4] = 0x60;  // FCS flag 1: 2 bytes, value - 256
        const uint32_t v = (uint32_t)(len - 256);
        o[5] = (uint8_t)v;
        o[6] = (uint8_t)(v >> 8);
        return 7;
    }
    if (len <= 0xFFFFFFFFull) {
        o[4] = 0xA0;  // FCS flag 2: 4 bytes
        for (int i = 0; i < 4; ++i) o[5 + i] = (uint8_t)(len >> (8 * i));
        return 9;
    }
    o[4] = 0xE0;  // FCS flag 3: 8 bytes
    for (int i = 0; i < 8; ++i) o[5 + i] = (uint8_t)(len >> (8 * i));
    return 13;
}

PBS_HD inline uint32_t frame_header_size(uint64_t len) {
    return len < 256 ? 6 : len < 65536 + 256 ? 7 : len <= 0xFFFFFFFFull ? 9 : 13;
}

// Largest frame for a chunk: header + every block raw (3-byte header each; an empty
// chunk is one empty raw block).
PBS_HD inline uint64_t frame_bound(uint64_t len) {
    const uint64_t nb = len ? (len + kEncBlock - 1) / kEncBlock : 1;
    return frame_header_size(len) + len + 3 * nb;
}

}  // namespace zstd
}  // namespace pbs
