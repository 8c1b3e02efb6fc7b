// zstd frame writer primitives (RFC 8878), shared by the GPU block kernel
// (pbs_zstd.hip) and its host twin oracle/zstd_twin.cpp (same parse, same bytes).
//
// The reference compresses every chunk with `zstd::stream::copy_encode(data, .., 1)`
// (pbs-datastore/src/data_blob.rs:151; `bulk::compress(data, 1)` with a crypt config, :99)
// and reads it back with `zstd::stream::decode_all` (:214), which accepts any valid frame.
// The bytes a compressor emits depend on its match finder, so they are not the
// reference's (libzstd 1.5.x level 1): the frames written here are checked by decoding
// them with the image's libzstd (1.4.8) -- "parity unpinned", DESIGN.md section 10.
//
// What is written:
//   frame   magic FD2FB528, single-segment frame header with the content size (no window
//           descriptor, no checksum, no dictionary), then the blocks;
//   blocks  64 KiB of the chunk each (the last shorter): RLE when every byte is equal,
//           compressed when that is shorter than the bytes, else raw;
//   compressed block = raw literals section + sequences with the PREDEFINED FSE tables
//           for literal lengths, match lengths and offsets (symbol compression modes 0),
//           offsets as offset + 3 (no repeat-offset codes).
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
constexpr uint32_t kEncBlock = 64u * 1024u;   // the blocks this encoder writes (LDS-resident)
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

PBS_HD inline uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

PBS_HD inline uint32_t ll_code(uint32_t ll) {
    if (ll < 16) return ll;
    if (ll >= 64) return highbit(ll) + 19;
    uint32_t c = 16;
    while (c < 24 && kLLBase[c + 1] <= ll) ++c;
    return c;
}

PBS_HD inline uint32_t ml_code(uint32_t ml) {  // ml >= 3
    const uint32_t b = ml - 3;
    if (b < 32) return b;
    if (b >= 128) return highbit(b) + 36;
    uint32_t c = 32;
    while (c < 42 && kMLBase[c + 1] <= ml) ++c;
    return c;
}

// FSE compression table (the tANS encoder of RFC 8878 section 4.1 run forwards): `next`
// holds the table's states sorted by symbol, per symbol deltaNbBits / deltaFindState.
struct FseCTable {
    uint16_t next[64];
    int32_t dnb[53];
    int32_t dfs[53];
    uint32_t log;
};

// Build from a normalized distribution (host; the three predefined tables are built once).
inline void build_ctable(FseCTable& t, const int16_t* norm, int nsym, int log) {
    const int size = 1 << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    int high = size - 1;
    uint8_t sym_at[64];
    int cumul[54];
    cumul[0] = 0;
    for (int s = 0; s < nsym; ++s) {
        if (norm[s] == -1) {  // "less than 1" symbols take the last cells
            cumul[s + 1] = cumul[s] + 1;
            sym_at[high--] = (uint8_t)s;
        } else {
            cumul[s + 1] = cumul[s] + norm[s];
        }
    }
    int pos = 0;
    for (int s = 0; s < nsym; ++s)
        for (int k = 0; k < norm[s]; ++k) {
            sym_at[pos] = (uint8_t)s;
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    int cum[54];
    for (int s = 0; s <= nsym; ++s) cum[s] = cumul[s];
    for (int u = 0; u < size; ++u) t.next[cum[sym_at[u]]++] = (uint16_t)(size + u);
    int total = 0;
    for (int s = 0; s < nsym; ++s) {
        const int n = norm[s];
        if (n == 0) {
            t.dnb[s] = ((log + 1) << 16) - size;
            t.dfs[s] = 0;
        } else if (n == -1 || n == 1) {
            t.dnb[s] = (log << 16) - size;
            t.dfs[s] = total - 1;
            ++total;
        } else {
            const int maxbits = log - (int)highbit((uint32_t)(n - 1));
            const int minstate = n << maxbits;
            t.dnb[s] = (maxbits << 16) - minstate;
            t.dfs[s] = total - n;
            total += n;
        }
    }
    t.log = (uint32_t)log;
}

// Backward bit stream of RFC 8878 4.1 as the encoder writes it: bits are appended at the
// low end of a 64-bit container and whole bytes are flushed little-endian; `p` needs 8
// bytes of slack after the last byte written.
struct BitW {
    uint64_t c;
    uint32_t n;
    uint8_t* p;
    uint8_t* start;
    PBS_HD void init(uint8_t* dst) {
        c = 0;
        n = 0;
        p = start = dst;
    }
    PBS_HD void add(uint64_t v, uint32_t nb) {
        c |= (v & ((1ull << nb) - 1ull)) << n;  // nb <= 31 here
        n += nb;
    }
    PBS_HD void flush() {
        const uint32_t nbytes = n >> 3;
        for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(c >> (8 * i));
        p += nbytes;
        n &= 7;
        c = nbytes == 8 ? 0 : c >> (8 * nbytes);
    }
    PBS_HD size_t close() {
        add(1, 1);  // end mark
        flush();
        return (size_t)(p - start) + (n > 0);
    }
};

struct FseState {
    uint32_t v;
    PBS_HD void init(const FseCTable& t, uint32_t sym) {
        const uint32_t nb = (uint32_t)((t.dnb[sym] + (1 << 15)) >> 16);
        const uint32_t v0 = (nb << 16) - (uint32_t)t.dnb[sym];
        v = t.next[(v0 >> nb) + t.dfs[sym]];
    }
    PBS_HD void encode(BitW& b, const FseCTable& t, uint32_t sym) {
        const uint32_t nb = (v + (uint32_t)t.dnb[sym]) >> 16;
        b.add(v, nb);
        v = t.next[(v >> nb) + t.dfs[sym]];
    }
    PBS_HD void flush(BitW& b, const FseCTable& t) {
        b.add(v, t.log);
        b.flush();
    }
};

struct Seq {
    uint32_t ll, ml, off;  // literals before the match, match length (>= 4), offset (>= 1)
};

// Sequences section (RFC 8878 3.1.1.3.2): count, modes byte (predefined x3), bit stream.
// Returns bytes written at dst (needs 8 bytes of slack), or SIZE_MAX as soon as the
// stream passes `limit` (the block would not be shorter than its bytes: stored raw).
PBS_HD inline size_t write_sequences(uint8_t* dst, const Seq* s, uint32_t ns, const FseCTable& tll,
                                     const FseCTable& tml, const FseCTable& tof, const uint8_t* limit) {
    uint8_t* o = dst;
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
    if (ns == 0) return (size_t)(o - dst);
    *o++ = 0;  // LL, OF, ML: predefined mode
    BitW b;
    b.init(o);
    // the last sequence first: its codes seed the three states
    {
        const Seq& q = s[ns - 1];
        const uint32_t llc = ll_code(q.ll), mlc = ml_code(q.ml), ofv = q.off + 3, ofc = highbit(ofv);
        FseState sll, sml, sof;
        sml.init(tml, mlc);
        sof.init(tof, ofc);
        sll.init(tll, llc);
        b.add(q.ll - kLLBase[llc], kLLBits[llc]);
        b.add(q.ml - kMLBase[mlc], kMLBits[mlc]);
        b.add(ofv - (1u << ofc), ofc);
        b.flush();
        Seq nx = ns >= 2 ? s[ns - 2] : Seq{0, 0, 0};  // one sequence ahead (hides the load)
        for (uint32_t k = ns - 1; k-- > 0;) {
            const Seq x = nx;
            if (k) nx = s[k - 1];
            const uint32_t lc = ll_code(x.ll), mc = ml_code(x.ml), ov = x.off + 3, oc = highbit(ov);
            sof.encode(b, tof, oc);
            sml.encode(b, tml, mc);
            sll.encode(b, tll, lc);
            b.flush();
            b.add(x.ll - kLLBase[lc], kLLBits[lc]);
            b.add(x.ml - kMLBase[mc], kMLBits[mc]);
            b.flush();
            b.add(ov - (1u << oc), oc);
            b.flush();
            if (b.p > limit) return SIZE_MAX;
        }
        sml.flush(b, tml);
        sof.flush(b, tof);
        sll.flush(b, tll);
    }
    return (size_t)(o - dst) + b.close();
}

// Raw literals section header (RFC 8878 3.1.1.3.1.1, Literals_Block_Type 0).
PBS_HD inline size_t write_raw_literals_header(uint8_t* o, uint32_t n) {
    if (n < 32) {
        o[0] = (uint8_t)(n << 3);
        return 1;
    }
    if (n < 4096) {
        o[0] = (uint8_t)(1u << 2 | (n << 4));
        o[1] = (uint8_t)(n >> 4);
        return 2;
    }
    o[0] = (uint8_t)(3u << 2 | (n << 4));
    o[1] = (uint8_t)(n >> 4);
    o[2] = (uint8_t)(n >> 12);
    return 3;
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
