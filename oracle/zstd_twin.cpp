// TEST INFRASTRUCTURE ONLY (imported by tests/ and nothing in the product path).
//
// Host twin of the GPU zstd block encoder (proxmox-backup_amd/csrc/pbs_zstd.hip): the
// same round-parallel greedy parse written as plain loops, through the same frame
// writer primitives (csrc/zstd_enc.h), so the GPU's frames can be compared byte for byte
// while libzstd (the image's libzstd.so.1, 1.4.8) checks that every frame decodes to the
// chunk.  The reference's own compressor is libzstd level 1 (data_blob.rs:99, :151),
// whose bytes cannot be reproduced here: parity of the compressed bytes is UNPINNED;
// what is pinned is decode(frame) == chunk and the blob rules of data_blob.rs:139-176.
//
// Parse (per 64 KiB block, in 16 KiB sub-blocks -- one wave each on the GPU -- with their
// own table; positions in rounds of kRound):
//   1. every position p of the round with 4 bytes left looks up h = hash(p) in the
//      sub-block's table, holding per hash 1 + the last position of an EARLIER round;
//   2. then the round's positions are inserted (largest position wins);
//   3. a candidate c matches if 4 bytes agree; its length is the common prefix, capped at
//      kCap while matching and at the sub-block end (the parse extends a chosen capped
//      match to its true end inside the sub-block); the run candidate p - 1 (offset 1)
//      is compared too and the longer match wins (ties: the table's), so a run of equal
//      bytes is one match even inside the round it starts in;
//   4. greedy: from the current position, the first matching position starts a sequence
//      {literals since the last match, length, offset p - c}; parsing resumes after it
//      (each sub-block starts at its first byte; literals carry over sub-block ends);
//   5. a round samples every step-th position: step 1 after a round with a match,
//      doubling up to kMaxStep while rounds find none (incompressible data is crossed
//      8x faster -- the acceleration of zstd's fast strategy, in round units).
#include <stdint.h>

#include <cstring>
#include <vector>

#include "zstd_enc.h"

namespace {

using namespace pbs::zstd;

constexpr uint32_t kRound = 256, kHashLog = 9, kCap = 32, kSub = 16384, kMaxStep = 8;

inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
inline uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

struct Tables {
    FseCTable ll, ml, of;
    Tables() {
        build_ctable(ll, kLLNorm, 36, kLLLog);
        build_ctable(ml, kMLNorm, 53, kMLLog);
        build_ctable(of, kOFNorm, 29, kOFLog);
    }
};
const Tables& tables() {
    static Tables t;
    return t;
}

// One block of n <= 64 KiB bytes at src; writes header + body at out, returns its size.
size_t block(const uint8_t* src, uint32_t n, bool last, uint8_t* out) {
    bool rle = n > 0;
    for (uint32_t i = 1; i < n && rle; ++i) rle = src[i] == src[0];
    if (rle) {
        write_block_header(out, last, 1, n);
        out[3] = src[0];
        return 4;
    }
    std::vector<uint32_t> table(1u << kHashLog), cand(kRound), mlen(kRound);
    std::vector<Seq> seqs;
    std::vector<uint8_t> lits;
    uint32_t lit_start = 0;
    for (uint32_t s0 = 0; s0 < n; s0 += kSub) {  // sub-blocks: one wave each on the GPU
        const uint32_t se = s0 + kSub < n ? s0 + kSub : n;
        std::fill(table.begin(), table.end(), 0u);
        uint32_t cur = s0, step = 1;
        for (uint32_t r0 = s0, rn; r0 < se; r0 = rn) {
            rn = r0 + kRound * step;  // the next round starts where this one's samples end
            // the round's positions: r0 + j * step, j < kRound (step 1 after a match,
            // doubling up to kMaxStep while rounds find none)
            uint32_t pos[kRound];
            uint32_t np = 0;
            for (uint32_t j = 0; j < kRound && r0 + j * step < se; ++j) pos[np++] = r0 + j * step;
            for (uint32_t k = 0; k < np; ++k) {
                const uint32_t p = pos[k];
                cand[k] = p + 4 <= n ? table[hash4(rd32(src + p))] : 0;
            }
            for (uint32_t k = 0; k < np; ++k) {
                const uint32_t p = pos[k];
                if (p + 4 > n) continue;
                uint32_t& t = table[hash4(rd32(src + p))];
                if (p + 1 > t) t = p + 1;
            }
            for (uint32_t k = 0; k < np; ++k) {
                const uint32_t p = pos[k];
                const uint32_t lim = se - p < kCap ? se - p : kCap;
                uint32_t L = 0, R = 0;
                if (cand[k]) {
                    const uint32_t c = cand[k] - 1;
                    while (L < lim && src[c + L] == src[p + L]) ++L;
                }
                if (p > 0)  // the run candidate p - 1 (offset 1); the longer one wins, ties the table's
                    while (R < lim && src[p - 1 + R] == src[p + R]) ++R;
                if (R >= 4 && R > (L >= 4 ? L : 0)) {
                    L = R;
                    cand[k] = p;  // 1 + (p - 1)
                }
                mlen[k] = L >= 4 ? L : 0;
            }
            bool found = false;
            for (uint32_t k = 0; k < np; ++k) {
                const uint32_t p = pos[k];
                if (p < cur || !mlen[k]) continue;
                const uint32_t c = cand[k] - 1;
                uint32_t L = mlen[k];
                if (L == kCap)
                    while (p + L < se && src[c + L] == src[p + L]) ++L;
                seqs.push_back({p - lit_start, L, p - c});
                lits.insert(lits.end(), src + lit_start, src + p);
                cur = p + L;
                lit_start = cur;
                found = true;
            }
            step = found ? 1 : (step * 2 < kMaxStep ? step * 2 : kMaxStep);
        }
    }
    lits.insert(lits.end(), src + lit_start, src + n);
    std::vector<uint8_t> body(3 + (size_t)n + 64);
    size_t o = 3;
    o += write_raw_literals_header(body.data() + o, (uint32_t)lits.size());
    if (!lits.empty()) std::memcpy(body.data() + o, lits.data(), lits.size());
    o += lits.size();
    const Tables& t = tables();
    const size_t sq = o - 3 >= n ? SIZE_MAX
                                 : write_sequences(body.data() + o, seqs.data(), (uint32_t)seqs.size(), t.ll,
                                                   t.ml, t.of, body.data() + 3 + n);
    if (sq == SIZE_MAX || o + sq - 3 >= n) {  // not shorter: raw block
        write_block_header(out, last, 0, n);
        std::memcpy(out + 3, src, n);
        return 3 + (size_t)n;
    }
    o += sq;
    write_block_header(body.data(), last, 2, (uint32_t)(o - 3));
    std::memcpy(out, body.data(), o);
    return o;
}

}  // namespace

extern "C" {

uint64_t zstd_twin_bound(uint64_t len) { return frame_bound(len); }

// The frame of one chunk; returns its size (cap >= zstd_twin_bound(len)).
uint64_t zstd_twin_frame(const uint8_t* src, uint64_t len, uint8_t* out) {
    size_t o = write_frame_header(out, len);
    if (len == 0) {
        write_block_header(out + o, true, 0, 0);
        return o + 3;
    }
    for (uint64_t b = 0; b < len; b += kEncBlock) {
        const uint32_t n = (uint32_t)(len - b < kEncBlock ? len - b : kEncBlock);
        o += block(src + b, n, b + n == len, out + o);
    }
    return o;
}

}  // extern "C"
