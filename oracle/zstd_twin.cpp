// TEST INFRASTRUCTURE ONLY (imported by tests/ and nothing in the product path).
//
// Host twin of the GPU zstd blob encoder (proxmox-backup_amd/csrc/pbs_zstd.hip): the same
// parse and the same entropy-coding decisions written as plain serial loops, with its OWN
// frame writer (nothing is shared with the product's sources: the bit streams, the
// Huffman construction, the FSE normalisation / table description and the repeat-offset
// coding are restated here from RFC 8878), so byte equality with the GPU's frames checks
// the product's parallel bit packing against an independent serial writer.  libzstd (the
// image's libzstd.so.1, 1.4.8) checks that every frame decodes to the chunk.  The
// reference's own compressor is libzstd level 1 (pbs-datastore/src/data_blob.rs:99, :151),
// whose bytes cannot be reproduced here: parity of the compressed bytes is UNPINNED.
//
// Format decisions (every one deterministic, integer-only, mirrored by the GPU):
//   frame    single segment, content size, blocks of kBlock = 64 KiB (last shorter);
//   block    RLE when every byte is equal; else compressed when shorter than raw, else raw;
//   literals raw, RLE (one distinct byte), or Huffman (RFC 8878 4.2): code lengths from a
//            two-queue Huffman merge limited to 11 bits, weights in the direct 4-bit form
//            when at most 128 are transmitted else FSE-compressed (two interleaved states,
//            accuracy <= 6); 1 stream below 256 literals, else 4 streams + jump table;
//            Huffman only when its estimate beats raw -- first on the literals at block
//            positions divisible by 16 (cheap: random literals never build a histogram of
//            all bytes), then on all of them;
//   sequences per stream (LL / OF / ML) the cheapest of predefined, RLE and FSE-compressed
//            (own table, normalised counts), by an integer cost estimate; offsets as
//            repeat codes when they equal a repeat offset set EARLIER IN THE SAME BLOCK
//            (the blocks are encoded independently, so the decoder's repeat offsets at a
//            block start are unknown to the encoder), else offset + 3.
//
// Parse (per 64 KiB block; eight ~8 KiB sub-blocks -- kSubA bytes for the first four,
// kSubB for the last four -- one GPU wave each, own hash table; round 5):
//   history  the kWin bytes before the sub-block enter the table in rounds of kHistRound
//            positions every `hs` bytes (hs >= kHistMinStep; the table keeps 1 + the LAST
//            position per hash of kHashBytes bytes);
//   rounds   of kRound positions sampled every `step` bytes (step 1 after a round in which
//            the walk took a match, doubling to kMaxStep without; a round starts at the end
//            of a match that ran past the previous one, the positions inside it are not
//            searched).  Per position p at or after the walk's position at the round start
//            (`cur`), from state fixed at the round start only: the candidates are (a) the
//            round-start repeat offset (the last match's offset; p - rep), (b) the table
//            (the last position of an EARLIER round with the same hash), (c) the run
//            candidate p - 1; a candidate counts from kMinMatch equal bytes.  The repeat
//            candidate wins when it counts; else the longer of (b) and (c) within kCap (ties:
//            the table's).  Its length is the common prefix capped at kCap (and the sub-block
//            end); for (b) / (c) also how far the match extends backwards (at most kBack
//            bytes, not before the window).
//   walk     from `cur`, the first position with a match is taken: it starts up to its
//            backward extension earlier (never before `cur`), a capped length is extended
//            forwards to the match's end (within the sub-block), and `cur` moves to the
//            match's end.  Nothing the walk does feeds back into the round's per-position
//            data, so the GPU computes that data lane-parallel and walks with scalar steps.
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

constexpr uint32_t kBlock = 64 * 1024;
// one GPU wave's sub-block: the first four 8 KiB + 768 bytes, the last four 8 KiB - 768
constexpr uint32_t kSubA = 8192 + 768, kSubB = 8192 - 768;
constexpr uint32_t sub_start(uint32_t w) { return w <= 4 ? w * kSubA : 4 * kSubA + (w - 4) * kSubB; }
uint32_t sub_of(uint32_t pos) {  // the sub-block holding block position pos
    uint32_t w = 0;
    while (w < 7 && pos >= sub_start(w + 1)) ++w;
    return w;
}
// the window before a sub-block (reaches into the previous block) and the history rounds'
// smallest step: 12 KiB and 2 since round 6 (16 KiB and 1 before; the GPU's kZWin /
// kZHistMinStep, csrc/pbs_zstd.hip)
constexpr uint32_t kWin = 12288, kHistMinStep = 2;
constexpr uint32_t kRound = 256, kMaxStep = 8, kHistRound = 512, kHistMaxStep = 8, kHistStep0 = kHistMinStep;
constexpr uint32_t kHashLog = 12, kCap = 32, kMinMatch = 5, kBack = 8;
constexpr uint32_t kHufStreams = 48 * 1024;  // largest Huffman stream bytes of a block

// ------------------------------------------------------------------------ parse
inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}
// hash of the 5 bytes at p (GPU: one LDS word and one byte)
inline uint32_t hash5(const uint8_t* p) {
    return ((rd32(p) * 2654435761u) ^ (p[4] * 2246822519u)) >> (32 - kHashLog);
}

struct Seq {
    uint32_t pos, ml, off;  // match start (block position), length, offset
};

// common prefix of src[a..] and src[b..] (a < b), at most lim bytes
inline uint32_t prefix(const uint8_t* s, uint32_t a, uint32_t b, uint32_t lim) {
    uint32_t L = 0;
    while (L < lim && s[a + L] == s[b + L]) ++L;
    return L;
}

// src = the block (n bytes); src[-avail .. -1] = the chunk bytes before it
uint64_t g_hist_inserts = 0;
void parse(const uint8_t* src, uint32_t n, uint32_t avail, std::vector<Seq>& seqs) {
    const uint32_t hb = kMinMatch;
    const uint8_t* const b = src - avail;  // positions P = p + avail
    const uint32_t N = avail + n;
    std::vector<uint32_t> table(1u << kHashLog);
    for (uint32_t w = 0; w < 8 && avail + sub_start(w) < N; ++w) {
        const uint32_t s0 = avail + sub_start(w), se = std::min(avail + sub_start(w + 1), N);
        std::fill(table.begin(), table.end(), 0u);
        const uint32_t wlo = s0 - std::min(s0, kWin);  // the sub-block's window start
        // history: the window before the sub-block in rounds of kHistRound positions every
        // `hs` bytes (inserts only; the table keeps the last position per hash); a round's
        // first 64 positions look up their candidates before its inserts, and when one of
        // them matches kMinMatch bytes (not a run of one byte) the next round steps
        // kHistMinStep, else the step doubles up to kHistMaxStep
        uint32_t hs = kHistStep0;
        for (uint32_t r0 = wlo, rn; r0 < s0; r0 = rn) {
            rn = r0 + kHistRound * hs;
            uint32_t cand[64];
            for (uint32_t j = 0; j < 64; ++j) {
                const uint32_t p = r0 + j * hs;
                cand[j] = p < s0 && p + hb <= N ? table[hash5(b + p)] : 0;
            }
            for (uint32_t j = 0; j < kHistRound; ++j) {
                const uint32_t p = r0 + j * hs;
                if (p >= s0) break;
                if (p + hb <= N) {
                    table[hash5(b + p)] = p + 1;
                    ++g_hist_inserts;
                }
            }
            bool hit = false;
            for (uint32_t j = 0; j < 64; ++j) {
                const uint32_t p = r0 + j * hs;
                if (!cand[j]) continue;
                const bool run = rd32(b + p) == b[p] * 0x01010101u && b[p + 4] == b[p];
                hit |= !run && std::memcmp(b + cand[j] - 1, b + p, hb) == 0;
            }
            hs = hit ? kHistMinStep : std::min(2 * hs, kHistMaxStep);
        }
        uint32_t cur = s0, step = std::min(hs, kMaxStep), rep = 0;  // rep 0: no offset in this sub-block yet
        for (uint32_t r0 = s0, rn; r0 < se; r0 = rn) {
            rn = r0 + kRound * step;
            uint32_t pos[kRound], cand[kRound], len[kRound], msrc[kRound], back[kRound], np = 0;
            for (uint32_t j = 0; j < kRound && r0 + j * step < se; ++j) pos[np++] = r0 + j * step;
            for (uint32_t k = 0; k < np; ++k) cand[k] = pos[k] + hb <= N ? table[hash5(b + pos[k])] : 0;
            for (uint32_t k = 0; k < np; ++k) {
                const uint32_t p = pos[k];
                if (p + hb > N) continue;
                uint32_t& t = table[hash5(b + p)];
                if (p + 1 > t) t = p + 1;
            }
            // per position, from the round-start state (cur, rep) only
            for (uint32_t k = 0; k < np; ++k) {
                const uint32_t p = pos[k];
                len[k] = 0;
                if (p < cur || p + hb > se) continue;
                const uint32_t lim = std::min(se - p, kCap);
                const bool mrep = rep && p >= wlo + rep && std::memcmp(b + p - rep, b + p, hb) == 0;
                const bool mt = cand[k] && std::memcmp(b + cand[k] - 1, b + p, hb) == 0;
                const bool mr = p > wlo && std::memcmp(b + p - 1, b + p, hb) == 0;
                uint32_t s = 0, L = 0;
                if (mrep) {
                    s = p - rep;
                } else if (mt && mr) {
                    const uint32_t Lt = prefix(b, cand[k] - 1, p, lim), Lr = prefix(b, p - 1, p, lim);
                    s = Lr > Lt ? p - 1 : cand[k] - 1;
                } else if (mt) {
                    s = cand[k] - 1;
                } else if (mr) {
                    s = p - 1;
                } else {
                    continue;
                }
                L = prefix(b, s, p, lim);
                uint32_t e = 0;  // backwards (table and run candidates)
                if (!mrep)
                    while (e < kBack && s - e > wlo && b[p - 1 - e] == b[s - 1 - e]) ++e;
                len[k] = L;
                msrc[k] = s;
                back[k] = e;
            }
            // the walk
            bool found = false;
            for (uint32_t k = 0; k < np; ++k) {
                if (pos[k] < cur || !len[k]) continue;
                const uint32_t p = pos[k], e = std::min(back[k], p - cur);
                const uint32_t mpos = p - e, ms = msrc[k] - e;
                uint32_t mlen = len[k] + e;
                if (len[k] == kCap)  // to its true end (a shorter length already stopped there)
                    while (mpos + mlen < se && b[ms + mlen] == b[mpos + mlen]) ++mlen;
                seqs.push_back({mpos - avail, mlen, mpos - ms});
                rep = mpos - ms;
                cur = mpos + mlen;
                found = true;
            }
            step = found ? 1 : std::min(step * 2, kMaxStep);
            if (cur > rn) rn = cur;  // positions inside a match that ran past the round: not searched
        }
    }
}

// ------------------------------------------------------------------------ bits
// Forward-written bit stream (RFC 8878 4.1: the decoder reads it backwards from the end
// mark): fields are appended at increasing bit positions, bytes emitted little-endian.
struct Bits {
    std::vector<uint8_t> b;
    uint64_t acc = 0;
    uint32_t n = 0;
    void put(uint64_t v, uint32_t nb) {
        if (nb == 0) return;
        acc |= (v & ((1ull << nb) - 1)) << n;
        n += nb;
        while (n >= 8) {
            b.push_back((uint8_t)acc);
            acc >>= 8;
            n -= 8;
        }
    }
    void close() {  // end mark, then the partial byte
        put(1, 1);
        if (n) b.push_back((uint8_t)acc);
        acc = 0;
        n = 0;
    }
};

// floor(256 * log2(x)), x >= 1, integer only (repeated squaring of the mantissa)
uint32_t lg256(uint32_t x) {
    uint32_t e = 31 - (uint32_t)__builtin_clz(x);
    uint64_t m = (uint64_t)x << (16 - e);  // in [2^16, 2^17) for x < 2^16
    if (e > 16) m = (uint64_t)x >> (e - 16);
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

uint32_t highbit(uint32_t v) { return 31 - (uint32_t)__builtin_clz(v); }

// ------------------------------------------------------------------------ FSE
constexpr int kMaxFseLog = 9;
struct Fse {
    int log = 0;
    uint16_t next[1 << kMaxFseLog];
    int32_t dnb[256];
    int32_t dfs[256];
};

// RFC 8878 4.1.1 table construction: "less than 1" (-1) symbols from the top cell down,
// the others spread with step (size >> 1) + (size >> 3) + 3; then the encoder's view
void fse_build(Fse& t, const int16_t* norm, int nsym, int log) {
    const int size = 1 << log, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    int high = size - 1;
    std::vector<uint8_t> sym_at(size);
    std::vector<int> cum(nsym + 1);
    cum[0] = 0;
    for (int s = 0; s < nsym; ++s) {
        if (norm[s] == -1) {
            cum[s + 1] = cum[s] + 1;
            sym_at[high--] = (uint8_t)s;
        } else {
            cum[s + 1] = cum[s] + norm[s];
        }
    }
    int pos = 0;
    for (int s = 0; s < nsym; ++s)
        for (int k = 0; k < norm[s]; ++k) {
            sym_at[pos] = (uint8_t)s;
            do pos = (pos + step) & mask;
            while (pos > high);
        }
    std::vector<int> c2(cum);
    for (int u = 0; u < size; ++u) t.next[c2[sym_at[u]]++] = (uint16_t)(size + u);
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

struct FseSt {
    uint32_t v;
    void init(const Fse& t, uint32_t s) {
        const uint32_t nb = (uint32_t)((t.dnb[s] + (1 << 15)) >> 16);
        const uint32_t v0 = (nb << 16) - (uint32_t)t.dnb[s];
        v = t.next[(v0 >> nb) + t.dfs[s]];
    }
    void enc(Bits& b, const Fse& t, uint32_t s) {
        const uint32_t nb = (v + (uint32_t)t.dnb[s]) >> 16;
        b.put(v, nb);
        v = t.next[(v >> nb) + t.dfs[s]];
    }
    void flush(Bits& b, const Fse& t) { b.put(v, (uint32_t)t.log); }
};

// zstd's table-log rule (FSE_optimalTableLog with minus = 2), clamped to [5, max_log]
int fse_log(uint32_t total, uint32_t max_sym, int max_log) {
    int log = max_log;
    const int src = (int)highbit(total - 1) - 2;
    const int minb = (int)std::min(highbit(total) + 1, highbit(max_sym) + 2);
    if (src < log) log = src;
    if (minb > log) log = minb;
    return std::max(5, std::min(log, max_log));
}

// Counts -> normalised counts summing to 2^log: every present symbol >= 1, the others
// round(count * 2^log / total); the difference goes to (or comes from) the largest.
void fse_normalize(int16_t* norm, const uint32_t* cnt, int nsym, uint32_t total, int log) {
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
        int big = -1;  // the largest normalised count (lowest symbol on ties)
        for (int s = 0; s < nsym; ++s)
            if (norm[s] > 0 && (big < 0 || norm[s] > norm[big])) big = s;
        if (sum < scale) {
            norm[big] = (int16_t)(norm[big] + (scale - sum));
            sum = scale;
        } else {
            const int64_t take = std::min<int64_t>(sum - scale, norm[big] - 1);
            norm[big] = (int16_t)(norm[big] - take);
            sum -= take;
        }
    }
}

// RFC 8878 4.1.1 table description (the variable-length counts, zero-run flags)
void fse_write_ncount(std::vector<uint8_t>& o, const int16_t* norm, int nsym, int log) {
    const int size = 1 << log;
    uint64_t bs = (uint64_t)(log - 5);
    int nb = 4;
    auto out = [&]() {
        while (nb >= 8) {
            o.push_back((uint8_t)bs);
            bs >>= 8;
            nb -= 8;
        }
    };
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
                out();
            }
            while (s >= start + 3) {
                start += 3;
                bs |= 3ull << nb;
                nb += 2;
            }
            bs |= (uint64_t)(s - start) << nb;
            nb += 2;
            out();
        }
        int count = norm[s++];
        const int max = (2 * threshold - 1) - remaining;
        remaining -= count < 0 ? -count : count;
        ++count;
        if (count >= threshold) count += max;
        bs |= (uint64_t)count << nb;
        nb += nbits;
        nb -= count < max;
        prev0 = count == 1;
        while (remaining < threshold) {
            --nbits;
            threshold >>= 1;
        }
        out();
    }
    while (nb > 0) {
        o.push_back((uint8_t)bs);
        bs >>= 8;
        nb -= 8;
    }
}

// ------------------------------------------------------------------------ Huffman
constexpr uint32_t kHufMax = 11;

// Code lengths (0 = absent): two-queue Huffman merge over the symbols sorted by (count,
// symbol), ties taking the leaf; lengths over kHufMax are cut to it and the Kraft excess
// paid back by lengthening the longest codes below the limit (least frequent first), a
// deficit filled by shortening codes (most frequent first).
void huf_lengths(const uint32_t* cnt, uint8_t* len) {
    std::vector<int> sym;
    for (int s = 0; s < 256; ++s) {
        len[s] = 0;
        if (cnt[s]) sym.push_back(s);
    }
    std::stable_sort(sym.begin(), sym.end(), [&](int a, int b) { return cnt[a] < cnt[b]; });
    const int m = (int)sym.size();
    // nodes 0..m-1 leaves (sorted), m.. internal in creation order
    std::vector<uint64_t> w(2 * m);
    std::vector<int> parent(2 * m, -1);
    for (int i = 0; i < m; ++i) w[i] = cnt[sym[i]];
    int li = 0, ii = m, nn = m;
    auto pick = [&]() {
        if (li < m && (ii >= nn || w[li] <= w[ii])) return li++;
        return ii++;
    };
    while (nn < 2 * m - 1) {
        const int a = pick(), b = pick();
        w[nn] = w[a] + w[b];
        parent[a] = parent[b] = nn;
        ++nn;
    }
    std::vector<uint32_t> depth(2 * m, 0);
    for (int i = nn - 2; i >= 0; --i) depth[i] = depth[parent[i]] + 1;
    for (int i = 0; i < m; ++i) len[sym[i]] = (uint8_t)depth[i];
    // limit
    int64_t k = -(1ll << kHufMax);
    for (int i = 0; i < m; ++i) {
        uint8_t& L = len[sym[i]];
        if (L > kHufMax) L = kHufMax;
        k += 1ll << (kHufMax - L);
    }
    while (k > 0) {  // lengthen: the longest code under the limit, least frequent first
        int best = -1;
        for (int i = 0; i < m; ++i) {
            const uint8_t L = len[sym[i]];
            if (L < kHufMax && (best < 0 || L > len[sym[best]])) best = i;
        }
        uint8_t& L = len[sym[best]];
        k -= 1ll << (kHufMax - L - 1);
        ++L;
    }
    while (k < 0) {  // shorten: most frequent first, while the deficit allows
        for (int i = m - 1; i >= 0 && k < 0; --i) {
            uint8_t& L = len[sym[i]];
            while (L > 1 && (1ll << (kHufMax - L)) <= -k) {
                k += 1ll << (kHufMax - L);
                --L;
            }
        }
    }
}

struct Huf {
    uint8_t len[256];
    uint16_t code[256];
    uint32_t max_bits;
    int last;  // highest symbol present
};

void huf_codes(Huf& h) {
    h.max_bits = 0;
    h.last = -1;
    for (int s = 0; s < 256; ++s)
        if (h.len[s]) {
            h.max_bits = std::max<uint32_t>(h.max_bits, h.len[s]);
            h.last = s;
        }
    // canonical: by (length descending, symbol ascending), codes increasing
    uint32_t code = 0, prev = 0;
    bool first = true;
    for (uint32_t L = h.max_bits; L >= 1; --L)
        for (int s = 0; s < 256; ++s) {
            if (h.len[s] != L) continue;
            if (!first) code = (code + 1) >> (prev - L);
            h.code[s] = (uint16_t)code;
            prev = L;
            first = false;
        }
}

// Huffman tree description (RFC 8878 4.2.1): weights of symbols 0..last-1 (the last one
// implied); direct 4-bit form when it is the only option or shorter.  Returns false when
// no form applies (the caller writes raw literals).
bool huf_describe(const Huf& h, std::vector<uint8_t>& o) {
    const int nw = h.last;  // weights transmitted
    std::vector<uint8_t> wt(nw);
    for (int s = 0; s < nw; ++s) wt[s] = h.len[s] ? (uint8_t)(h.max_bits + 1 - h.len[s]) : 0;
    std::vector<uint8_t> fse;
    bool fse_ok = false;
    if (nw > 2) {
        uint32_t cnt[16] = {0};
        uint32_t maxw = 0;
        for (int s = 0; s < nw; ++s) {
            ++cnt[wt[s]];
            maxw = std::max<uint32_t>(maxw, wt[s]);
        }
        bool single = false;
        for (int v = 0; v < 16; ++v) single |= cnt[v] == (uint32_t)nw;
        if (!single) {
            const int log = fse_log((uint32_t)nw, maxw, 6);
            int16_t norm[16];
            fse_normalize(norm, cnt, (int)maxw + 1, (uint32_t)nw, log);
            fse_write_ncount(fse, norm, (int)maxw + 1, log);
            Fse t;
            fse_build(t, norm, (int)maxw + 1, log);
            Bits b;
            FseSt s1, s2;  // s1 codes the even indices, s2 the odd ones (decoded first: s1)
            int i = nw;
            if (nw & 1) {
                s1.init(t, wt[--i]);
                s2.init(t, wt[--i]);
                s1.enc(b, t, wt[--i]);
            } else {
                s2.init(t, wt[--i]);
                s1.init(t, wt[--i]);
            }
            while (i > 0) {
                s2.enc(b, t, wt[--i]);
                s1.enc(b, t, wt[--i]);
            }
            s2.flush(b, t);
            s1.flush(b, t);
            b.close();
            fse.insert(fse.end(), b.b.begin(), b.b.end());
            fse_ok = fse.size() < 128;
        }
    }
    const size_t direct = nw <= 128 ? 1 + (size_t)(nw + 1) / 2 : SIZE_MAX;
    if (fse_ok && fse.size() + 1 < direct) {
        o.push_back((uint8_t)fse.size());
        o.insert(o.end(), fse.begin(), fse.end());
        return true;
    }
    if (direct == SIZE_MAX) return false;
    o.push_back((uint8_t)(127 + nw));
    for (int s = 0; s < nw; s += 2) o.push_back((uint8_t)(wt[s] << 4 | (s + 1 < nw ? wt[s + 1] : 0)));
    return true;
}

void huf_stream(const Huf& h, const uint8_t* lit, uint32_t n, std::vector<uint8_t>& o) {
    Bits b;
    for (uint32_t i = n; i-- > 0;) b.put(h.code[lit[i]], h.len[lit[i]]);
    b.close();
    o.insert(o.end(), b.b.begin(), b.b.end());
}

// Literals section (RFC 8878 3.1.1.3.1)
void raw_literals(std::vector<uint8_t>& o, const uint8_t* lit, uint32_t n, uint32_t type) {
    const uint32_t t = type;  // 0 raw, 1 RLE
    if (n < 32) {
        o.push_back((uint8_t)(t | n << 3));
    } else if (n < 4096) {
        o.push_back((uint8_t)(t | 1u << 2 | n << 4));
        o.push_back((uint8_t)(n >> 4));
    } else {
        o.push_back((uint8_t)(t | 3u << 2 | n << 4));
        o.push_back((uint8_t)(n >> 4));
        o.push_back((uint8_t)(n >> 12));
    }
    if (type == 0)
        o.insert(o.end(), lit, lit + n);
    else
        o.push_back(lit[0]);
}

// samp = the literal bytes at block positions divisible by 16 (a first, cheap estimate)
void literals(std::vector<uint8_t>& o, const std::vector<uint8_t>& lit, const std::vector<uint8_t>& samp) {
    const uint32_t n = (uint32_t)lit.size();
    if (n >= 32 && !samp.empty()) {  // sampled estimate: clearly incompressible literals stay raw
        uint32_t cs[256] = {0};
        for (uint8_t c : samp) ++cs[c];
        const uint32_t m = (uint32_t)samp.size(), lm = lg256(m);
        uint64_t es = 0;
        for (int s = 0; s < 256; ++s)
            if (cs[s]) es += (uint64_t)cs[s] * (lm - lg256(cs[s]));
        if (es * n / m / 2048 + 64 >= (uint64_t)n - n / 64) {
            raw_literals(o, lit.data(), n, 0);
            return;
        }
    }
    uint32_t cnt[256] = {0};
    for (uint8_t c : lit) ++cnt[c];
    int distinct = 0;
    for (int s = 0; s < 256; ++s) distinct += cnt[s] != 0;
    if (n > 0 && distinct == 1) {
        raw_literals(o, lit.data(), n, 1);
        return;
    }
    if (n < 32) {
        raw_literals(o, lit.data(), n, 0);
        return;
    }
    // entropy estimate (1/256 bits): Huffman only when it may save > 1/64 of the bytes
    uint64_t est = 0;
    const uint32_t ln = lg256(n);
    for (int s = 0; s < 256; ++s)
        if (cnt[s]) est += (uint64_t)cnt[s] * (ln - lg256(cnt[s]));
    if (est / 2048 + 64 >= (uint64_t)n - n / 64) {
        raw_literals(o, lit.data(), n, 0);
        return;
    }
    Huf h;
    huf_lengths(cnt, h.len);
    huf_codes(h);
    std::vector<uint8_t> body;
    if (!huf_describe(h, body)) {
        raw_literals(o, lit.data(), n, 0);
        return;
    }
    const bool four = n >= 256;
    const size_t desc = body.size();
    if (!four) {
        huf_stream(h, lit.data(), n, body);
    } else {
        const uint32_t seg = (n + 3) / 4;
        std::vector<uint8_t> st[4];
        for (int k = 0; k < 4; ++k) {
            const uint32_t a = seg * k, e = std::min(n, seg * (k + 1));
            huf_stream(h, lit.data() + a, e - a, st[k]);
        }
        for (int k = 0; k < 3; ++k) {
            body.push_back((uint8_t)st[k].size());
            body.push_back((uint8_t)(st[k].size() >> 8));
        }
        for (int k = 0; k < 4; ++k) body.insert(body.end(), st[k].begin(), st[k].end());
    }
    const uint32_t c = (uint32_t)body.size();
    // the GPU stages the streams in 48 KiB of LDS: longer ones are written raw
    if (c - desc - (four ? 6 : 0) > kHufStreams) {
        raw_literals(o, lit.data(), n, 0);
        return;
    }
    // header: type 2, size format 0 (1 stream, 10+10 bits), 1 (4 streams, 10+10), 2 (14+14),
    // 3 (18+18)
    const uint32_t mx = std::max(n, c);
    const uint32_t hs = mx < 1024 ? 3 : mx < 16384 ? 4 : 5;
    if (hs + c >= (n < 32 ? 1u : n < 4096 ? 2u : 3u) + n) {  // not shorter than raw
        raw_literals(o, lit.data(), n, 0);
        return;
    }
    if (hs == 3) {
        const uint32_t v = 2u | (four ? 1u : 0u) << 2 | n << 4 | c << 14;
        o.push_back((uint8_t)v);
        o.push_back((uint8_t)(v >> 8));
        o.push_back((uint8_t)(v >> 16));
    } else if (hs == 4) {
        const uint32_t v = 2u | 2u << 2 | n << 4 | c << 18;
        for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(v >> (8 * i)));
    } else {
        const uint64_t v = 2u | 3u << 2 | (uint64_t)n << 4 | (uint64_t)c << 22;
        for (int i = 0; i < 5; ++i) o.push_back((uint8_t)(v >> (8 * i)));
    }
    o.insert(o.end(), body.begin(), body.end());
}

// ------------------------------------------------------------------------ sequences
const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,   16,   18,
                              20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  1,  1,
                             1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,  16,  17,  18,   19,   20,
                              21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33,  34,  35,  37,   39,   41,
                              43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                             0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                             2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
const int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                             1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
const int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                             1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

uint32_t ll_code(uint32_t v) {
    if (v < 16) return v;
    if (v >= 64) return highbit(v) + 19;
    uint32_t c = 16;
    while (kLLBase[c + 1] <= v) ++c;
    return c;
}
uint32_t ml_code(uint32_t ml) {
    const uint32_t b = ml - 3;
    if (b < 32) return b;
    if (b >= 128) return highbit(b) + 36;
    uint32_t c = 32;
    while (kMLBase[c + 1] <= ml) ++c;
    return c;
}

struct Coded {
    uint32_t ll, ml, ofv;  // literal length, match length, offset value (repeat code 1-3 or offset + 3)
    uint8_t llc, mlc, ofc;
};

// one symbol stream's table: mode 0 predefined, 1 RLE, 2 FSE-compressed (cheapest by the
// integer estimate; ties keep the earlier mode)
struct SeqTab {
    int mode;
    uint8_t rle;
    Fse t;
    std::vector<uint8_t> desc;
};

void seq_table(SeqTab& st, const uint32_t* cnt, int nsym, uint32_t nseq, const int16_t* pre, int pre_log,
               int max_log) {
    int distinct = 0, maxs = 0;
    for (int s = 0; s < nsym; ++s)
        if (cnt[s]) {
            ++distinct;
            maxs = s;
        }
    uint64_t c_pre = 0;
    for (int s = 0; s < nsym; ++s)
        if (cnt[s]) c_pre += (uint64_t)cnt[s] * (256u * pre_log - lg256(pre[s] < 1 ? 1 : pre[s]));
    st.mode = 0;
    st.desc.clear();
    if (distinct == 1 && nseq > 2) {
        st.mode = 1;
        st.rle = (uint8_t)maxs;
        st.desc.push_back((uint8_t)maxs);
        return;
    }
    if (nseq >= 16) {
        const int log = fse_log(nseq, (uint32_t)maxs, max_log);
        int16_t norm[64];
        fse_normalize(norm, cnt, maxs + 1, nseq, log);
        std::vector<uint8_t> d;
        fse_write_ncount(d, norm, maxs + 1, log);
        uint64_t c = 2048ull * d.size();
        for (int s = 0; s <= maxs; ++s)
            if (cnt[s]) c += (uint64_t)cnt[s] * (256u * log - lg256(norm[s]));
        if (c < c_pre) {
            st.mode = 2;
            st.desc = d;
            fse_build(st.t, norm, maxs + 1, log);
            return;
        }
    }
    fse_build(st.t, pre, nsym, pre_log);
}

void sequences(std::vector<uint8_t>& o, const std::vector<Coded>& q) {
    const uint32_t ns = (uint32_t)q.size();
    if (ns < 128) {
        o.push_back((uint8_t)ns);
    } else if (ns < 0x7F00) {
        o.push_back((uint8_t)((ns >> 8) + 0x80));
        o.push_back((uint8_t)ns);
    } else {
        o.push_back(0xFF);
        o.push_back((uint8_t)(ns - 0x7F00));
        o.push_back((uint8_t)((ns - 0x7F00) >> 8));
    }
    if (ns == 0) return;
    uint32_t cl[36] = {0}, cm[53] = {0}, co[32] = {0};
    for (const Coded& c : q) {
        ++cl[c.llc];
        ++cm[c.mlc];
        ++co[c.ofc];
    }
    SeqTab tl, tm, to;
    seq_table(tl, cl, 36, ns, kLLNorm, 6, 9);
    seq_table(to, co, 29, ns, kOFNorm, 5, 8);
    seq_table(tm, cm, 53, ns, kMLNorm, 6, 9);
    o.push_back((uint8_t)(tl.mode << 6 | to.mode << 4 | tm.mode << 2));
    o.insert(o.end(), tl.desc.begin(), tl.desc.end());
    o.insert(o.end(), to.desc.begin(), to.desc.end());
    o.insert(o.end(), tm.desc.begin(), tm.desc.end());
    Bits b;
    FseSt sl{}, sm{}, so{};
    auto init = [](FseSt& s, const SeqTab& t, uint32_t sym) {
        if (t.mode != 1) s.init(t.t, sym);
    };
    auto enc = [&](FseSt& s, const SeqTab& t, uint32_t sym) {
        if (t.mode != 1) s.enc(b, t.t, sym);
    };
    const Coded& z = q[ns - 1];
    init(sm, tm, z.mlc);
    init(so, to, z.ofc);
    init(sl, tl, z.llc);
    b.put(z.ll - kLLBase[z.llc], kLLBits[z.llc]);
    b.put(z.ml - kMLBase[z.mlc], kMLBits[z.mlc]);
    b.put(z.ofv - (1u << z.ofc), z.ofc);
    for (uint32_t k = ns - 1; k-- > 0;) {
        const Coded& x = q[k];
        enc(so, to, x.ofc);
        enc(sm, tm, x.mlc);
        enc(sl, tl, x.llc);
        b.put(x.ll - kLLBase[x.llc], kLLBits[x.llc]);
        b.put(x.ml - kMLBase[x.mlc], kMLBits[x.mlc]);
        b.put(x.ofv - (1u << x.ofc), x.ofc);
    }
    if (tm.mode != 1) sm.flush(b, tm.t);
    if (to.mode != 1) so.flush(b, to.t);
    if (tl.mode != 1) sl.flush(b, tl.t);
    b.close();
    o.insert(o.end(), b.b.begin(), b.b.end());
}

// offsets -> offset values: repeat codes for offsets set earlier in this block
std::vector<Coded> code_sequences(const std::vector<Seq>& s) {
    std::vector<Coded> q;
    uint32_t rep[3] = {0, 0, 0};  // 0 = not known in this block
    uint32_t lit_end = 0, sub = 0;
    for (const Seq& e : s) {
        if (sub_of(e.pos) != sub) {  // repeat offsets tracked per sub-block (one GPU lane each)
            sub = sub_of(e.pos);
            rep[0] = rep[1] = rep[2] = 0;
        }
        Coded c;
        c.ll = e.pos - lit_end;
        c.ml = e.ml;
        const uint32_t o = e.off;
        uint32_t rc = 0;  // repeat code 0..3 as ZSTD_updateRep sees it (offset value - 1 + ll0)
        c.ofv = o + 3;
        {
            const bool ll0 = c.ll == 0;
            if (!ll0 && rep[0] == o) {
                c.ofv = 1;
            } else if (rep[1] && rep[1] == o) {
                c.ofv = ll0 ? 1 : 2;
            } else if (rep[2] && rep[2] == o) {
                c.ofv = ll0 ? 2 : 3;
            } else if (ll0 && rep[0] > 1 && rep[0] - 1 == o) {
                c.ofv = 3;
            }
            if (c.ofv <= 3) rc = c.ofv - 1 + (ll0 ? 1 : 0);
        }
        if (c.ofv > 3) {
            rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = o;
        } else if (rc > 0) {
            const uint32_t curo = rc == 3 ? rep[0] - 1 : rep[rc];
            if (rc >= 2) rep[2] = rep[1];
            rep[1] = rep[0];
            rep[0] = curo;
        }
        c.llc = (uint8_t)ll_code(c.ll);
        c.mlc = (uint8_t)ml_code(c.ml);
        c.ofc = (uint8_t)highbit(c.ofv);
        q.push_back(c);
        lit_end = e.pos + e.ml;
    }
    return q;
}

void block_header(uint8_t* o, bool last, uint32_t type, uint32_t size) {
    const uint32_t h = (last ? 1u : 0u) | type << 1 | size << 3;
    o[0] = (uint8_t)h;
    o[1] = (uint8_t)(h >> 8);
    o[2] = (uint8_t)(h >> 16);
}

size_t block(const uint8_t* src, uint32_t n, uint32_t avail, bool last, uint8_t* out) {
    bool rle = n > 0;
    for (uint32_t i = 1; i < n && rle; ++i) rle = src[i] == src[0];
    if (rle) {
        block_header(out, last, 1, n);
        out[3] = src[0];
        return 4;
    }
    std::vector<Seq> seqs;
    parse(src, n, avail, seqs);
    std::vector<uint8_t> lit, samp;
    uint32_t at = 0;
    auto run = [&](uint32_t a, uint32_t e) {
        lit.insert(lit.end(), src + a, src + e);
        for (uint32_t p = (a + 15) & ~15u; p < e; p += 16) samp.push_back(src[p]);
    };
    for (const Seq& e : seqs) {
        run(at, e.pos);
        at = e.pos + e.ml;
    }
    run(at, n);
    std::vector<uint8_t> body;
    literals(body, lit, samp);
    sequences(body, code_sequences(seqs));
    if (body.size() >= n) {
        block_header(out, last, 0, n);
        std::memcpy(out + 3, src, n);
        return 3 + (size_t)n;
    }
    block_header(out, last, 2, (uint32_t)body.size());
    std::memcpy(out + 3, body.data(), body.size());
    return 3 + body.size();
}

size_t frame_header(uint8_t* o, uint64_t len) {
    o[0] = 0x28;
    o[1] = 0xB5;
    o[2] = 0x2F;
    o[3] = 0xFD;
    if (len < 256) {
        o[4] = 0x20;
        o[5] = (uint8_t)len;
        return 6;
    }
    if (len < 65536 + 256) {
        o[4] = 0x60;
        o[5] = (uint8_t)(len - 256);
        o[6] = (uint8_t)((len - 256) >> 8);
        return 7;
    }
    if (len <= 0xFFFFFFFFull) {
        o[4] = 0xA0;
        for (int i = 0; i < 4; ++i) o[5 + i] = (uint8_t)(len >> (8 * i));
        return 9;
    }
    o[4] = 0xE0;
    for (int i = 0; i < 8; ++i) o[5 + i] = (uint8_t)(len >> (8 * i));
    return 13;
}

}  // namespace

extern "C" {

uint64_t zstd_twin_hist_inserts(void) { return g_hist_inserts; }

// The parse of one block (diagnostics: the GPU's PBS_ZSTD_DEBUG_ITEM dump is compared with
// it): src = the block, src[-avail..-1] the chunk before it; {pos, ml, off} triples.
uint64_t zstd_twin_parse(const uint8_t* src, uint32_t n, uint32_t avail, uint32_t* out, uint64_t cap) {
    std::vector<Seq> s;
    parse(src, n, avail, s);
    for (size_t i = 0; i < s.size() && i < cap; ++i) {
        out[3 * i] = s[i].pos;
        out[3 * i + 1] = s[i].ml;
        out[3 * i + 2] = s[i].off;
    }
    return s.size();
}

uint64_t zstd_twin_bound(uint64_t len) {
    const uint64_t nb = len ? (len + kBlock - 1) / kBlock : 1;
    return 13 + len + 3 * nb;
}

// The frame of one chunk; returns its size (cap >= zstd_twin_bound(len)).
uint64_t zstd_twin_frame(const uint8_t* src, uint64_t len, uint8_t* out) {
    size_t o = frame_header(out, len);
    if (len == 0) {
        block_header(out + o, true, 0, 0);
        return o + 3;
    }
    for (uint64_t b = 0; b < len; b += kBlock) {
        const uint32_t n = (uint32_t)(len - b < kBlock ? len - b : kBlock);
        o += block(src + b, n, (uint32_t)b, b + n == len, out + o);
    }
    return o;
}

}  // extern "C"
