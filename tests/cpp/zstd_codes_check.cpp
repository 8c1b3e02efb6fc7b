// The arithmetic literal-length / match-length code functions of zstd_enc.h (ll_code,
// ml_code, ll_bits, ll_base, ml_bits, ml_base) against the RFC 8878 3.1.1.3.2.1 tables and
// the table searches, for every length a 64 KiB block can produce.  Exit 0 = equal.
#include <cstdio>
#include "zstd_enc.h"
using namespace pbs::zstd;
int main() {
    int bad = 0;
    for (uint32_t c = 0; c < 36; ++c) if (ll_bits(c) != kLLBits[c] || ll_base(c) != kLLBase[c]) { printf("ll %u\n", c); ++bad; }
    for (uint32_t c = 0; c < 53; ++c) if (ml_bits(c) != kMLBits[c] || ml_base(c) != kMLBase[c]) { printf("ml %u\n", c); ++bad; }
    for (uint32_t v = 0; v < 131072; ++v) {
        uint32_t c = 0; while (c < 35 && kLLBase[c + 1] <= v) ++c;
        if (ll_code(v) != c) { if (bad < 10) printf("llc %u %u %u\n", v, ll_code(v), c); ++bad; }
    }
    for (uint32_t v = 3; v < 131072; ++v) {
        uint32_t c = 0; while (c < 52 && kMLBase[c + 1] <= v) ++c;
        if (ml_code(v) != c) { if (bad < 10) printf("mlc %u %u %u\n", v, ml_code(v), c); ++bad; }
    }
    printf("bad %d\n", bad); return bad != 0;
}
