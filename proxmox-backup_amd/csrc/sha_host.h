// Host SHA-256 (pbs_sha_host.cpp): the SHA-extension block function behind the hybrid
// digest's host share and pbs_digest_chunks_host.  Plain C++ (no HIP types).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

namespace pbs {

struct HostSha {
    uint32_t h[8];
    uint64_t total;  // message bytes absorbed so far (whole blocks)
};

void sha256_host_init(HostSha& s);
// nbytes is a multiple of 64 except on the last call before final (the rest is ignored)
void sha256_host_blocks(HostSha& s, const uint8_t* p, size_t nbytes);
// absorbs the last r < 64 message bytes and key, pads, writes the big-endian digest
void sha256_host_final(HostSha& s, const uint8_t* rest, size_t r, const uint8_t* key, size_t key_len,
                       uint8_t out[32]);
void sha256_host_one(const uint8_t* msg, size_t len, const uint8_t* key, size_t key_len, uint8_t out[32]);
// One message for sha256_host_lanes: `len` bytes at `p`, digest to `out`; `tag` is the
// caller's.
struct ShaJob {
    const uint8_t* p;
    uint64_t len;
    uint8_t* out;
    uint64_t tag;
};
// Hashes the messages next(job, may_block) hands out (false: none now -- and, when
// may_block was true, none to come) on this thread, up to four in step; done(job) after
// each digest is written.  next is asked with may_block = false while other messages are
// open, so the open ones keep going.
void sha256_host_lanes(const std::function<bool(ShaJob&, bool)>& next, const std::function<void(const ShaJob&)>& done,
                       const uint8_t* key, size_t key_len);
void sha256_host_items(const uint8_t* host, uint64_t base, const uint64_t* bounds, const uint32_t* items,
                       size_t n, const uint8_t* key, size_t key_len, uint8_t* digests, int threads);
bool sha256_host_has_ni();
bool all_zero(const uint8_t* p, size_t n);

}  // namespace pbs
