// Shared bits of the example ports: the synthetic random stream of DESIGN.md section 7
// (byte x = LE byte x & 7 of splitmix64(seed ^ (x >> 3))), standing in for /dev/urandom
// and random-test.dat so the outputs are reproducible and checkable against the oracle.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// bytes [off, off + n) of the seeded random stream
inline void random_bytes(uint64_t seed, uint64_t off, uint8_t* out, size_t n) {
    size_t i = 0;
    for (; i < n && ((off + i) & 7); ++i)
        out[i] = (uint8_t)(splitmix64(seed ^ ((off + i) >> 3)) >> (((off + i) & 7) * 8));
    for (; i + 8 <= n; i += 8) {  // whole words (little-endian host)
        const uint64_t w = splitmix64(seed ^ ((off + i) >> 3));
        std::memcpy(out + i, &w, 8);
    }
    for (; i < n; ++i)
        out[i] = (uint8_t)(splitmix64(seed ^ ((off + i) >> 3)) >> (((off + i) & 7) * 8));
}
