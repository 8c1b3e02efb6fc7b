// Microbenchmark of scan_main_kernel variants (research tool, not product code).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I proxmox-backup_amd/csrc mb_scan.hip -o mb_scan
// Run:   ./mb_scan [GiB=16] [reps=5]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "buzhash_table.h"
#include "scan_variants.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill(uint64_t* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// kind 1: the product's VM-image generator (40% zero 4 KiB pages, one 64 MiB zero
// extent per GiB); kind 2: all zero
__global__ void fill_kind(uint64_t* p, uint64_t n, int kind) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < n; w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t v = 0;
        if (kind == 1) {
            const uint64_t seed = 0x5EED0003ull, x = w << 3, g = x >> 30;
            const uint64_t ext = (sm64(seed ^ 0x4558544E54000000ull ^ g) & 15u) << 26;
            const uint64_t in_g = x & ((1ull << 30) - 1);
            if (!(in_g >= ext && in_g < ext + (1ull << 26)) &&
                sm64(seed ^ 0x7A65726F50414745ull ^ (x >> 12)) % 100u >= 40u)
                v = sm64(seed ^ 0x52414E44574F5244ull ^ w);
        }
        p[w] = v;
    }
}

// plain coalesced streaming read (16 B/lane), the HBM reference point
template <bool NT>
__global__ __launch_bounds__(256) void stream_read(const uint4* __restrict__ p, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        u4 w = NT ? __builtin_nontemporal_load((const u4*)(p + i)) : *(const u4*)(p + i);
        uint4 v = make_uint4(w.x, w.y, w.z, w.w);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

static uint32_t rotl(uint32_t x, int r) { return r ? (x << r) | (x >> (32 - r)) : x; }

int main(int argc, char** argv) {
    double gib = argc > 1 ? atof(argv[1]) : 16.0;
    int reps = argc > 2 ? atoi(argv[2]) : 5;
    int only = argc > 3 ? atoi(argv[3]) : -1;  // run a single variant (for PMC collection)
    int kind = argc > 4 ? atoi(argv[4]) : 0;   // 0 random, 1 vmimage-like, 2 zeros
    int vid = 0;
    uint64_t n = (uint64_t)(gib * (1ull << 30));
    n = n / (1ull << 20) * (1ull << 20);
    uint8_t* d; CK(hipMalloc(&d, n));
    if (kind == 0)
        hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (uint64_t*)d, n / 8);
    else
        hipLaunchKernelGGL(fill_kind, dim3(8192), dim3(256), 0, 0, (uint64_t*)d, n / 8, kind);
    printf("data kind %d (%s)\n", kind, kind == 0 ? "random" : kind == 1 ? "vmimage" : "zeros");
    uint32_t *tab, *cnt; uint64_t* susp;
    uint32_t* tab2;
    CK(hipMalloc(&tab, 1024)); CK(hipMalloc(&tab2, 2048)); CK(hipMalloc(&cnt, 16)); CK(hipMalloc(&susp, 1 << 24));
    const uint64_t avg = 4ull << 20;
    const uint32_t mask = (uint32_t)(avg * 2 - 1), minimum = mask - 2;
    const int nb = __builtin_popcount(mask), rot = (32 - nb) & 31;
    std::vector<uint32_t> t(256);
    for (int i = 0; i < 256; ++i) t[i] = rotl(pbs::kBuzhashTable[i], rot);
    CK(hipMemcpy(tab, t.data(), 1024, hipMemcpyHostToDevice));
    const uint32_t thr = minimum << rot;
    std::vector<uint32_t> t2(512);  // parity frame (FR 2): [rotl(T, rot+1) | rotl(T, rot)]
    for (int i = 0; i < 256; ++i) { t2[i] = rotl(pbs::kBuzhashTable[i], (rot + 1) & 31); t2[256 + i] = t[i]; }
    CK(hipMemcpy(tab2, t2.data(), 2048, hipMemcpyHostToDevice));
    const uint32_t thr2 = ((1u << (nb - 1)) - 3u) << ((33 - nb) & 31);
    hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
    int cu = prop.multiProcessorCount;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    auto report = [&](const char* name, float ms) {
        printf("%-34s %8.3f ms  %8.1f GB/s  (%.1f%% of 8 TB/s)\n", name, ms, n / ms / 1e6, n / ms / 1e6 / 80.0);
        fflush(stdout);
    };
    for (int nt = 0; nt < 2; ++nt) if (only < 0 || only == 100 + nt) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            if (nt) hipLaunchKernelGGL(stream_read<true>, dim3(cu * 8), dim3(256), 0, 0, (const uint4*)d, n / 16, cnt);
            else hipLaunchKernelGGL(stream_read<false>, dim3(cu * 8), dim3(256), 0, 0, (const uint4*)d, n / 16, cnt);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;
        }
        report(nt ? "stream_read 16B/lane nt" : "stream_read 16B/lane", best);
    }
#define RUN(SEG, NW, MODE, ASM, AUX)                                                             \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_v1<SEG, NW, MODE, ASM, AUX>), dim3(cu), dim3(NW * 64), 0, 0, \
                               d, tiles, tab, thr, susp, cnt, 1u << 21);                    \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "scan SEG=%d W=%d mode=%d asm=%d aux=%d susp=%u", SEG, NW, MODE, (int)ASM, AUX, h_cnt); \
        report(nm, best);                                                                   \
    }
#define RUN2(SEG, NW, MODE, AUX)                                                             \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_v2<SEG, NW, MODE, AUX>), dim3(cu), dim3(NW * 64), 0, 0, \
                               d, tiles, tab, thr, susp, cnt, 1u << 21);                    \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "v2 SEG=%d W=%d mode=%d aux=%d susp=%u", SEG, NW, MODE, AUX, h_cnt); \
        report(nm, best);                                                                   \
    }
#define RUN3(SEG, MODE, AUX, G, PF) RUN3Z(SEG, MODE, AUX, G, PF, 1)
#define RUN3Z(SEG, MODE, AUX, G, PF, ZS) RUN3F(SEG, MODE, AUX, G, PF, ZS, 1)
#define RUN3F(SEG, MODE, AUX, G, PF, ZS, FR)                                                    \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_kernel<SEG, MODE, AUX, G, PF, ZS, FR>), dim3(cu), dim3(8 * 64), 0, 0, \
                               d, tiles, FR == 2 ? tab2 : tab, FR == 2 ? thr2 : thr, susp, cnt, 1u << 21); \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "v3 SEG=%d mode=%d G=%d ZS=%d FR=%d susp=%u", SEG, MODE, G, ZS, FR, h_cnt); \
        report(nm, best * (double)n / (double)(tiles * 64ull * SEG));                                                                   \
    }
#define RUNR96(SEG, MODE)                                                                   \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_r96<SEG, MODE>), dim3(cu), dim3(pbs::kR96Waves * 64), 0, 0, \
                               d, tiles, tab2, thr2, susp, cnt, 1u << 21);                  \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "r96 SEG=%d mode=%d susp=%u", SEG, MODE, h_cnt); \
        report(nm, best);                                                                   \
    }
#define RUN4(SEG, MODE, AUX, G)                                                             \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_v4<SEG, MODE, AUX, G>), dim3(cu), dim3(8 * 64), 0, 0, \
                               d, tiles, tab, thr, susp, cnt, 1u << 21);                    \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "v4 SEG=%d mode=%d aux=%d G=%d susp=%u", SEG, MODE, AUX, G, h_cnt); \
        report(nm, best);                                                                   \
    }
#define RUN5(SEG, MODE, AUX)                                                             \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_v5<SEG, MODE, AUX>), dim3(cu), dim3(8 * 64), 0, 0, \
                               d, tiles, tab, thr, susp, cnt, 1u << 21);                    \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "v5 SEG=%d mode=%d aux=%d susp=%u", SEG, MODE, AUX, h_cnt); \
        report(nm, best);                                                                   \
    }
#define RUN6(SEG, MODE, AUX, G)                                                             \
    if (only < 0 || only == vid++) {                                                        \
        float best = 1e30f; uint32_t h_cnt = 0;                                             \
        const uint64_t tiles = n / (64ull * SEG);                                           \
        for (int r = 0; r < reps; ++r) {                                                    \
            CK(hipMemset(cnt, 0, 16));                                                      \
            CK(hipEventRecord(e0));                                                         \
            hipLaunchKernelGGL((pbs::scan_main_v6<SEG, MODE, AUX, G>), dim3(cu), dim3(8 * 64), 0, 0, \
                               d, tiles, tab, thr, susp, cnt, 1u << 21);                    \
            CK(hipGetLastError());                                                          \
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));                            \
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best;   \
            CK(hipMemcpy(&h_cnt, cnt, 4, hipMemcpyDeviceToHost));                           \
        }                                                                                   \
        char nm[96]; snprintf(nm, sizeof nm, "v6 SEG=%d mode=%d aux=%d G=%d susp=%u", SEG, MODE, AUX, G, h_cnt); \
        report(nm, best);                                                                   \
    }
    RUN3F(32768, 0, 2, 4, 0, 0, 1)
    RUN3F(32768, 0, 2, 4, 0, 0, 2)
    RUN3F(32768, 0, 2, 4, 0, 0, 1)
    RUN3F(32768, 0, 2, 4, 0, 0, 2)
    RUN3F(32768, 0, 2, 4, 0, 0, 1)
    RUN3F(32768, 0, 2, 4, 0, 0, 2)
    RUN3F(32768, 0, 2, 4, 0, 0, 1)
    RUN3F(32768, 0, 2, 4, 0, 0, 2)
    return 0;
}
