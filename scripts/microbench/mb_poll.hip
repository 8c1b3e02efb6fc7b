// Microbenchmark: what one scan() request through the scan server (scan_server.h) costs
// beyond the kernel's own work, split into
//   lat   : one 16-byte load of pinned (fine-grained) host memory, dependent chain of 64
//           loads timed on the device (wall_clock64, 100 MHz)
//   bw    : 256 threads reading N bytes of pinned host memory (16 B per load, all issued
//           before the first wait), N = 64 B .. 64 KiB, timed on the device
//   ping  : host store -> kernel sees -> system-scope ack -> host sees, no payload, with
//           P pollers (lane 0 of P waves), each polling its own 64-byte record copy, and
//           S = the s_sleep between polls (0 = spin)
// Every kernel exits on a quit flag or after 1 s without a request.
//
//   hipcc --offload-arch=gfx950 -O3 -o mb_poll mb_poll.hip && ./mb_poll
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct alignas(64) Rec {
    uint32_t seq, quit, pad[14];
};

__global__ void lat_kernel(const uint64_t* host, uint64_t* out) {
    if (threadIdx.x != 0) return;
    uint64_t i = 0;
    const uint64_t t0 = wall_clock64();
    for (int k = 0; k < 64; ++k) i = *reinterpret_cast<const volatile uint64_t*>(host + (i & 7));
    const uint64_t t1 = wall_clock64();
    out[0] = t1 - t0;
    out[1] = i;
}

__global__ __launch_bounds__(256) void bw_kernel(const u32x4* host, uint32_t n16, uint64_t* out) {
    __shared__ uint32_t red[256];
    const uint64_t t0 = wall_clock64();
    u32x4 acc = {0, 0, 0, 0};
    constexpr int U = 16;
    for (uint32_t i0 = threadIdx.x; i0 < n16; i0 += 256 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + 256u * u;
            v[u] = i < n16 ? __builtin_nontemporal_load(host + i) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    red[threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t t1 = wall_clock64();
        uint32_t s = 0;
        for (int i = 0; i < 256; ++i) s ^= red[i];
        out[0] = t1 - t0;
        out[1] = s;
    }
}

__global__ __launch_bounds__(256) void ping_kernel(const Rec* rec, uint64_t* ack, int pollers, int sleep, int relaxed) {
    __shared__ uint32_t s_go, s_seq;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t last = 0;
    uint64_t t_idle = wall_clock64();
    if (tid == 0) s_go = 0;
    __syncthreads();
    for (;;) {
        if (lane == 0 && wave < pollers) {
            for (int d = 0; d < wave; ++d) __builtin_amdgcn_s_sleep(4);
            const volatile Rec* r = rec + wave;
            for (;;) {
                if (__hip_atomic_load(&s_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                const u32x4 v = *reinterpret_cast<const volatile u32x4*>(r);
                uint32_t go = 0;
                if (v.y) go = 2;
                else if (v.x != last) go = 1;
                else if (wall_clock64() - t_idle > 100000000ull) go = 2;
                if (go) {
                    if (go == 1) s_seq = v.x;
                    __hip_atomic_store(&s_go, go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (sleep == 1) __builtin_amdgcn_s_sleep(1);
                if (sleep == 2) __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        if (s_go != 1) return;
        const uint32_t seq = s_seq;
        if (tid == 0) {
            s_go = 0;
            if (relaxed)
                __hip_atomic_store(ack, (uint64_t)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else
                __hip_atomic_store(ack, (uint64_t)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        last = seq;
        t_idle = wall_clock64();
    }
}

int main() {
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    uint64_t *h_lat = nullptr, *d_out = nullptr, h_out[2];
    CK(hipHostMalloc((void**)&h_lat, 4096, fl));
    memset(h_lat, 0, 4096);
    CK(hipMalloc(&d_out, 64));
    uint64_t* d_lat = nullptr;
    CK(hipHostGetDevicePointer((void**)&d_lat, h_lat, 0));
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, d_lat, d_out);
        CK(hipMemcpy(h_out, d_out, 16, hipMemcpyDeviceToHost));
        printf("lat: dependent 16-byte load of pinned host memory %.3f us\n", h_out[0] / 64.0 / 100.0);
    }
    uint8_t *h_buf = nullptr, *d_buf = nullptr;
    CK(hipHostMalloc((void**)&h_buf, 1 << 20, fl));
    memset(h_buf, 1, 1 << 20);
    CK(hipHostGetDevicePointer((void**)&d_buf, h_buf, 0));
    for (uint32_t n : {64u, 1024u, 4096u, 8192u, 16384u, 32768u, 65536u, 262144u}) {
        double best = 1e30, avg = 0;
        for (int rep = 0; rep < 20; ++rep) {
            hipLaunchKernelGGL(bw_kernel, dim3(1), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(d_buf), n / 16, d_out);
            CK(hipMemcpy(h_out, d_out, 16, hipMemcpyDeviceToHost));
            const double us = h_out[0] / 100.0;
            best = std::min(best, us);
            avg += us / 20;
        }
        printf("bw: %6u bytes by 256 threads: best %.2f us avg %.2f us (%.2f GB/s best)\n", n, best, avg, n / best / 1e3);
    }
    Rec* h_rec = nullptr;
    uint64_t* h_ack = nullptr;
    CK(hipHostMalloc((void**)&h_rec, 4 * sizeof(Rec), fl));
    CK(hipHostMalloc((void**)&h_ack, 64, fl));
    Rec* d_rec = nullptr;
    uint64_t* d_ack = nullptr;
    CK(hipHostGetDevicePointer((void**)&d_rec, h_rec, 0));
    CK(hipHostGetDevicePointer((void**)&d_ack, h_ack, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int relaxed : {0, 1})
    for (int pollers : {1, 4}) {
        for (int sleep : {2}) {
            memset(h_rec, 0, 4 * sizeof(Rec));
            *h_ack = 0;
            hipLaunchKernelGGL(ping_kernel, dim3(1), dim3(256), 0, st, d_rec, d_ack, pollers, sleep, relaxed);
            std::vector<double> rt;
            const int N = 20000;
            for (uint32_t s = 1; s <= N; ++s) {
                const auto t0 = std::chrono::steady_clock::now();
                for (int p = 0; p < pollers; ++p) __atomic_store_n(&h_rec[p].seq, s, __ATOMIC_RELEASE);
                while (__atomic_load_n(h_ack, __ATOMIC_ACQUIRE) != s) __builtin_ia32_pause();
                rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            }
            for (int p = 0; p < 4; ++p) __atomic_store_n(&h_rec[p].quit, 1u, __ATOMIC_RELEASE);
            CK(hipStreamSynchronize(st));
            std::sort(rt.begin(), rt.end());
            double m = 0;
            for (double x : rt) m += x / rt.size();
            printf("ping: %s ack, pollers %d sleep %d: mean %.2f us p10 %.2f p50 %.2f p90 %.2f\n", relaxed ? "relaxed" : "release", pollers, sleep, m,
                   rt[rt.size() / 10], rt[rt.size() / 2], rt[rt.size() * 9 / 10]);
        }
    }
    return 0;
}
