// Microbenchmark: latency of one host <-> persistent-kernel request round trip, the
// quantity that bounds scan() per 8 KiB read through the scan server (scan_server.h).
//
//   mode 0: request record polled in pinned host memory (the product's mailbox), the
//           8 KiB payload read by the kernel from pinned host memory;
//   mode 1: request record and payload in device memory written by the host through
//           its CPU mapping (only if the allocation has one), ack in pinned host memory.
//
// Each round: host writes payload + seq, kernel sees seq, reads the payload (sums it so
// the loads are real), writes ack; host spins on ack.  Device-side stamps (wall_clock64,
// 100 MHz) split the round: host store -> kernel sees (not measurable alone), kernel
// sees -> payload staged, staged -> ack stored.  Every kernel exits on a quit flag or
// after 2 s without a request.
//
//   hipcc --offload-arch=gfx950 -O3 -o mb_mailbox mb_mailbox.hip && ./mb_mailbox
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

struct alignas(64) Req {
    uint32_t seq, len;
    uint32_t quit, pad;
};
struct alignas(64) Ack {
    uint64_t seq;
    uint64_t sum;
    uint64_t t_seen, t_staged, t_done;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void server(const Req* req, const uint8_t* payload, Ack* ack,
                                              uint64_t idle) {
    __shared__ uint32_t ctl[2];
    __shared__ uint64_t part[4];
    const int tid = threadIdx.x;
    uint32_t last = 0;
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (tid == 0) {
            uint32_t cmd = 2;
            for (;;) {
                const u32x4 r = *reinterpret_cast<const volatile u32x4*>(req);
                if (r.z) break;
                if (r.x != last) {
                    cmd = 1;
                    ctl[1] = r.y;
                    last = r.x;
                    break;
                }
                if (wall_clock64() - t0 > idle) break;
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            ctl[0] = cmd;
        }
        __syncthreads();
        if (ctl[0] != 1) return;
        const uint64_t ts = wall_clock64();
        const uint32_t len = ctl[1];
        uint64_t s = 0;
        const u32x4* p = reinterpret_cast<const u32x4*>(payload);
        for (uint32_t i = tid; i < len / 16; i += 256) {
            const u32x4 v = __builtin_nontemporal_load(p + i);
            s += (uint64_t)v.x + v.y + v.z + v.w;
        }
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((tid & 63) == 0) part[tid >> 6] = s;
        __syncthreads();
        const uint64_t tg = wall_clock64();
        if (tid == 0) {
            ack->sum = part[0] + part[1] + part[2] + part[3];
            ack->t_seen = ts;
            ack->t_staged = tg;
            ack->t_done = wall_clock64();
            __hip_atomic_store(&ack->seq, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        t0 = wall_clock64();
    }
}

// mode 3: every wave's lane 0 polls (staggered: ~4 loads in flight over PCIe instead of
// one), the first to see the request raises an LDS flag; the payload is read with all of
// a thread's loads in flight before any is used
__global__ __launch_bounds__(256) void server4(const Req* req, const uint8_t* payload, Ack* ack, uint64_t idle) {
    __shared__ uint32_t s_go, s_len, s_seq;
    __shared__ uint64_t part[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t last = 0;
    if (tid == 0) s_go = 0;
    __syncthreads();
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (lane == 0) {
            for (int d = 0; d < wave; ++d) __builtin_amdgcn_s_sleep(8);  // stagger the pollers
            for (;;) {
                if (__hip_atomic_load(&s_go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                const u32x4 r = *reinterpret_cast<const volatile u32x4*>(req);
                if (r.z) {
                    __hip_atomic_store(&s_go, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (r.x != last) {
                    s_len = r.y;
                    s_seq = r.x;
                    __hip_atomic_store(&s_go, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
                if (wall_clock64() - t0 > idle) {
                    __hip_atomic_store(&s_go, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    break;
                }
            }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (s_go != 1) return;
        const uint64_t ts = wall_clock64();
        const uint32_t len = s_len;
        last = s_seq;
        const u32x4* p = reinterpret_cast<const u32x4*>(payload);
        const uint32_t n16 = len / 16;
        uint64_t s = 0;
        for (uint32_t i0 = tid; i0 < n16; i0 += 16 * 256) {  // 16 loads in flight per thread
            u32x4 v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (i0 + 256 * u < n16) v[u] = __builtin_nontemporal_load(p + i0 + 256 * u);
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (i0 + 256 * u < n16) s += (uint64_t)v[u].x + v[u].y + v[u].z + v[u].w;
        }
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) part[wave] = s;
        __syncthreads();
        const uint64_t tg = wall_clock64();
        if (tid == 0) {
            ack->sum = part[0] + part[1] + part[2] + part[3];
            ack->t_seen = ts;
            ack->t_staged = tg;
            ack->t_done = wall_clock64();
            s_go = 0;
            __hip_atomic_store(&ack->seq, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        t0 = wall_clock64();
    }
}

static int run(int mode, uint32_t len, int iters) {
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    Ack* ack = nullptr;
    CK(hipHostMalloc((void**)&ack, sizeof(Ack), fl));
    memset(ack, 0, sizeof(Ack));
    Ack* ack_d = nullptr;
    CK(hipHostGetDevicePointer((void**)&ack_d, ack, 0));
    Req* req_h = nullptr;      // host's view
    Req* req_d = nullptr;      // kernel's view
    uint8_t* pay_h = nullptr;  // host's view
    uint8_t* pay_d = nullptr;
    void* dev_alloc[2] = {nullptr, nullptr};
    if (mode == 0 || mode == 3) {
        CK(hipHostMalloc((void**)&req_h, sizeof(Req), fl));
        CK(hipHostMalloc((void**)&pay_h, 1 << 20, fl));
        CK(hipHostGetDevicePointer((void**)&req_d, req_h, 0));
        CK(hipHostGetDevicePointer((void**)&pay_d, pay_h, 0));
    } else {
        const unsigned df = mode == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
        CK(hipExtMallocWithFlags(&dev_alloc[0], 4096, df));
        CK(hipExtMallocWithFlags(&dev_alloc[1], 1 << 20, df));
        hipPointerAttribute_t a{};
        CK(hipPointerGetAttributes(&a, dev_alloc[0]));
        printf("mode %d: device alloc %p type %d hostPointer %p devicePointer %p\n", mode, dev_alloc[0],
               (int)a.type, a.hostPointer, a.devicePointer);
        if (!a.hostPointer) {
            printf("mode %d: no host mapping; skipped\n", mode);
            return 0;
        }
        hipPointerAttribute_t b{};
        CK(hipPointerGetAttributes(&b, dev_alloc[1]));
        req_h = (Req*)a.hostPointer;
        req_d = (Req*)dev_alloc[0];
        pay_h = (uint8_t*)b.hostPointer;
        pay_d = (uint8_t*)dev_alloc[1];
        // first host write, then read it back through the runtime
        const uint32_t probe = 0x12345678u;
        memcpy(pay_h, &probe, 4);
        uint32_t back = 0;
        CK(hipMemcpy(&back, dev_alloc[1], 4, hipMemcpyDeviceToHost));
        printf("mode %d: host write through the mapping read back as %08x\n", mode, back);
        if (back != probe) return 0;
    }
    memset(req_h, 0, sizeof(Req));
    std::vector<uint8_t> src(len);
    for (uint32_t i = 0; i < len; ++i) src[i] = (uint8_t)(i * 7 + 1);
    uint64_t want = 0;
    for (uint32_t i = 0; i < len / 4; ++i) {
        uint32_t w;
        memcpy(&w, src.data() + 4 * i, 4);
        want += w;
    }
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (mode == 3)
        hipLaunchKernelGGL(server4, dim3(1), dim3(256), 0, st, req_d, pay_d, ack_d, (uint64_t)200000000);
    else
        hipLaunchKernelGGL(server, dim3(1), dim3(256), 0, st, req_d, pay_d, ack_d, (uint64_t)200000000);
    CK(hipGetLastError());
    double tot = 0, t_seen_staged = 0, t_staged_done = 0;
    int bad = 0;
    std::vector<double> lat;
    for (int it = 1; it <= iters; ++it) {
        const auto t0 = std::chrono::steady_clock::now();
        memcpy(pay_h, src.data(), len);
        __atomic_store_n(&req_h->len, len, __ATOMIC_RELAXED);
        __builtin_ia32_sfence();  // write-combined device mappings: payload before seq
        __atomic_store_n(&req_h->seq, (uint32_t)it, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();  // and flush the seq itself
        const auto tw = std::chrono::steady_clock::now();
        while (__atomic_load_n(&ack->seq, __ATOMIC_ACQUIRE) != (uint64_t)it) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count() > 2.0) {
                printf("mode %d: request %d timed out\n", mode, it);
                req_h->quit = 1;
                (void)hipStreamSynchronize(st);
                return 1;
            }
            __builtin_ia32_pause();
        }
        const auto t1 = std::chrono::steady_clock::now();
        const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
        if (it > 100) {
            tot += us;
            lat.push_back(us);
            t_seen_staged += (ack->t_staged - ack->t_seen) / 100.0;
            t_staged_done += (ack->t_done - ack->t_staged) / 100.0;
        }
        if (ack->sum != want) ++bad;
    }
    __atomic_store_n(&req_h->quit, 1u, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(st));
    const int n = iters - 100;
    std::sort(lat.begin(), lat.end());
    printf("mode %d len %6u: round trip mean %.2f us p50 %.2f p90 %.2f | kernel: staging %.2f us, "
           "ack %.2f us | wrong sums %d\n",
           mode, len, tot / n, lat[n / 2], lat[n * 9 / 10], t_seen_staged / n, t_staged_done / n, bad);
    CK(hipStreamDestroy(st));
    return 0;
}

int main() {
    int rc = 0;
    for (int mode : {0, 3})
        for (uint32_t len : {0u, 8192u, 65536u}) rc |= run(mode, len, 3000);
    return rc;
}
