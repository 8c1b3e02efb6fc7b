// Dependent-latency and issue-rate probe for the VALU ops of the roll loop (research tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1;} } while (0)

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int K>
__global__ void lat(unsigned* out, unsigned seed) {
    unsigned a = seed ^ threadIdx.x, b = seed * 3, c = seed * 7, d0 = a + 1, d1 = a + 2, d2 = a + 3, d3 = a + 4;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int it = 0; it < 16; ++it) {
        if constexpr (K == 0) asm volatile(REP64("v_xor_b32 %0, %0, %1\n") : "+v"(a) : "v"(b));
        if constexpr (K == 1) asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 31\n") : "+v"(a));
        if constexpr (K == 2) asm volatile(REP64("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n") : "+v"(a) : "v"(b), "v"(c));
        if constexpr (K == 3) asm volatile(REP64("v_perm_b32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "s"(0x0c0c0500u));
        if constexpr (K == 4) asm volatile(REP64("v_max3_u32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c));
        if constexpr (K == 5) asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 31\nv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n") : "+v"(a) : "v"(b), "v"(c));
        // 4 independent chains interleaved: issue-rate bound
        if constexpr (K == 6) asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 31\nv_alignbit_b32 %1, %1, %1, 31\nv_alignbit_b32 %2, %2, %2, 31\nv_alignbit_b32 %3, %3, %3, 31\n") : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
        if constexpr (K == 7) asm volatile(REP64("v_xor_b32 %0, %0, %4\nv_xor_b32 %1, %1, %4\nv_xor_b32 %2, %2, %4\nv_xor_b32 %3, %3, %4\n") : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(b));
        if constexpr (K == 8) asm volatile(REP64("v_lshl_or_b32 %0, %0, 1, %1\n") : "+v"(a) : "v"(b));
    }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    unsigned long long rt0, rt1;
    if (threadIdx.x == 0) {
        out[blockIdx.x * 4 + 0] = (unsigned)(t1 - t0);
        out[blockIdx.x * 4 + 1] = a ^ d0 ^ d1 ^ d2 ^ d3;
    }
}

__global__ void clk(unsigned* out) {
    unsigned long long t0, t1, r0, r1;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
    unsigned a = threadIdx.x;
    for (int i = 0; i < 100000; ++i) asm volatile(REP8("v_xor_b32 %0, %0, %0\n") : "+v"(a));
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
    if (threadIdx.x == 0) { out[0] = (unsigned)(t1 - t0); out[1] = (unsigned)(r1 - r0); out[2] = a; }
}

int main() {
    unsigned* d; CK(hipMalloc(&d, 1 << 20));
    unsigned h[8];
    const char* names[] = {"xor", "alignbit", "bitop3", "perm", "max3", "alignbit+bitop3 pair", "4x alignbit indep", "4x xor indep", "lshl_or"};
    const int nops[] = {1024, 1024, 1024, 1024, 1024, 2048, 4096, 4096, 1024};
#define RUN(K) for (int waves = 1; waves <= 2; ++waves) { \
        hipLaunchKernelGGL(lat<K>, dim3(1), dim3(64 * 4 * waves), 0, 0, d, 5u); CK(hipDeviceSynchronize()); \
        hipLaunchKernelGGL(lat<K>, dim3(1), dim3(64 * 4 * waves), 0, 0, d, 5u); CK(hipDeviceSynchronize()); \
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost)); \
        printf("%-24s waves/SIMD=%d  %6.2f cyc/op (per wave)\n", names[K], waves, h[0] / (double)nops[K]); }
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8)
    hipLaunchKernelGGL(clk, dim3(256), dim3(256), 0, 0, d); CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
    printf("clock: %u shader cycles in %u x 10ns -> %.3f GHz\n", h[0], h[1], h[0] / (h[1] * 10.0));
    return 0;
}
