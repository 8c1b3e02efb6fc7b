// VALU dependency latency on gfx950, one wave alone on a SIMD: cycles per instruction
// for (a) a chain where every op needs the previous result, (b) two interleaved chains
// (each op needs the result 2 back), (c) four interleaved chains, all v_add3_u32, and
// (d) the SHA-256 round mix (v_alignbit / v_bitop3 / v_add3) as one chain.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void dep1(unsigned* out, unsigned long long* cyc) {
    unsigned a = threadIdx.x, b = 3, c = 5;
    unsigned long long t0 = clock64();
    for (int i = 0; i < 64; ++i) {
        asm volatile(REP64("v_add3_u32 %0, %0, %1, %2\n\t") : "+v"(a) : "v"(b), "v"(c));
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void dep2(unsigned* out, unsigned long long* cyc) {
    unsigned a = threadIdx.x, a2 = 7, b = 3, c = 5;
    unsigned long long t0 = clock64();
    for (int i = 0; i < 64; ++i) {
        asm volatile(REP64("v_add3_u32 %0, %0, %2, %3\n\tv_add3_u32 %1, %1, %2, %3\n\t") : "+v"(a), "+v"(a2) : "v"(b), "v"(c));
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = a + a2;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void dep4(unsigned* out, unsigned long long* cyc) {
    unsigned a = threadIdx.x, a2 = 7, a3 = 9, a4 = 11, b = 3, c = 5;
    unsigned long long t0 = clock64();
    for (int i = 0; i < 64; ++i) {
        asm volatile(REP64("v_add3_u32 %0, %0, %4, %5\n\tv_add3_u32 %1, %1, %4, %5\n\tv_add3_u32 %2, %2, %4, %5\n\tv_add3_u32 %3, %3, %4, %5\n\t")
                     : "+v"(a), "+v"(a2), "+v"(a3), "+v"(a4) : "v"(b), "v"(c));
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = a + a2 + a3 + a4;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void dep1_align(unsigned* out, unsigned long long* cyc) {
    unsigned a = threadIdx.x;
    unsigned long long t0 = clock64();
    for (int i = 0; i < 64; ++i) {
        asm volatile(REP64("v_alignbit_b32 %0, %0, %0, 7\n\t") : "+v"(a));
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void dep1_bitop3(unsigned* out, unsigned long long* cyc) {
    unsigned a = threadIdx.x, b = 3, c = 5;
    unsigned long long t0 = clock64();
    for (int i = 0; i < 64; ++i) {
        asm volatile(REP64("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\t") : "+v"(a) : "v"(b), "v"(c));
    }
    unsigned long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    unsigned* out;
    unsigned long long* cyc;
    hipMalloc(&out, 4096);
    hipMalloc(&cyc, 8);
    struct K { const char* name; void (*f)(unsigned*, unsigned long long*); int ops; } ks[] = {
        {"1 chain v_add3", dep1, 4096}, {"2 chains v_add3", dep2, 8192}, {"4 chains v_add3", dep4, 16384},
        {"1 chain v_alignbit", dep1_align, 4096}, {"1 chain v_bitop3", dep1_bitop3, 4096}};
    for (auto& k : ks) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, out, cyc);
            hipDeviceSynchronize();
        }
        unsigned long long c;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-22s %8llu clock64 ticks, %.2f per instruction\n", k.name, c, (double)c / k.ops);
    }
    return 0;
}
