// VGPR bank-conflict probe for 3-source VOP3 ops (research tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)
#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))
template <int K>
__global__ void k(unsigned* out) {
    unsigned long long t0, t1;
    asm volatile("v_mov_b32 v20, 1\n v_mov_b32 v21, 2\n v_mov_b32 v22, 3\n v_mov_b32 v23, 4\n v_mov_b32 v24, 5\n v_mov_b32 v25, 6\n v_mov_b32 v26, 7\n v_mov_b32 v27, 8\n v_mov_b32 v28, 9\n v_mov_b32 v29, 10\n v_mov_b32 v30, 11\n v_mov_b32 v31, 12\n v_mov_b32 v32, 13" ::: "v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32");
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
    for (int it = 0; it < 32; ++it) {
        // 4 independent destinations (v20..v23), sources chosen by bank
        if constexpr (K == 0) asm volatile(R64("v_bitop3_b32 v20, v20, v24, v28 bitop3:0x96\n v_bitop3_b32 v21, v21, v25, v29 bitop3:0x96\n v_bitop3_b32 v22, v22, v26, v30 bitop3:0x96\n v_bitop3_b32 v23, v23, v27, v31 bitop3:0x96\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 1) asm volatile(R64("v_bitop3_b32 v20, v20, v25, v30 bitop3:0x96\n v_bitop3_b32 v21, v21, v26, v31 bitop3:0x96\n v_bitop3_b32 v22, v22, v27, v28 bitop3:0x96\n v_bitop3_b32 v23, v23, v24, v29 bitop3:0x96\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 2) asm volatile(R64("v_xor_b32 v20, v20, v24\n v_xor_b32 v21, v21, v25\n v_xor_b32 v22, v22, v26\n v_xor_b32 v23, v23, v27\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 3) asm volatile(R64("v_xor_b32 v20, v20, v25\n v_xor_b32 v21, v21, v26\n v_xor_b32 v22, v22, v27\n v_xor_b32 v23, v23, v24\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 4) asm volatile(R64("v_max3_u32 v20, v20, v24, v28\n v_max3_u32 v21, v21, v25, v29\n v_max3_u32 v22, v22, v26, v30\n v_max3_u32 v23, v23, v27, v31\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 5) asm volatile(R64("v_max3_u32 v20, v20, v25, v30\n v_max3_u32 v21, v21, v26, v31\n v_max3_u32 v22, v22, v27, v28\n v_max3_u32 v23, v23, v24, v29\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 6) asm volatile(R64("v_alignbit_b32 v20, v20, v20, 31\n v_alignbit_b32 v21, v21, v21, 31\n v_alignbit_b32 v22, v22, v22, 31\n v_alignbit_b32 v23, v23, v23, 31\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 7) asm volatile(R64("v_perm_b32 v20, v24, v28, s0\n v_perm_b32 v21, v25, v29, s0\n v_perm_b32 v22, v26, v30, s0\n v_perm_b32 v23, v27, v31, s0\n") ::: "v20","v21","v22","v23");
        if constexpr (K == 8) asm volatile(R64("v_perm_b32 v20, v25, v30, s0\n v_perm_b32 v21, v26, v31, s0\n v_perm_b32 v22, v27, v28, s0\n v_perm_b32 v23, v24, v29, s0\n") ::: "v20","v21","v22","v23");
    }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
    if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)(t1 - t0);
}
int main() {
    unsigned* d; CK(hipMalloc(&d, 4096)); unsigned h[4];
    const char* nm[] = {"bitop3 same-bank srcs", "bitop3 diff-bank srcs", "xor same-bank", "xor diff-bank", "max3 same-bank", "max3 diff-bank", "alignbit (h,h,31)", "perm same-bank", "perm diff-bank"};
#define RUN(K) for (int w = 1; w <= 4; w *= 2) { hipLaunchKernelGGL(k<K>, dim3(1), dim3(256 * w), 0, 0, d); CK(hipDeviceSynchronize()); hipLaunchKernelGGL(k<K>, dim3(1), dim3(256 * w), 0, 0, d); CK(hipDeviceSynchronize()); CK(hipMemcpy(h, d, 4, hipMemcpyDeviceToHost)); printf("%-24s waves/SIMD=%d  %.2f cyc/instr/wave -> SIMD %.2f cyc/instr\n", nm[K], w, h[0] / (32.0 * 256), h[0] / (32.0 * 256) / w); }
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8)
    return 0;
}
