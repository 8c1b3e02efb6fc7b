"""Generate mb_lds.hip: LDS lookup throughput probe (perm + ds_read_b32 into a
replicated 64 KiB table, P reads in flight per wave, optional VALU filler per byte)."""
import sys

def body(P, valu):
    if valu == 5:  # roll mix with the LDS read replaced by the perm result (VALU only)
        L = []
        for i in range(64):
            L.append(f"v_perm_b32 %{i % 16}, %{22 + (i//4)%8}, %{30}, %{31 + i%4}")
            L.append(f"v_alignbit_b32 %{20}, %{20}, %{20}, 31")
            L.append(f"v_bitop3_b32 %{20}, %{20}, %{i % 16}, %{(i+8) % 16} bitop3:0x96")
            if i % 2: L.append(f"v_max3_u32 %{21}, %{21}, %{20}, %{(i+3)%16}")
        return "\\n\\t".join(L)
    L = ["s_waitcnt lgkmcnt(0)"]
    nreg = 16
    issued = 0
    def iss(b):
        L.append(f"v_perm_b32 %{16+ (b%4)}, %{22 + (b//4)%8}, %{30}, %{31 + b%4}")
        L.append(f"ds_read_b32 %{b % nreg}, %{16 + (b%4)}")
    for b in range(P):
        iss(b)
    issued = P
    for i in range(64):
        if i + P < 64:
            iss(i + P); issued = i + P + 1
        L.append(f"s_waitcnt lgkmcnt({issued - i - 1})")
        if valu == 0:
            L.append(f"v_xor_b32 %{20}, %{20}, %{i % nreg}")
        elif valu == 2:  # roll mix, waits every 4 bytes
            if (i % 4) != 3: L.pop()
            L.append(f"v_alignbit_b32 %{20}, %{20}, %{20}, 31")
            L.append(f"v_bitop3_b32 %{20}, %{20}, %{i % nreg}, %{(i+8) % nreg} bitop3:0x96")
            if i % 2: L.append(f"v_max3_u32 %{21}, %{21}, %{20}, %{(i+3)%nreg}")
        elif valu == 3:  # roll mix without max3
            L.append(f"v_alignbit_b32 %{20}, %{20}, %{20}, 31")
            L.append(f"v_bitop3_b32 %{20}, %{20}, %{i % nreg}, %{(i+8) % nreg} bitop3:0x96")
        elif valu == 4:  # roll mix, 2 independent chains (even/odd bytes), waits every 4
            if (i % 4) != 3: L.pop()
            c = 20 + (i % 2)
            L.append(f"v_alignbit_b32 %{c}, %{c}, %{c}, 31")
            L.append(f"v_bitop3_b32 %{c}, %{c}, %{i % nreg}, %{(i+8) % nreg} bitop3:0x96")
            if i % 2: L.append(f"v_max3_u32 %{21}, %{21}, %{20}, %{(i+3)%nreg}")
        else:  # the roll loop's dependent pair + half a max3
            L.append(f"v_alignbit_b32 %{20}, %{20}, %{20}, 31")
            L.append(f"v_bitop3_b32 %{20}, %{20}, %{i % nreg}, %{(i+8) % nreg} bitop3:0x96")
            if i % 2: L.append(f"v_max3_u32 %{21}, %{21}, %{20}, %{(i+3)%nreg}")
    return "\\n\\t".join(L)

out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>',
       '#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)']
variants = []
for valu in (1, 2, 3, 4, 5):
    for P in ((14,) if valu != 1 else (14,)):
        name = f"k_v{valu}_p{P}"
        variants.append((name, valu, P))
        outs = ", ".join([f'"=&v"(r{i})' for i in range(16)] + [f'"=&v"(a{i})' for i in range(4)])
        ins = ", ".join([f'"v"(d{i})' for i in range(8)] + ['"v"(lb)'] + [f'"s"(s{i})' for i in range(4)] )
        out.append(f'''template <int NW> __global__ __launch_bounds__(NW * 64) void {name}(uint32_t* out, int iters) {{
    __shared__ uint32_t tab[16384];
    for (int i = threadIdx.x; i < 16384; i += NW * 64) tab[i] = i * 2654435761u;
    __syncthreads();
    uint32_t lb = (threadIdx.x & 63) * 4, acc = threadIdx.x, mx = 0;
    uint32_t d0 = threadIdx.x * 2654435761u, d1 = d0 * 3, d2 = d0 * 5, d3 = d0 * 7, d4 = d0 * 11, d5 = d0 * 13, d6 = d0 * 17, d7 = d0 * 19;
    const uint32_t s0 = 0x0c0c0400u, s1 = 0x0c0c0500u, s2 = 0x0c0c0600u, s3 = 0x0c0c0700u;
    uint32_t r0,r1,r2,r3,r4,r5,r6,r7,r8,r9,r10,r11,r12,r13,r14,r15,a0,a1,a2,a3;
    for (int it = 0; it < iters; ++it) {{
        asm volatile("{body(P, valu)}" : {outs}, "+v"(acc), "+v"(mx) : {ins} : "memory");
        d0 += acc; d3 ^= mx;
    }}
    if (acc == 0x12345 && mx == 7) out[0] = acc;
}}''')
out.append('int main() {')
out.append('  uint32_t* o; CK(hipMalloc(&o, 64)); hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));')
out.append('  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0)); int cu = p.multiProcessorCount; const int iters = 4096;')
for name, valu, P in variants:
    for NW, WGPERCU in ((4, 1), (8, 1), (8, 2), (12, 1)):
        out.append(f'''  {{ float best = 1e9; for (int r = 0; r < 3; ++r) {{ CK(hipEventRecord(e0)); hipLaunchKernelGGL(({name}<{NW}>), dim3(cu * {WGPERCU}), dim3({NW} * 64), 0, 0, o, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = ms < best ? ms : best; }}
    double reads = (double)cu * {WGPERCU} * {NW} * iters * 64; printf("%-10s waves/CU=%2d  %.3f ms  %.3f wave-reads/clk/CU (@2.3GHz)  bytes/clk/CU=%.1f\\n", "{name}", {NW * WGPERCU}, best, reads / (best * 1e-3 * 2.3e9) / cu, 64 * reads / (best * 1e-3 * 2.3e9) / cu); }}''')
out.append('  return 0; }')
open(sys.argv[1], 'w').write("\n".join(out) + "\n")
