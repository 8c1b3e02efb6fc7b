// Microbenchmark of the per-block exact scan (scan_blocks_kernel) in isolation
// (research tool, not product code).  Per-launch time vs block count, back to back,
// and a loads-only variant, to separate launch/latency from work.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I proxmox-backup_amd/csrc -I include \
//          scripts/microbench/mb_exact.hip -o scripts/microbench/mb_exact
#include "../../proxmox-backup_amd/csrc/pbs_chunker_kernels.hip"

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void loads_only(const uint8_t* data, uint4* hits, uint64_t nblk) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk || b == 0) return;
    const uint4* src = reinterpret_cast<const uint4*>(data + b * 128 - 64);
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const uint4 v = src[k];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    hits[b] = acc;
}

__global__ void empty_kernel() {}

// table from a device buffer instead of the code object's constant array
// table init from the constant array only
__global__ __launch_bounds__(64) void tab_init_only(uint4* hits) {
    __shared__ uint32_t tab[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = pbs::kBuzhashTable[i];
    __syncthreads();
    if (threadIdx.x == 0) hits[blockIdx.x] = make_uint4(tab[3], tab[5], tab[7], tab[9]);
}

int main() {
    const uint64_t n = 64ull << 20;
    uint8_t* d;
    CK(hipMalloc(&d, n));
    CK(hipMemset(d, 0x5a, n));
    hipLaunchKernelGGL(pbs::gen_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t*)d, n / 8, 7ull, 0ull, 1);
    uint4* hits;
    CK(hipMalloc(&hits, (n / 128) * 16));
    uint8_t* pre;
    CK(hipMalloc(&pre, 64));
    uint32_t* gtab;
    CK(hipMalloc(&gtab, 1024));
    CK(hipMemcpy(gtab, pbs::kBuzhashTable, 1024, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t mask = (4u << 20) * 2 - 1, minimum = mask - 2;
    for (int rep = 0; rep < 2; ++rep) {
        for (uint64_t nblk : {64ull, 2048ull, 8192ull, 65536ull, 524288ull}) {
            for (int variant = 0; variant < 5; ++variant) {
                if (variant == 3) continue;
                const int iters = 20;
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                for (int i = 0; i < iters; ++i) {
                    if (variant == 0)
                        hipLaunchKernelGGL(pbs::scan_blocks_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, 0,
                                           d, nblk * 128, pre, 0u, mask, minimum, hits, nblk);
                    else if (variant == 1)
                        hipLaunchKernelGGL(loads_only, dim3((unsigned)((nblk + 63) / 64)), dim3(64), 0, 0, d, hits, nblk);
                    else if (variant == 2)
                        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0);
                    else
                        hipLaunchKernelGGL(tab_init_only, dim3((unsigned)((nblk + 63) / 64)), dim3(64), 0, 0, hits);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                static const char* nm[] = {"scan_blocks", "loads_only", "empty", "devtab", "tabinit"};
                printf("rep %d %-12s nblk=%7llu : %8.2f us/launch", rep, nm[variant],
                       (unsigned long long)nblk, ms * 1e3 / iters);
                printf("\n");
            }
        }
    }
    return 0;
}
