// Probe of the two-wave SHA-256 kernel: one workgroup, 64 chunks of 4 MiB; per wave the
// cycles spent in its own work vs at the per-block barrier (clock64 of wave 0 / wave 1).
#define PBS_SHA_PROBE 1
#include "../../proxmox-backup_amd/csrc/pbs_digest.hip"

#include <cstdio>
#include <vector>

int main() {
    const size_t n = 64, len = 4u << 20;
    uint8_t* d = nullptr;
    hipMalloc(&d, n * len);
    hipMemset(d, 0x5a, n * len);
    std::vector<uint64_t> b(n + 1);
    for (size_t i = 0; i <= n; ++i) b[i] = i * len;
    std::vector<uint8_t> dig(n * 32);
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0, 0);
        int rc = pbs_digest_chunks_device(d, n * len, 0, b.data(), n, nullptr, 0, dig.data(), 0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        uint64_t pr[5];
        hipMemcpyFromSymbol(pr, HIP_SYMBOL(pbs::g_sha_probe), sizeof(pr));
        printf("rc %d  %.3f ms  blocks %llu  rounds wave: work %.0f wait %.0f cyc/block  producer: work %.0f wait %.0f cyc/block\n",
               rc, ms, (unsigned long long)pr[4], (double)pr[0] / pr[4], (double)pr[1] / pr[4],
               (double)pr[2] / pr[4], (double)pr[3] / pr[4]);
    }
    return 0;
}
