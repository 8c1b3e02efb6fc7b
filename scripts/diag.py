import sys, os
sys.path.insert(0, 'proxmox-backup_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import numpy as np
import torch
import oracle, pbschunk, gen_np
MiB, KiB = 1 << 20, 1 << 10

def cmp(name, got, ref):
    ok = np.array_equal(got, ref)
    print(f"{name}: ok={ok} got={got.size} ref={ref.size}", flush=True)
    if not ok:
        sg, sr = set(got.tolist()), set(ref.tolist())
        print("   missing:", sorted(sr - sg)[:10], " extra:", sorted(sg - sr)[:10], flush=True)
    return ok

for n, avg, name in [(300 * KiB, 4096, "exact-only 300K"), (100, 64, "tiny"), (1 * MiB, 4096, "1 tile"),
                     (3 * MiB + 77, 4096, "3 tiles+tail"), (3 * MiB + 77, 64 * KiB, "3 tiles 64K"),
                     (8 * MiB, 256 * KiB, "8 tiles 256K")]:
    d = gen_np.gen_random(n, 0x5EED0002)
    cmp("cand " + name, pbschunk.candidates_host(d, avg), oracle.candidates(avg, d))
d = gen_np.gen_random(6 * MiB + 8, 7)
ref = oracle.chunk_feed(64 * KiB, d)
with pbschunk.Chunker(64 * KiB) as c:
    got = c.find_cuts(d, is_final=False)
    print(c.last_timing())
cmp("find_cuts host", got, ref)
cand = oracle.candidates(64 * KiB, d)
print("oracle cands", cand.size, cand[:8])
print("ref cuts", ref[:8], "got", got[:8])
