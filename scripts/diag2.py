import sys
sys.path.insert(0, 'proxmox-backup_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import numpy as np
import torch  # noqa
import oracle, pbschunk, gen_np
MiB, KiB = 1 << 20, 1 << 10
for n, avg, seed in [(2 * MiB + 5, 128, 3), (2 * MiB, 128, 3), (2 * MiB, 256, 3), (2 * MiB, 64, 3), (4 * MiB, 128, 3), (2 * MiB + 5, 4096, 3)]:
    d = gen_np.gen_random(n, seed)
    got = pbschunk.candidates_host(d, avg)
    ref = oracle.candidates(avg, d)
    sg, sr = set(got.tolist()), set(ref.tolist())
    miss, extra = sorted(sr - sg), sorted(sg - sr)
    print(f"n={n} avg={avg}: got={got.size} ref={ref.size} missing={len(miss)} extra={len(extra)} dup={got.size - len(sg)}")
    if miss or extra:
        seg = 4096
        print("   missing:", miss[:8], "mod seg:", [m % seg for m in miss[:8]], "lane:", [(m // seg) % 64 for m in miss[:8]])
        print("   extra:", extra[:8])
