"""A/B of scan_main tile orders (PBS_SCAN_DYN) and segment caps (PBS_MAX_SEG), same
process, same VM-image buffer, modes alternating; cut lists must agree.
usage: ab_dyn.py <GiB> <avg> <mode> [<mode> ...]   mode = "<dyn 0|1>:<max seg>[:<small tiles 0|1>]"."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbschunk  # noqa: E402

torch.cuda.set_device(0)
size = int(float(sys.argv[1]) * (1 << 30))
avg = int(sys.argv[2])
modes = sys.argv[3:] or ["0:32768", "1:32768"]
st = torch.cuda.current_stream()
buf = torch.empty(size, dtype=torch.uint8, device="cuda")
kind = os.environ.get("AB_WORKLOAD", "vmimage")
pbschunk.generate_device(buf.data_ptr(), size, pbschunk.GEN_RANDOM if kind == "random" else pbschunk.GEN_VMIMAGE,
                         0x5EED0002 if kind == "random" else 0x5EED0003, 0, st.cuda_stream)
ch = pbschunk.Chunker(avg)
ch.set_stream(st.cuda_stream)
torch.cuda.synchronize()
res = {m: [] for m in modes}
ref = None
for rep in range(10):
    for m in modes:
        f = m.split(":")
        os.environ["PBS_SCAN_DYN"] = f[0]
        os.environ["PBS_MAX_SEG"] = f[1]
        os.environ["PBS_SCAN_SMALL"] = f[2] if len(f) > 2 else "1"
        cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
        t = ch.last_timing()
        if ref is None:
            ref = cuts
        assert np.array_equal(cuts, ref), "cut lists differ"
        res[m].append((t["scan_ms"], t["total_ms"]))
for m, v in res.items():
    s = sorted(x[0] for x in v[1:])
    p = sorted(x[1] for x in v[1:])
    print(f"{size >> 30} GiB avg {avg} dyn:seg={m}: scan_ms min {s[0]:.3f} median {s[len(s)//2]:.3f} | "
          f"pass_ms min {p[0]:.3f} median {p[len(p)//2]:.3f}", flush=True)
