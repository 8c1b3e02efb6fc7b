"""Per-pass host overhead of the 64 GiB headline pass: wall time of find_cuts_device
(Python -> C ABI -> kernels -> sync -> cut list) against the device span (events from
the first launch to the end of resolve_small) and the scan kernel alone."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbschunk  # noqa: E402

torch.cuda.set_device(0)
size = 64 << 30
st = torch.cuda.current_stream()
buf = torch.empty(size, dtype=torch.uint8, device="cuda")
pbschunk.generate_device(buf.data_ptr(), size, pbschunk.GEN_VMIMAGE, 0x5EED0003, 0, st.cuda_stream)
ch = pbschunk.Chunker(4 << 20)
ch.set_stream(st.cuda_stream)
torch.cuda.synchronize()
rows = []
for i in range(25):
    t0 = time.perf_counter()
    ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
    wall = (time.perf_counter() - t0) * 1e3
    t = ch.last_timing()
    rows.append((wall, t["total_ms"], t["scan_ms"]))
r = np.array(rows[3:])
print("wall ms  median %.3f min %.3f max %.3f" % (np.median(r[:, 0]), r[:, 0].min(), r[:, 0].max()))
print("device   median %.3f (first launch .. resolve end)" % np.median(r[:, 1]))
print("scan     median %.3f" % np.median(r[:, 2]))
print("host-only (wall - device) median %.3f min %.3f max %.3f" % (np.median(r[:, 0] - r[:, 1]), (r[:, 0] - r[:, 1]).min(), (r[:, 0] - r[:, 1]).max()))
