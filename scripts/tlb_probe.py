"""Experiment: is the per-allocation speed of the 64 GiB scan a translation (TLB)
effect?  Two 64 GiB buffers, each scanned 4 times (scan kernel dispatches alternate
buffer 0 x4, buffer 1 x4); run under rocprofv3 --pmc with UTCL1 counters."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
import torch  # noqa: E402

import pbschunk  # noqa: E402

torch.cuda.set_device(0)
size = 64 << 30
st = torch.cuda.current_stream()
ch = pbschunk.Chunker(4 << 20)
ch.set_stream(st.cuda_stream)
bufs = []
for a in range(2):
    bufs.append(torch.empty(size, dtype=torch.uint8, device="cuda"))
    pbschunk.generate_device(bufs[-1].data_ptr(), size, 2, 0x5EED0003, 0, st.cuda_stream)
torch.cuda.synchronize()
for a, b in enumerate(bufs):
    for k in range(4):
        ch.find_cuts_device(b.data_ptr(), size, is_final=True)
        print(f"buf {a} ptr {b.data_ptr():#x} scan_ms {ch.last_timing()['scan_ms']:.3f}", flush=True)
