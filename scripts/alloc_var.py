"""Experiment: per-allocation vs per-run variance of the 64 GiB scan (same process)."""
import sys, os, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
import torch
import pbschunk

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
for rep in range(3):
    for a, b in enumerate(bufs):
        ms = []
        for k in range(8):
            ch.find_cuts_device(b.data_ptr(), size, is_final=True)
            ms.append(ch.last_timing()["scan_ms"])
        print(f"rep {rep} buf {a} ptr {b.data_ptr():#x} scan_ms min {min(ms):.3f} avg {sum(ms[2:])/6:.3f}", flush=True)
