"""Phase breakdown of resolve_small on the 64 GiB headline stream (PBS_DEBUG_PHASES=1
makes the library print the kernel's wall_clock64 phase times to stderr)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "proxmox-backup_amd"))
import torch  # noqa: E402

import pbschunk  # noqa: E402

torch.cuda.set_device(0)
size = 64 << 30
st = torch.cuda.current_stream()
buf = torch.empty(size, dtype=torch.uint8, device="cuda")
pbschunk.generate_device(buf.data_ptr(), size, pbschunk.GEN_VMIMAGE, 0x5EED0003, 0, st.cuda_stream)
ch = pbschunk.Chunker(4 << 20)
ch.set_stream(st.cuda_stream)
for _ in range(5):
    ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
    print(ch.last_timing(), flush=True)
