"""Per-wave start/finish spread of scan_main on the 64 GiB headline stream, static vs
dynamic tile order, from the probe build (make -C scripts/microbench/probe)."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "proxmox-backup_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbschunk  # noqa: E402

pbschunk.LIB_PATH = os.path.join(HERE, "probe", "libpbschunk_probe.so")
L = pbschunk.lib()
torch.cuda.set_device(0)
size = 64 << 30
st = torch.cuda.current_stream()
buf = torch.empty(size, dtype=torch.uint8, device="cuda")
pbschunk.generate_device(buf.data_ptr(), size, pbschunk.GEN_VMIMAGE, 0x5EED0003, 0, st.cuda_stream)
ch = pbschunk.Chunker(4 << 20)
ch.set_stream(st.cuda_stream)
pr = np.zeros(8192, dtype=np.uint64)
for rep in range(3):
    for mode in ("0", "1"):
        os.environ["PBS_SCAN_DYN"] = mode
        ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
        ms = ch.last_timing()["scan_ms"]
        assert L.pbs_scan_probe_read(ctypes.c_void_p(pr.ctypes.data)) == 0
        fin, sta = pr[:2048].astype(np.int64), pr[4096:4096 + 2048].astype(np.int64)
        t0 = sta.min()
        f = (fin - t0) / 100.0  # us (100 MHz)
        s = (sta - t0) / 100.0
        per_xcd = [float(np.median(f[np.arange(2048) // 8 % 8 == x])) for x in range(8)]
        print(f"dyn={mode} scan {ms:.3f} ms | start spread {s.max():.1f} us | finish min {f.min():.0f} "
              f"p10 {np.percentile(f, 10):.0f} median {np.median(f):.0f} p90 {np.percentile(f, 90):.0f} "
              f"max {f.max():.0f} us | median finish per (block % 8) {' '.join(f'{x:.0f}' for x in per_xcd)}",
              flush=True)
