"""Per-wave timeline of scan_fused_kernel from the probe build (make -C
scripts/microbench/probe): start, tiles done, tail items done, per scanner wave.
usage: python fused_probe.py SIZE_GIB WORKLOAD AVG  (env PBS_SCAN_DYN etc. pass through;
PBS_FUSED=1 is set here)"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "proxmox-backup_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbschunk  # noqa: E402

os.environ["PBS_FUSED"] = "1"
pbschunk.LIB_PATH = os.path.join(HERE, "probe", "libpbschunk_probe.so")
L = pbschunk.lib()
size_gib, workload, avg = float(sys.argv[1]), sys.argv[2], int(sys.argv[3])
gen = {"random": (pbschunk.GEN_RANDOM, 0x5EED0002), "vmimage": (pbschunk.GEN_VMIMAGE, 0x5EED0003)}[workload]
torch.cuda.set_device(0)
size = int(size_gib * (1 << 30)) // 8 * 8
st = torch.cuda.current_stream()
buf = torch.empty(size, dtype=torch.uint8, device="cuda")
pbschunk.generate_device(buf.data_ptr(), size, gen[0], gen[1], 0, st.cuda_stream)
ch = pbschunk.Chunker(avg)
ch.set_stream(st.cuda_stream)
for _ in range(10):
    ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
pr = np.zeros(4 * 4096, dtype=np.uint64)
nw = 2048
for rep in range(3):
    ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
    t = ch.last_timing()
    assert L.pbs_fused_probe_read(ctypes.c_void_p(pr.ctypes.data)) == 0
    sta, til, don, sim = (pr[k * 4096:k * 4096 + nw].astype(np.int64) for k in range(4))
    if rep == 0:
        print("SIMD|partner<<8 of the waves of workgroups 0-2:", [hex(x) for x in sim[:24]], flush=True)
    scan = np.ones(nw, bool)
    scan[:3] = False  # workgroup 0's resolver waves
    t0 = sta[scan].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731  (100 MHz)
    s, ti, d = us(sta[scan]), us(til[scan]), us(don[scan])
    q = lambda v: " ".join(f"{np.percentile(v, p):.0f}" for p in (0, 10, 50, 90, 100))  # noqa: E731
    wv = np.arange(nw)[scan] % 8
    per_w = " ".join(f"{np.median(ti[wv == w]):.0f}" for w in range(8))
    wg0 = ti[np.arange(nw)[scan] < 8]
    # SIMD pairs (w, partner): finish of the later minus the earlier, per pair
    idx = np.arange(nw)
    part = (sim >> 8) & 0xFF
    pw = [(i, (i // 8) * 8 + part[i]) for i in idx if i >= 8 and part[i] > i % 8]
    gap = np.array([abs(til[i] - til[j]) / 100.0 for i, j in pw])
    print(f"rep {rep}: pair finish gap us p10/med/p90 {np.percentile(gap, 10):.0f} {np.median(gap):.0f} "
          f"{np.percentile(gap, 90):.0f}", flush=True)
    print(f"rep {rep}: kernel {t['scan_ms'] * 1e3:.0f} us fused={t['fused'] > 0} | start spread {s.max():.1f} us | "
          f"tiles done min/p10/med/p90/max {q(ti)} | all done {q(d)} | median tiles-done by wave-in-WG {per_w} | "
          f"WG0 scanners {' '.join(f'{x:.0f}' for x in wg0)}", flush=True)
