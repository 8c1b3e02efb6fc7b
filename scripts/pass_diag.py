"""Per-pass time split (scan / exact / resolve / whole pass) of one stream under several
knob settings (DIAG_CONFIGS: ';'-separated, each a ','-separated list of VAR=VALUE;
default multi-launch vs fused pass), alternating in one process so every setting sees the
same buffer and clock history.  usage: python scripts/pass_diag.py SIZE_GIB WORKLOAD AVG [STEPS]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "proxmox-backup_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import pbschunk  # noqa: E402

if os.environ.get("DIAG_LIB"):  # noqa: SIM102  # another build of the library (A/B across builds)
    pbschunk.LIB_PATH = os.path.abspath(os.environ["DIAG_LIB"])

size_gib, workload, avg = float(sys.argv[1]), sys.argv[2], int(sys.argv[3])
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 30
gen = {"random": (pbschunk.GEN_RANDOM, 0x5EED0002), "vmimage": (pbschunk.GEN_VMIMAGE, 0x5EED0003)}[workload]
torch.cuda.set_device(0)
size = int(size_gib * (1 << 30)) // 8 * 8
st = torch.cuda.current_stream()
buf = torch.empty(size, dtype=torch.uint8, device="cuda")
pbschunk.generate_device(buf.data_ptr(), size, gen[0], gen[1], 0, st.cuda_stream)
torch.cuda.synchronize()
ch = pbschunk.Chunker(avg)
ch.set_stream(st.cuda_stream)
ref = None
BASE_ENV = dict(os.environ)
for w in range(20):  # clock ramp
    ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
for rnd in range(3):
    for cfg in os.environ.get("DIAG_CONFIGS", "PBS_FUSED=0;PBS_FUSED=1").split(";"):
        os.environ.clear()  # each setting starts from the launch environment
        os.environ.update(BASE_ENV)
        for kv in cfg.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
        ch.close()
        ch = pbschunk.Chunker(avg)
        ch.set_stream(st.cuda_stream)
        rows, walls = [], []
        for s in range(steps + 3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cuts = ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
            walls.append(time.perf_counter() - t0)
            rows.append(ch.last_timing())
        rows, walls = rows[3:], walls[3:]
        if ref is None:
            ref = cuts
        assert np.array_equal(cuts, ref), "cut lists differ between modes"
        m = lambda k: float(np.mean([r[k] for r in rows]))  # noqa: E731
        wall = float(np.mean(walls)) * 1e3
        print(f"round {rnd} {cfg}: fused={rows[-1]['fused'] > 0} pass {wall:.4f} ms "
              f"({size / (1 << 30) / wall * 1e3:.1f} GiB/s) | scan {m('scan_ms'):.4f} exact {m('exact_ms'):.4f} "
              f"resolve {m('resolve_ms'):.4f} total {m('total_ms'):.4f} | suspects {rows[-1]['suspects']} "
              f"candidates {rows[-1]['candidates']} cuts {cuts.size}", flush=True)
