"""A/B of the blob-CRC chunk order (PBS_CRC_DYN 0 = static stride, 1 = counter), same
process, the 64 GiB VM-image stream's chunks (4 MiB average), CRCs asserted equal."""
import os
import sys

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
ends = ch.find_cuts_device(buf.data_ptr(), size, is_final=True)
bounds = np.concatenate([[0], ends]).astype(np.uint64)
n = bounds.size - 1
lens = np.diff(bounds.astype(np.int64))
order = np.argsort(-lens, kind="stable").astype(np.int32)
bd = torch.from_numpy(bounds.view(np.int64)).cuda()
od = torch.from_numpy(order).cuda()
out = torch.empty(n, dtype=torch.int32, device="cuda")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
res = {"0": [], "1": []}
ref = None
for rep in range(8):
    for m in ("0", "1"):
        os.environ["PBS_CRC_DYN"] = m
        ev[0].record(st)
        pbschunk.crc32_chunks_async(buf.data_ptr(), size, bd.data_ptr(), od.data_ptr(), n, out.data_ptr(),
                                    hip_stream=st.cuda_stream)
        ev[1].record(st)
        torch.cuda.synchronize()
        res[m].append(ev[0].elapsed_time(ev[1]))
        got = out.cpu().numpy()
        if ref is None:
            ref = got
        assert np.array_equal(got, ref)
for m, v in res.items():
    v = sorted(v[1:])
    print(f"PBS_CRC_DYN={m}: ms min {v[0]:.3f} median {v[len(v)//2]:.3f} -> {size / (1 << 30) / (v[len(v)//2] / 1e3):.0f} GiB/s")
