"""One stream chunked by several GPUs ("single stream across GPUs").

Rank r holds the contiguous stream range [base_r, base_r + len_r) in its HBM.  The cut
test at position p depends only on the 64 bytes ending at p (pbs-datastore/src/
chunker.rs:146: once the window is full, rotl by 64 is the identity), so:

  1. halo:    every rank receives the 63 bytes before its range from its left
              neighbour (one all-gather of 63-byte tails: a few hundred bytes);
  2. phase A: every rank scans its own range (pbs_chunker_candidates_device) and gets
              its sorted absolute candidate positions -- no data-path traffic;
  3. gather:  one all-gather of the candidate lists (KiBs: ~1.5 per avg bytes), whose
              concatenation in rank order is the stream's sorted list;
  4. phase B: the min/max rule (chunker.rs:172-183) is resolved over the whole list
              (pbs_chunker_resolve_device) on every rank, so each has the cut list.

The result equals one chunker over the concatenated stream (tests/test_shard.py).
Collectives go through ``torch.distributed`` (RCCL over xGMI with the "nccl" backend on
the GPU box, gloo in the CPU tests); nothing else crosses GPUs.  gloo reduces CPU tensors
only, so with a gloo group (the CPU tests, and bench.py's one-GPU rehearsal) the halo and
the candidate lists are staged through host memory around each collective.
"""
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

HALO = 63  # window - 1 bytes of history a range needs


def shard_ranges(total: int, world: int, align: int = 8) -> List[Tuple[int, int]]:
    """Contiguous [base, base + len) ranges of a ``total``-byte stream, one per rank,
    ``align``-aligned starts; the last rank takes the remainder."""
    per = (total // world) // align * align
    out = []
    for r in range(world):
        base = r * per
        ln = per if r < world - 1 else total - base
        out.append((base, ln))
    return out


def collective_device(dist, device):
    """Where the collectives' tensors must live: the data's device for RCCL ("nccl"),
    the host for gloo (which does not take device tensors)."""
    import torch

    if dist is not None and dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def _live(dist) -> bool:
    """A process group to run collectives in (the torch.distributed module passed without
    an initialised group, or None, means one rank: nothing to exchange)."""
    return dist is not None and dist.is_initialized()


def exchange_halo(tail: "torch.Tensor", dist, rank: int, world: int) -> bytes:
    """All-gather every rank's last <= 63 bytes and return the left neighbour's (b"" on
    rank 0)."""
    import torch

    if not _live(dist):
        if int(tail.numel()) > HALO:
            raise ValueError("tail longer than the halo")
        return b""
    tail = tail.to(collective_device(dist, tail.device))
    buf = torch.zeros(HALO + 1, dtype=torch.uint8, device=tail.device)
    n = int(tail.numel())
    if n > HALO:
        raise ValueError("tail longer than the halo")
    buf[:n] = tail
    buf[HALO] = n
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    if rank == 0:
        return b""
    left = parts[rank - 1].cpu().numpy()
    return left[: int(left[HALO])].tobytes()


def gather_candidates(cand: "torch.Tensor", dist, world: int) -> "torch.Tensor":
    """All-gather variable-length int64 candidate lists and concatenate in rank order
    (the result on ``cand``'s device)."""
    import torch

    if not _live(dist):
        return cand
    home = cand.device
    cand = cand.to(collective_device(dist, home))
    cnt = torch.tensor([cand.numel()], dtype=torch.int64, device=cand.device)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    width = max(1, max(counts))
    pad = torch.zeros(width, dtype=torch.int64, device=cand.device)
    pad[: cand.numel()] = cand
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)]).to(home)


def phase_a(ch, dev_ptr: int, length: int, base: int, pre: bytes, device,
            cap_hint: Optional[int] = None) -> "torch.Tensor":
    """Sorted absolute candidates of this rank's range as an int64 tensor on ``device``
    (grows the output once if the first capacity guess is short)."""
    import torch

    cap = cap_hint if cap_hint is not None else max(1024, length // 4096)
    for _ in range(2):
        out = torch.empty(cap, dtype=torch.int64, device=device)
        try:
            n = ch.candidates_device(dev_ptr, length, pre, base, out.data_ptr(), cap)
            return out[:n]
        except Exception as e:  # ChunkerError with .needed on PBS_ERR_CAPACITY
            needed = getattr(e, "needed", None)
            if needed is None or needed <= cap:
                raise
            cap = needed
    raise RuntimeError("candidate capacity did not converge")


def chunk_sharded(ch, dev_ptr: int, length: int, base: int, total: int, tail: "torch.Tensor",
                  dist, rank: int, world: int, device, is_final: bool = True) -> np.ndarray:
    """Cut list of the whole ``total``-byte stream, computed from this rank's range
    [base, base + length) (device bytes at ``dev_ptr``) and the other ranks'.
    ``tail`` = this range's last min(length, 63) bytes as a tensor on the collective's
    device (the halo the right neighbour needs).

    The handle is put on torch's current stream of ``device``: the gathered candidate
    list is written there (all_gather + cat), and the handle's own stream is
    non-blocking (include/pbs_chunker.h), so resolving on it could read the list before
    it is complete."""
    import torch

    if getattr(device, "type", None) == "cuda":
        ch.set_stream(torch.cuda.current_stream(device).cuda_stream)
    pre = exchange_halo(tail, dist, rank, world)
    if len(pre) != min(base, HALO):
        raise ValueError(f"rank {rank}: halo of {len(pre)} bytes for base {base}")
    cand = phase_a(ch, dev_ptr, length, base, pre, device)
    allc = gather_candidates(cand, dist, world)
    allc = allc.contiguous()
    return ch.resolve_device(allc.data_ptr(), int(allc.numel()), total, is_final)
