"""Record sharding across GPUs (one process per GPU) and the column gather of BASELINE config 5.

Records are independent: a batch splits into contiguous record ranges, one
per rank, with no data-path collective.  `shard_bounds` gives rank k's records;
`shard_batch` cuts its bytes and rebases its `ends`; decoded string/bytes spans then point
into the rank's shard (a span's global offset = shard byte base + off: a 16M-record batch is
> 4 GiB, beyond 32-bit offsets, so spans stay shard-relative and the bases travel alongside).
`gather_columns` is the one collective of config 5: every rank's columns to rank 0
(torch.distributed, backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests).
"""
from __future__ import annotations

import numpy as np
import torch


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous record range [r0, r1) of rank `rank` (sizes differ by at most one)."""
    return n * rank // world, n * (rank + 1) // world


def shard_batch(stream, ends, world: int, rank: int):
    """-> (stream slice, rebased ends, byte base, (r0, r1)) for numpy arrays or tensors."""
    n = len(ends)
    r0, r1 = shard_bounds(n, world, rank)
    b0 = int(ends[r0 - 1]) if r0 else 0
    b1 = int(ends[r1 - 1]) if r1 else 0
    s = stream[b0:b1]
    e = ends[r0:r1] - (np.uint64(b0) if isinstance(ends, np.ndarray) else b0)
    return s, e, b0, (r0, r1)


def gather_columns(cols, dist, dst: int = 0, group=None):
    """Gather every rank's decoded columns (list of uint8 [n_k, w] tensors, equal n_k or not)
    to rank `dst`.  Returns on dst a list (per column) of per-rank tensors, else None."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_local = torch.tensor([cols[0].shape[0] if cols else 0], dtype=torch.int64, device=cols[0].device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    nmax = max(sizes)
    out = [] if rank == dst else None
    for c in cols:
        pad = c
        if c.shape[0] < nmax:  # collectives need equal shapes: pad, trim after
            pad = torch.zeros((nmax, c.shape[1]), dtype=c.dtype, device=c.device)
            pad[: c.shape[0]] = c
        bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
        dist.gather(pad, gather_list=bufs, dst=dst, group=group)
        if rank == dst:
            out.append([b[: sizes[k]] for k, b in enumerate(bufs)])
    return out
