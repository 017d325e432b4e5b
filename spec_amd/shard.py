"""Record sharding across GPUs (one process per GPU) and the column gather of BASELINE config 5.

Records are independent: a batch splits into contiguous record ranges, one
per rank, with no data-path collective.  `shard_bounds` gives rank k's records;
`shard_batch` cuts its bytes and rebases its `ends`; decoded string/bytes spans then point
into the rank's shard (a span's global offset = shard byte base + off: a 16M-record batch is
> 4 GiB, beyond 32-bit offsets, so spans stay shard-relative and the bases travel alongside).

The one collective of config 5 gathers every rank's decoded columns to rank 0.  Each rank's
columns and status live in ONE packed buffer (`PackedColumns`: column 0 of all records, then
column 1, ..., then the status bytes), which the decode kernel writes directly, so the gather
is a single `dist.gather` per rank — on backend "nccl" (RCCL over xGMI on MI355X) torch runs it
as grouped ncclSend/ncclRecv; "gloo" (CPU tests) gets host copies.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from .schema import Schema


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


PACK_ALIGN = 256  # column starts in a packed buffer: aligned for the kernels' 4/8/16-byte stores


def packed_layout(widths, n: int):
    """Byte offsets of the columns of n records packed one after another (each start rounded up
    to PACK_ALIGN), then the status bytes: -> (column offsets, status offset, total bytes)."""
    offs, off = [], 0
    for w in widths:
        offs.append(off)
        off = (off + n * w + PACK_ALIGN - 1) // PACK_ALIGN * PACK_ALIGN
    return offs, off, off + n


class PackedColumns:
    """Decoded columns + status of n records in one contiguous uint8 buffer (record-major per
    column, every column starting on a PACK_ALIGN boundary): `cols[f]` is a [n, width_f] view,
    `status` a [n] view.  Pass `cols`/`status` to spec_amd.Decoder so the decode writes the
    packed layout directly."""

    def __init__(self, schema: Schema, n: int, device="cuda", buf: torch.Tensor | None = None):
        self.schema, self.n = schema, n
        offs, soff, self.nbytes = packed_layout(schema.widths, n)
        self.buf = buf if buf is not None else torch.empty(max(self.nbytes, 1), dtype=torch.uint8, device=device)
        if self.buf.numel() < self.nbytes:
            raise ValueError("packed buffer too small")
        self.cols = [self.buf[o: o + n * w].view(n, w) for o, w in zip(offs, schema.widths)]
        self.status = self.buf[soff: soff + n]

    @staticmethod
    def nbytes_for(schema: Schema, n: int) -> int:
        return packed_layout(schema.widths, n)[2]


def _gather_sizes(nbytes: int, dist, group, device):
    t = torch.tensor([nbytes], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(sizes, t, group=group)
    return [int(s.item()) for s in sizes]


def gather_packed(buf: torch.Tensor, dist, dst: int = 0, group=None, sizes=None):
    """Gather every rank's packed uint8 buffer to rank `dst` with ONE collective.  Buffers may
    differ in size (padded to the largest for the collective, trimmed after); pass `sizes`
    (bytes per rank) when known to skip the size exchange.  Returns the per-rank buffers on
    dst (a list of 1-D uint8 tensors), None elsewhere."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    on_host = dist.get_backend(group) == "gloo"
    src = buf.reshape(-1)
    if on_host and src.is_cuda:
        src = src.cpu()
    if sizes is None:
        sizes = _gather_sizes(src.numel(), dist, group, src.device)
    nmax = max(sizes) if sizes else 0
    if src.numel() < nmax:  # collectives need equal shapes
        pad = torch.zeros(nmax, dtype=torch.uint8, device=src.device)
        pad[: src.numel()] = src
        src = pad
    bufs = [torch.empty(nmax, dtype=torch.uint8, device=src.device) for _ in range(world)] if rank == dst else None
    dist.gather(src, gather_list=bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return [b[: sizes[k]] for k, b in enumerate(bufs)]


def gather_columns(cols, dist, dst: int = 0, group=None):
    """Gather every rank's decoded columns (list of uint8 [n_k, w] tensors) to rank `dst`,
    packed into one buffer per rank (one collective).  Returns on dst a list (per column) of
    per-rank [n_k, w] tensors, else None.  Every rank must pass the same column widths."""
    if not cols:
        return [] if dist.get_rank(group) == dst else None
    widths = [int(c.shape[1]) for c in cols]
    n_local = int(cols[0].shape[0])
    offs, cbytes, _ = packed_layout(widths, n_local)
    packed = cols[0].new_zeros(cbytes + 8)  # the columns, then the record count (int64)
    for o, c in zip(offs, cols):
        packed[o: o + c.numel()] = c.reshape(-1)
    packed[cbytes:].view(torch.int64)[0] = n_local
    parts = gather_packed(packed, dist, dst, group)
    if parts is None:
        return None
    out = [[] for _ in cols]
    for p in parts:
        n_k = int(p[-8:].cpu().view(torch.int64)[0])
        po, _, _ = packed_layout(widths, n_k)
        for f, w in enumerate(widths):
            out[f].append(p[po[f]: po[f] + n_k * w].view(n_k, w))
    return out


class NativeShard:
    """One process driving several devices through the C ABI (include/spec_amd.h spec_shard_*):
    a stream and an RCCL communicator per device, shards decoded into packed buffers
    (PackedColumns' layout, spec_packed_layout), one grouped RCCL send/recv gather to a root
    device.  What a cgo caller of INTEGRATION.md drives, without torch.distributed."""

    def __init__(self, devices):
        from . import _lib

        self._lib = _lib
        self.devices = list(devices)
        arr = (C.c_int * len(self.devices))(*self.devices)
        self._h = C.c_void_p()
        _lib.check(_lib.lib().spec_shard_create(arr, len(self.devices), C.byref(self._h)), "spec_shard_create")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and h.value:
            try:
                self._lib.lib().spec_shard_destroy(h)
            except Exception:
                pass

    @property
    def ndev(self) -> int:
        return len(self.devices)

    def bounds(self, n: int, k: int):
        r0, r1 = C.c_uint64(), C.c_uint64()
        self._lib.lib().spec_shard_bounds(n, self.ndev, k, C.byref(r0), C.byref(r1))
        return r0.value, r1.value

    def decode_host(self, schema: Schema, stream: np.ndarray, ends: np.ndarray):
        """Split a host batch over the devices, decode each shard on its device: -> (packed
        buffers [PackedColumns per device], byte bases)."""
        stream = np.ascontiguousarray(stream, dtype=np.uint8)
        ends = np.ascontiguousarray(ends, dtype=np.uint64)
        n = len(ends)
        packs = []
        for k, d in enumerate(self.devices):
            r0, r1 = self.bounds(n, k)
            packs.append(PackedColumns(schema, r1 - r0, torch.device("cuda", d)))
        ptrs = (C.c_void_p * self.ndev)(*[p.buf.data_ptr() for p in packs])
        bases = (C.c_uint64 * self.ndev)()
        rc = self._lib.lib().spec_shard_decode_host(self._h, C.byref(schema.c), stream.ctypes.data, stream.size,
                                                    ends.ctypes.data, n, ptrs, bases)
        self._lib.check(rc, "spec_shard_decode_host")
        self._keep = (stream, ends)
        return packs, list(bases)

    def gather(self, packs, root: int = 0) -> torch.Tensor:
        """Every device's packed buffer to one buffer on device `root` (parts back to back)."""
        sizes = [p.nbytes for p in packs]
        out = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device=torch.device("cuda", self.devices[root]))
        ptrs = (C.c_void_p * self.ndev)(*[p.buf.data_ptr() for p in packs])
        nb = (C.c_uint64 * self.ndev)(*sizes)
        self._lib.check(self._lib.lib().spec_shard_gather(self._h, nb, ptrs, root, C.c_void_p(out.data_ptr())),
                        "spec_shard_gather")
        return out

    def sync(self):
        self._lib.check(self._lib.lib().spec_shard_sync(self._h), "spec_shard_sync")
