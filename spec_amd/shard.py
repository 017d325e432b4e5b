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
    device, sharded encode with one host scan of the shard totals, and the pinned host pipeline
    on every device at once.  What a cgo caller of INTEGRATION.md drives, without
    torch.distributed.

    `force_comm` builds the RCCL communicator even for one device (SPEC_SHARD_FORCE_COMM): the
    gather then moves every part through ncclSend/ncclRecv, the root's own as a send to itself.
    `shared` lets devices repeat (SPEC_SHARD_SHARED: several shards per GPU, no communicator),
    so the N-shard flow runs on a one-GPU box.

    The shard's work runs on its own per-device streams.  Every call below first makes each shard
    stream wait for the device's current torch stream (inputs torch just produced are complete),
    and afterwards makes the current torch stream wait for the shard stream, so torch code after
    the call sees finished data; the tensors a call touched are referenced until sync() (or the
    object's end, which synchronises first), so the caching allocator cannot hand their memory
    out while the shard still reads or writes it.  (No record_stream: the shard's streams may
    end before the tensors do.)"""

    def __init__(self, devices, force_comm: bool = False, shared: bool = False):
        from . import _lib

        self._lib = _lib
        self.devices = list(devices)
        arr = (C.c_int * len(self.devices))(*self.devices)
        self._h = C.c_void_p()
        flags = (1 if force_comm else 0) | (2 if shared else 0)  # SPEC_SHARD_FORCE_COMM, SPEC_SHARD_SHARED
        _lib.check(_lib.lib().spec_shard_create_ex(arr, len(self.devices), flags, C.byref(self._h)),
                   "spec_shard_create_ex")
        self._ext = [torch.cuda.ExternalStream(self._lib.lib().spec_shard_stream(self._h, k),
                                               device=torch.device("cuda", d))
                     for k, d in enumerate(self.devices)]
        self._inflight = []
        self._host = None  # (schema, per-device host decoders) after host_prepare

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and h.value:
            try:
                self._lib.lib().spec_shard_destroy(h)  # drains every stream first
            except Exception:
                pass
        self._inflight = []

    @property
    def ndev(self) -> int:
        return len(self.devices)

    @property
    def has_comm(self) -> bool:
        return bool(self._lib.lib().spec_shard_has_comm(self._h))

    @staticmethod
    def rccl_version() -> int:
        from . import _lib

        return int(_lib.lib().spec_shard_rccl_version())

    def stream(self, k: int) -> torch.cuda.ExternalStream:
        return self._ext[k]

    def set_chunks(self, chunks: int):
        self._lib.check(self._lib.lib().spec_shard_set_chunks(self._h, chunks), "spec_shard_set_chunks")

    def set_split(self, by_bytes: bool):
        """How decode_host / host_decode split a host batch: near-equal record counts (default)
        or near-equal bytes (spec_shard_bounds_bytes over the batch's ends)."""
        self._lib.check(self._lib.lib().spec_shard_set_split(self._h, 1 if by_bytes else 0), "spec_shard_set_split")
        self._by_bytes = bool(by_bytes)

    def bounds(self, n: int, k: int, ends=None):
        """Shard k's records [r0, r1) of n.  With the byte split, pass the batch's ends (host)."""
        r0, r1 = C.c_uint64(), C.c_uint64()
        if getattr(self, "_by_bytes", False):
            if ends is None:
                raise ValueError("byte-balanced bounds need the batch's ends")
            e = np.ascontiguousarray(ends.numpy() if isinstance(ends, torch.Tensor) else ends).view(np.uint64)
            self._lib.lib().spec_shard_bounds_bytes(e.ctypes.data, n, self.ndev, k, C.byref(r0), C.byref(r1))
        else:
            self._lib.lib().spec_shard_bounds(n, self.ndev, k, C.byref(r0), C.byref(r1))
        return r0.value, r1.value

    def _enter(self):
        """Order every shard stream after its device's current torch stream."""
        for k, d in enumerate(self.devices):
            self._ext[k].wait_stream(torch.cuda.current_stream(torch.device("cuda", d)))

    def _join(self, tensors_per_dev):
        """Order torch's current stream of every device after the shard streams; keep the
        tensors referenced until sync()."""
        for k, d in enumerate(self.devices):
            torch.cuda.current_stream(torch.device("cuda", d)).wait_stream(self._ext[k])
        self._inflight.append(tensors_per_dev)

    def decode_host(self, schema: Schema, stream: np.ndarray | torch.Tensor, ends: np.ndarray | torch.Tensor,
                    packs=None):
        """Split a host batch over the devices, decode each shard on its device: -> (packed
        buffers [PackedColumns per device], byte bases).  `stream`/`ends` may be numpy arrays or
        (pinned) CPU tensors; they are kept alive until sync()."""
        if isinstance(stream, torch.Tensor):
            sp, slen = stream.data_ptr(), stream.numel()
        else:
            stream = np.ascontiguousarray(stream, dtype=np.uint8)
            sp, slen = stream.ctypes.data, stream.size
        if isinstance(ends, torch.Tensor):
            ep, n = ends.data_ptr(), ends.numel()
        else:
            ends = np.ascontiguousarray(ends, dtype=np.uint64)
            ep, n = ends.ctypes.data, len(ends)
        if packs is None:
            packs = []
            for k, d in enumerate(self.devices):
                r0, r1 = self.bounds(n, k, ends)
                packs.append(PackedColumns(schema, r1 - r0, torch.device("cuda", d)))
        ptrs = (C.c_void_p * self.ndev)(*[p.buf.data_ptr() for p in packs])
        bases = (C.c_uint64 * self.ndev)()
        self._enter()
        rc = self._lib.lib().spec_shard_decode_host(self._h, C.byref(schema.c), sp, slen, ep, n, ptrs, bases)
        self._lib.check(rc, "spec_shard_decode_host")
        self._join([[p.buf] for p in packs])
        self._inflight.append((stream, ends))
        return packs, list(bases)

    def decode(self, schema: Schema, streams, ends, packs):
        """Device-resident shards: device k decodes (streams[k], ends[k]) (ends relative to its
        stream) into packs[k] (PackedColumns on device k)."""
        k_ = self.ndev
        sp = (C.c_void_p * k_)(*[s.data_ptr() for s in streams])
        lens = (C.c_uint64 * k_)(*[s.numel() for s in streams])
        ep = (C.c_void_p * k_)(*[e.data_ptr() for e in ends])
        ns = (C.c_uint64 * k_)(*[e.numel() for e in ends])
        pp = (C.c_void_p * k_)(*[p.buf.data_ptr() for p in packs])
        self._enter()
        self._lib.check(self._lib.lib().spec_shard_decode(self._h, C.byref(schema.c), sp, lens, ep, ns, pp),
                        "spec_shard_decode")
        self._join([[s, e, p.buf] for s, e, p in zip(streams, ends, packs)])

    def gather(self, packs, root: int = 0, out: torch.Tensor | None = None, sizes=None) -> torch.Tensor:
        """Every device's packed buffer (or any uint8 device buffers, `sizes` bytes each) to one
        buffer on device `root` (parts back to back)."""
        bufs = [p.buf if isinstance(p, PackedColumns) else p for p in packs]
        if sizes is None:
            sizes = [p.nbytes if isinstance(p, PackedColumns) else p.numel() for p in packs]
        if out is None:
            out = torch.empty(max(sum(sizes), 1), dtype=torch.uint8, device=torch.device("cuda", self.devices[root]))
        ptrs = (C.c_void_p * self.ndev)(*[b.data_ptr() for b in bufs])
        nb = (C.c_uint64 * self.ndev)(*sizes)
        self._enter()
        self._lib.check(self._lib.lib().spec_shard_gather(self._h, nb, ptrs, root, C.c_void_p(out.data_ptr())),
                        "spec_shard_gather")
        self._join([list(bufs[k:k + 1]) + ([out] if k == root else []) for k in range(self.ndev)])
        return out

    def _encode_args(self, schema: Schema, shards):
        k_ = self.ndev
        if len(shards) != k_:
            raise ValueError("one shard per device")
        nf = max(1, len(schema))
        cols, hp, hl = [], [], []
        for k, (cs, heaps, n) in enumerate(shards):
            if len(cs) != len(schema):
                raise ValueError("one column per schema field")
            for f, c in enumerate(cs):
                if not c.is_cuda or c.device.index != self.devices[k]:
                    raise ValueError(f"shard {k} column {f} is not on device {self.devices[k]}")
                if c.numel() * c.element_size() < int(n) * schema.fields[f].width:
                    raise ValueError(f"shard {k} column {f} too small")
            cols.append((C.c_void_p * nf)(*[c.data_ptr() for c in cs]))
            h, l_ = (C.c_void_p * nf)(), (C.c_uint64 * nf)()
            for f, fld in enumerate(schema.fields):
                if f in (heaps or {}):
                    h[f], l_[f] = heaps[f].data_ptr(), heaps[f].numel()
            hp.append(h)
            hl.append(l_)
        ns = (C.c_uint64 * k_)(*[int(s[2]) for s in shards])
        colsp = (C.c_void_p * k_)(*[C.cast(c, C.c_void_p) for c in cols])
        hpp = (C.c_void_p * k_)(*[C.cast(h, C.c_void_p) for h in hp])
        hlp = (C.c_void_p * k_)(*[C.cast(h, C.c_void_p) for h in hl])
        return (cols, hp, hl), ns, colsp, hpp, hlp

    def encode(self, schema: Schema, shards, outs=None, ends=None):
        """Sharded encode: shards[k] = (columns, heaps, n) on device k (as spec_amd.encode_flat
        takes them).  -> (outs, ends, totals, byte_bases): device k's bytes outs[k][:totals[k]]
        and ends[k] = its records' ends in the WHOLE batch; the outs back to back are exactly
        one encode of the batch.  Without `outs`, the totals are found first (a call with no
        capacity) and the buffers allocated."""
        k_ = self.ndev
        keepalive, ns, colsp, hpp, hlp = self._encode_args(schema, shards)
        totals = (C.c_uint64 * k_)()
        bases = (C.c_uint64 * k_)()
        devs = [torch.device("cuda", d) for d in self.devices]
        if ends is None:
            ends = [torch.empty(max(int(s[2]), 1), dtype=torch.int64, device=dv) for s, dv in zip(shards, devs)]
        L = self._lib.lib()

        def call(bufs, caps):
            op = (C.c_void_p * k_)(*[b.data_ptr() for b in bufs])
            cp = (C.c_uint64 * k_)(*caps)
            ep = (C.c_void_p * k_)(*[e.data_ptr() for e in ends])
            return L.spec_shard_encode(self._h, C.byref(schema.c), colsp, hpp, hlp, ns, op, cp, ep, totals, bases)

        self._enter()
        if outs is None:
            probe = [torch.empty(1, dtype=torch.uint8, device=dv) for dv in devs]
            rc = call(probe, [0] * k_)
            if rc not in (0, -4):  # SPEC_E_CAPACITY: the totals are known
                self._lib.check(rc, "spec_shard_encode")
            outs = [torch.empty(max(int(t), 1), dtype=torch.uint8, device=dv) for t, dv in zip(totals, devs)]
        self._lib.check(call(outs, [o.numel() for o in outs]), "spec_shard_encode")
        keep = [list(s[0]) + list(s[1].values()) if isinstance(s[1], dict) else list(s[0]) for s in shards]
        self._join([[o, e] + [t for t in kk if isinstance(t, torch.Tensor)] for o, e, kk in zip(outs, ends, keep)])
        self._inflight.append(keepalive)
        return outs, ends, list(totals), list(bases)

    def encode_call(self, schema: Schema, shards, outs, ends):
        """A prepared spec_shard_encode over fixed buffers: -> fn() that issues it (the C ABI call
        alone, as a cgo caller issues it; no torch stream ordering: synchronise the inputs first)."""
        k_ = self.ndev
        keepalive, ns, colsp, hpp, hlp = self._encode_args(schema, shards)
        totals, bases = (C.c_uint64 * k_)(), (C.c_uint64 * k_)()
        op = (C.c_void_p * k_)(*[b.data_ptr() for b in outs])
        cp = (C.c_uint64 * k_)(*[b.numel() for b in outs])
        ep = (C.c_void_p * k_)(*[e.data_ptr() for e in ends])
        L, h, sc = self._lib.lib(), self._h, C.byref(schema.c)
        self._inflight.append((keepalive, shards, outs, ends))

        def fn():
            self._lib.check(L.spec_shard_encode(h, sc, colsp, hpp, hlp, ns, op, cp, ep, totals, bases),
                            "spec_shard_encode")

        return fn

    def host_prepare(self, schema: Schema, shard_records: int, shard_bytes: int, chunks: int = 8):
        """A spec_host_decoder per device for shards of up to shard_records / shard_bytes."""
        self._lib.check(self._lib.lib().spec_shard_host_prepare(self._h, C.byref(schema.c), shard_records,
                                                                shard_bytes, chunks), "spec_shard_host_prepare")
        self._host = schema

    def host_out_bytes(self, k: int, n: int) -> int:
        L = self._lib.lib()
        return int(L.spec_host_decoder_out_bytes(L.spec_shard_host_decoder(self._h, k), n))

    def host_chunk(self, k: int, n: int, j: int):
        """Chunk j of device k's host output for an n-record shard: (r0, r1, column offsets, status offset)."""
        L = self._lib.lib()
        nf = len(self._host)
        r0, r1, so = C.c_uint64(), C.c_uint64(), C.c_uint64()
        co = (C.c_uint64 * nf)()
        self._lib.check(L.spec_host_decoder_chunk(L.spec_shard_host_decoder(self._h, k), n, j, C.byref(r0),
                                                  C.byref(r1), co, C.byref(so)), "spec_host_decoder_chunk")
        return r0.value, r1.value, list(co), so.value

    def host_decode(self, stream: torch.Tensor, ends: torch.Tensor, outs):
        """Pinned host batch -> every device's host output buffer (outs[k], pinned uint8 tensors
        of host_out_bytes(k, n_k)), all devices at once.  Synchronous.  -> byte bases."""
        n = ends.numel()
        op = (C.c_void_p * self.ndev)(*[o.data_ptr() for o in outs])
        bases = (C.c_uint64 * self.ndev)()
        self._lib.check(self._lib.lib().spec_shard_host_decode(self._h, stream.data_ptr(), stream.numel(),
                                                               ends.data_ptr(), n, op, bases),
                        "spec_shard_host_decode")
        return list(bases)

    def sync(self):
        self._lib.check(self._lib.lib().spec_shard_sync(self._h), "spec_shard_sync")
        self._inflight = []
