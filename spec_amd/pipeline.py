"""Host-resident batches: pinned host -> HBM -> decode -> host, pipelined in chunks.

The path's real source is host memory (mpx connection buffers, mpx/conn_reader.go:179-194),
so a receiver hands over a pinned buffer of records back to back plus their end offsets.
`HostDecoder` splits the batch into record chunks and overlaps, on three HIP streams, the
H2D copy of chunk k+1, the decode of chunk k (spec_decode_flat_range) and the D2H copy of
chunk k-1's outputs.

Output layout (chunk-major): chunk k's columns and status sit in ONE contiguous region —
field 0 of records [r0, r1), field 1, ..., status — in device memory and in the pinned host
mirror, so each chunk leaves the device in one copy instead of one per column.  (PCIe on
MI355X: ~57 GB/s per direction; the two directions only overlap when the copies are split into
chunks, and each extra copy costs launch time.)  `HostDecoder.chunk(k)` gives the chunk's
views, `columns()` gathers whole columns on the host.  Device buffers are allocated once.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .batch import _ptr
from .schema import Schema


def _align(x: int, a: int = 256) -> int:
    return (x + a - 1) // a * a


class HostDecoder:
    def __init__(self, schema: Schema, n: int, stream_cap: int, device="cuda", chunks: int = 16):
        self.schema, self.n = schema, n
        self.chunks = max(1, min(chunks, max(n, 1)))
        dev = torch.device(device)
        self.bounds = [n * k // self.chunks for k in range(self.chunks + 1)]
        widths = schema.widths
        # per chunk: [base, field offsets..., status offset, size] within the output region
        self.layout = []
        base = 0
        for k in range(self.chunks):
            nk = self.bounds[k + 1] - self.bounds[k]
            offs, o = [], 0
            for w in widths:
                offs.append(o)
                o = _align(o + w * nk)
            self.layout.append((base, offs, o, _align(o + nk)))
            base += _align(o + nk)
        self.out_bytes = max(base, 1)
        self.d_stream = torch.empty(max(stream_cap, 1), dtype=torch.uint8, device=dev)
        self.d_ends = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.d_out = torch.empty(self.out_bytes, dtype=torch.uint8, device=dev)
        self.h_out = torch.empty(self.out_bytes, dtype=torch.uint8, pin_memory=True)
        self.s_in = torch.cuda.Stream(dev)
        self.s_dec = torch.cuda.Stream(dev)
        self.s_out = torch.cuda.Stream(dev)
        # decode pointers: column f of chunk k shifted by -r0 rows, so record r lands at row r - r0
        dptr = self.d_out.data_ptr()
        self._ptrs = []
        for k, (cb, offs, soff, _) in enumerate(self.layout):
            r0 = self.bounds[k]
            cols = (C.c_void_p * max(1, len(widths)))(
                *[dptr + cb + offs[f] - r0 * widths[f] for f in range(len(widths))])
            self._ptrs.append((cols, C.c_void_p(dptr + cb + soff - r0)))

    def decode(self, h_stream: torch.Tensor, h_ends: torch.Tensor):
        """h_stream: pinned uint8 [stream_len]; h_ends: pinned int64 [n].  Returns the pinned
        output region once every chunk has landed (views: chunk(k), columns())."""
        n, L = self.n, _lib.lib()
        stream_len = h_stream.numel()
        ends_np = h_ends.numpy()
        for k in range(self.chunks):
            r0, r1 = self.bounds[k], self.bounds[k + 1]
            if r1 <= r0:
                continue
            b0 = int(ends_np[r0 - 1]) if r0 else 0
            b1 = int(ends_np[r1 - 1])
            ev_in, ev_dec = torch.cuda.Event(), torch.cuda.Event()
            with torch.cuda.stream(self.s_in):
                self.d_ends[r0:r1].copy_(h_ends[r0:r1], non_blocking=True)
                if b1 > b0:
                    self.d_stream[b0:b1].copy_(h_stream[b0:b1], non_blocking=True)
                ev_in.record(self.s_in)
            self.s_dec.wait_event(ev_in)
            cols, status = self._ptrs[k]
            rc = L.spec_decode_flat_range(C.byref(self.schema.c), _ptr(self.d_stream), stream_len,
                                          _ptr(self.d_ends), r0, r1, b1 - b0, cols, status,
                                          C.c_void_p(self.s_dec.cuda_stream))
            _lib.check(rc, "spec_decode_flat_range")
            ev_dec.record(self.s_dec)
            self.s_out.wait_event(ev_dec)
            cb, _, _, size = self.layout[k]
            with torch.cuda.stream(self.s_out):
                self.h_out[cb:cb + size].copy_(self.d_out[cb:cb + size], non_blocking=True)
        self.s_out.synchronize()
        return self.h_out

    def chunk(self, k: int):
        """(r0, r1, [host column views [r1-r0, width]], host status view) of chunk k."""
        r0, r1 = self.bounds[k], self.bounds[k + 1]
        nk = r1 - r0
        cb, offs, soff, _ = self.layout[k]
        cols = [self.h_out[cb + o:cb + o + w * nk].view(nk, w) for o, w in zip(offs, self.schema.widths)]
        return r0, r1, cols, self.h_out[cb + soff:cb + soff + nk]

    def columns(self):
        """Whole host columns + status, gathered from the chunks (a host copy)."""
        parts = [self.chunk(k) for k in range(self.chunks)]
        cols = [torch.cat([p[2][f] for p in parts]) for f in range(len(self.schema.widths))]
        return cols, torch.cat([p[3] for p in parts])
