"""Host-resident batches: pinned host -> HBM -> decode -> host, pipelined in chunks.

The path's real source is host memory (mpx connection buffers, mpx/conn_reader.go:179-194),
so a receiver hands over a pinned buffer of records back to back plus their end offsets.
`HostDecoder` splits the batch into record chunks and overlaps, on three HIP streams, the
H2D copy of chunk k+1, the decode of chunk k (spec_decode_flat_range) and the D2H copy of
chunk k-1's columns.  Device buffers are allocated once and reused.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .batch import _ptr, alloc_columns
from .schema import Schema


class HostDecoder:
    def __init__(self, schema: Schema, n: int, stream_cap: int, device="cuda", chunks: int = 8):
        self.schema, self.n, self.chunks = schema, n, max(1, chunks)
        dev = torch.device(device)
        self.d_stream = torch.empty(max(stream_cap, 1), dtype=torch.uint8, device=dev)
        self.d_ends = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.d_cols = alloc_columns(schema, max(n, 1), dev)
        self.d_status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.h_cols = [torch.empty(c.shape, dtype=torch.uint8, pin_memory=True) for c in self.d_cols]
        self.h_status = torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=True)
        self.s_in = torch.cuda.Stream(dev)
        self.s_dec = torch.cuda.Stream(dev)
        self.s_out = torch.cuda.Stream(dev)
        self._colptrs = (C.c_void_p * max(1, len(self.d_cols)))(*[c.data_ptr() for c in self.d_cols])

    def decode(self, h_stream: torch.Tensor, h_ends: torch.Tensor, ends_list=None):
        """h_stream: pinned uint8 [stream_len]; h_ends: pinned int64 [n].  Returns (host columns,
        host status) once everything has landed.  ends_list: the chunk byte bounds if known."""
        n, L = self.n, _lib.lib()
        stream_len = h_stream.numel()
        bounds = [n * k // self.chunks for k in range(self.chunks + 1)]
        ends_np = h_ends.numpy()
        evs = []
        for k in range(self.chunks):
            r0, r1 = bounds[k], bounds[k + 1]
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
            rc = L.spec_decode_flat_range(C.byref(self.schema.c), _ptr(self.d_stream), stream_len,
                                          _ptr(self.d_ends), r0, r1, b1 - b0, self._colptrs, _ptr(self.d_status),
                                          C.c_void_p(self.s_dec.cuda_stream))
            _lib.check(rc, "spec_decode_flat_range")
            ev_dec.record(self.s_dec)
            self.s_out.wait_event(ev_dec)
            with torch.cuda.stream(self.s_out):
                for h, d in zip(self.h_cols, self.d_cols):
                    h[r0:r1].copy_(d[r0:r1], non_blocking=True)
                self.h_status[r0:r1].copy_(self.d_status[r0:r1], non_blocking=True)
            evs.append(ev_dec)
        self.s_out.synchronize()
        return self.h_cols, self.h_status
