"""Host-resident batches: pinned host -> HBM -> decode -> host, pipelined in chunks.

The path's real source is host memory (mpx connection buffers, mpx/conn_reader.go:179-194),
so a receiver hands over a pinned buffer of records back to back plus their end offsets.
`HostDecoder` wraps the native pipeline of the C ABI (spec_host_decoder_*,
spec_amd/csrc/host_pipeline.cpp): the batch is split into record chunks and three HIP
streams overlap the H2D copy of chunk k+1, the decode of chunk k and the D2H copy of chunk
k-1's outputs.

Output layout (chunk-major): chunk k's columns and status sit in ONE contiguous region —
field 0 of records [r0, r1), field 1, ..., status — so each chunk leaves the device in one
copy instead of one per column (PCIe on MI355X: ~57 GB/s per direction; the two directions
overlap only when the traffic is split into chunks, and each copy costs a launch).
`chunk(k)` gives the chunk's views, `columns()` gathers whole columns on the host.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .batch import _ptr
from .schema import Schema


class HostDecoder:
    def __init__(self, schema: Schema, n: int, stream_cap: int, device="cuda", chunks: int = 8):
        self.schema, self.n = schema, n
        self.chunks = max(1, min(chunks, max(n, 1)))
        dev = torch.device(device)
        L = _lib.lib()
        h = C.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(L.spec_host_decoder_create(C.byref(schema.c), n, stream_cap, self.chunks, C.byref(h)),
                       "spec_host_decoder_create")
        self._h = h
        self.out_bytes = int(L.spec_host_decoder_out_bytes(h, n))
        self.h_out = torch.empty(max(self.out_bytes, 1), dtype=torch.uint8, pin_memory=True)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.lib().spec_host_decoder_destroy(h)
            self._h = None

    def decode(self, h_stream: torch.Tensor, h_ends: torch.Tensor):
        """h_stream: pinned uint8 [stream_len]; h_ends: pinned int64 [n].  Synchronous: returns
        the pinned output region once every chunk has landed (views: chunk(k), columns())."""
        if h_ends.numel() != self.n:
            raise ValueError("h_ends must hold n end offsets")
        rc = _lib.lib().spec_host_decoder_run(self._h, _ptr(h_stream), h_stream.numel(), _ptr(h_ends), self.n,
                                              _ptr(self.h_out))
        _lib.check(rc, "spec_host_decoder_run")
        return self.h_out

    def chunk(self, k: int):
        """(r0, r1, [host column views [r1-r0, width]], host status view) of chunk k."""
        r0, r1, so = C.c_uint64(), C.c_uint64(), C.c_uint64()
        offs = (C.c_uint64 * max(1, len(self.schema.widths)))()
        _lib.check(_lib.lib().spec_host_decoder_chunk(self._h, self.n, k, C.byref(r0), C.byref(r1), offs,
                                                      C.byref(so)), "spec_host_decoder_chunk")
        nk = r1.value - r0.value
        cols = [self.h_out[o:o + w * nk].view(nk, w) for o, w in zip(offs, self.schema.widths)]
        return r0.value, r1.value, cols, self.h_out[so.value:so.value + nk]

    def columns(self):
        """Whole host columns + status, gathered from the chunks (a host copy)."""
        parts = [self.chunk(k) for k in range(self.chunks)]
        cols = [torch.cat([p[2][f] for p in parts]) for f in range(len(self.schema.widths))]
        return cols, torch.cat([p[3] for p in parts])
