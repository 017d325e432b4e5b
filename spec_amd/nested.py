"""Batch decode of messages with a list<message> field (include/spec_amd.h spec_decode_nested).

Per record this is what a generated reader does:

    m, err := spec.OpenMessageErr(b)                           # msg.go:25-27
    outer getters ...                                           # internal/types/msg.go:219-475
    items := spec.NewMessageList(m.msg.List(tag), OpenItemErr)  # list_msg.go:20-26
    for i := 0; i < items.Len(); i++ { it := items.Get(i); it.Key() ... }   # list_msg.go:88-92

Outer columns are [n]; items are stored in record order, record i owning
[item_begin[i], item_begin[i+1]).  Two launches sequences: index (item totals) then decode.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from . import _lib
from .batch import _check_dev, _ptr, _stream_handle, alloc_columns
from .schema import Kind, NestedSchema


@dataclass
class NestedColumns:
    schema: NestedSchema
    outer: list          # one uint8 [n, width] tensor per outer field (None for the list field)
    status: torch.Tensor
    item_begin: torch.Tensor  # int32 view of uint32 [n + 1]
    items: list          # one uint8 [m, width] tensor per item field
    item_status: torch.Tensor
    total_items: int


class NestedDecoder:
    """Workspace + total for one schema and batch; call index() then decode()."""

    def __init__(self, schema: NestedSchema, stream: torch.Tensor, ends: torch.Tensor, cuda_stream=None):
        _check_dev(stream, "stream", torch.uint8)
        _check_dev(ends, "ends", torch.int64)
        self.schema, self.stream, self.ends = schema, stream, ends
        self.n = ends.numel()
        L = _lib.lib()
        ws = L.spec_decode_nested_workspace_size(self.n)
        self.workspace = torch.empty((ws + 7) // 8, dtype=torch.int64, device=stream.device)
        self.ws_bytes = ws
        self.total = torch.zeros(1, dtype=torch.int64, device=stream.device)
        self.cuda_stream = cuda_stream
        dev = stream.device
        self.outer = [None if f.kind == Kind.LIST else torch.empty((self.n, f.width), dtype=torch.uint8, device=dev)
                      for f in schema.outer.fields]
        self.status = torch.empty(self.n, dtype=torch.uint8, device=dev)
        self.item_begin = torch.empty(self.n + 1, dtype=torch.int32, device=dev)
        self.items, self.item_status, self.item_cap = [], None, 0

    def index(self) -> torch.Tensor:
        rc = _lib.lib().spec_decode_nested_index(C.byref(self.schema.c), _ptr(self.stream), self.stream.numel(),
                                                 _ptr(self.ends), self.n, _ptr(self.workspace), self.ws_bytes,
                                                 _ptr(self.total), _stream_handle(self.cuda_stream))
        _lib.check(rc, "spec_decode_nested_index")
        return self.total

    def reserve(self, m: int):
        if m > self.item_cap:
            self.items = alloc_columns(self.schema.item, m, self.stream.device)
            self.item_status = torch.empty(max(m, 1), dtype=torch.uint8, device=self.stream.device)
            self.item_cap = m

    def decode(self):
        outer = (C.c_void_p * max(1, len(self.outer)))(*[c.data_ptr() if c is not None else 0 for c in self.outer])
        items = (C.c_void_p * max(1, len(self.items)))(*[c.data_ptr() for c in self.items])
        rc = _lib.lib().spec_decode_nested(C.byref(self.schema.c), _ptr(self.stream), self.stream.numel(),
                                           _ptr(self.ends), self.n, outer, _ptr(self.status), _ptr(self.item_begin),
                                           items, _ptr(self.item_status), self.item_cap, _ptr(self.workspace),
                                           self.ws_bytes, _stream_handle(self.cuda_stream))
        _lib.check(rc, "spec_decode_nested")

    def decode_onepass(self) -> torch.Tensor:
        """spec_decode_nested_onepass into the reserved item columns (no index call); returns the
        device total.  Items beyond the reserved capacity are not written: if total > capacity,
        reserve(total) and call again."""
        outer = (C.c_void_p * max(1, len(self.outer)))(*[c.data_ptr() if c is not None else 0 for c in self.outer])
        items = (C.c_void_p * max(1, len(self.items)))(*[c.data_ptr() for c in self.items])
        rc = _lib.lib().spec_decode_nested_onepass(
            C.byref(self.schema.c), _ptr(self.stream), self.stream.numel(), _ptr(self.ends), self.n, outer,
            _ptr(self.status), _ptr(self.item_begin), items, _ptr(self.item_status), self.item_cap,
            _ptr(self.workspace), self.ws_bytes, _ptr(self.total), _stream_handle(self.cuda_stream))
        _lib.check(rc, "spec_decode_nested_onepass")
        return self.total

    def result(self) -> NestedColumns:
        return NestedColumns(self.schema, self.outer, self.status, self.item_begin, self.items, self.item_status,
                             int(self.total.item()))


def decode_nested(schema: NestedSchema, stream: torch.Tensor, ends: torch.Tensor, cuda_stream=None,
                  onepass: bool = False, item_cap: int | None = None) -> NestedColumns:
    """Two-pass: index, size the item columns from the device total, decode.  onepass: decode
    into item_cap items (default 4 per record) in one pass; if the batch holds more, grow the
    item columns to the reported total and decode again."""
    d = NestedDecoder(schema, stream, ends, cuda_stream)
    if onepass:
        d.reserve(max(1, item_cap if item_cap is not None else 4 * d.n))
        total = int(d.decode_onepass().item())
        if total > d.item_cap:
            d.reserve(total)
            d.decode_onepass()
        return d.result()
    total = int(d.index().item())
    d.reserve(total)
    d.decode()
    return d.result()


class NestedEncoder:
    """Reusable encode state for spec_encode_nested (workspace + device total)."""

    def __init__(self, schema: NestedSchema, n: int, device="cuda"):
        self.schema, self.n = schema, n
        ws = _lib.lib().spec_encode_nested_workspace_size(n)
        self.workspace = torch.empty((ws + 7) // 8, dtype=torch.int64, device=device)
        self.ws_bytes = ws
        self.total = torch.zeros(1, dtype=torch.int64, device=device)

    @staticmethod
    def _ptrs(ts):
        return (C.c_void_p * max(1, len(ts)))(*[t.data_ptr() if t is not None else 0 for t in ts])

    @staticmethod
    def _heaps(fields, heaps):
        hp = (C.c_void_p * max(1, len(fields)))()
        hl = (C.c_uint64 * max(1, len(fields)))()
        for f, fld in enumerate(fields):
            if fld.kind in (Kind.STRING, Kind.BYTES):
                h = heaps[f]
                _check_dev(h, f"heap {f}", torch.uint8)
                hp[f] = h.data_ptr()
                hl[f] = h.numel()
        return hp, hl

    def encode(self, outer_cols, outer_heaps, item_begin, item_cols, item_heaps, nitems, out=None, ends=None,
               cuda_stream=None):
        """outer_cols: one tensor per outer field (None for the list field); item_begin: int32/uint32
        [n+1]; writes out/ends when given, always self.total."""
        ws = _lib.lib().spec_encode_nested_workspace_size_items(self.n, nitems)
        if ws > self.ws_bytes:  # room for the size pass's item prefixes (the write pass reuses them)
            self.workspace = torch.empty((ws + 7) // 8, dtype=torch.int64, device=self.workspace.device)
            self.ws_bytes = ws
        ohp, ohl = self._heaps(self.schema.outer.fields, outer_heaps)
        ihp, ihl = self._heaps(self.schema.item.fields, item_heaps)
        rc = _lib.lib().spec_encode_nested(
            C.byref(self.schema.c), self._ptrs(outer_cols), ohp, ohl, _ptr(item_begin), self._ptrs(item_cols), ihp,
            ihl, nitems, self.n, _ptr(out), out.numel() if out is not None else 0, _ptr(ends), _ptr(self.workspace),
            self.ws_bytes, _ptr(self.total), _stream_handle(cuda_stream))
        _lib.check(rc, "spec_encode_nested")
        return self.total


def encode_nested(schema: NestedSchema, outer_cols, outer_heaps, item_begin, item_cols, item_heaps, n: int,
                  cuda_stream=None):
    """-> (stream uint8[total], ends int64[n]) on the device."""
    dev = item_begin.device
    enc = NestedEncoder(schema, n, dev)
    nitems = item_cols[0].shape[0] if item_cols else 0
    total = int(enc.encode(outer_cols, outer_heaps, item_begin, item_cols, item_heaps, nitems,
                           cuda_stream=cuda_stream).item())
    if total < 0:
        raise _lib.SpecError(-1, "spec_encode_nested: encoder error")
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    ends = torch.empty(n, dtype=torch.int64, device=dev)
    enc.encode(outer_cols, outer_heaps, item_begin, item_cols, item_heaps, nitems, out, ends, cuda_stream)
    return out[:total], ends
