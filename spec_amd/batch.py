"""Batch encode/decode of flat spec messages on the GPU (host side of include/spec_amd.h).

The reference has no batch API; its callers loop over records:

    for each record b:                       # internal/bench/parse_test.go:48-111
        m, err := spec.OpenMessageErr(b)     # msg.go:25-27
        v_f = m.<Kind_f>(tag_f)              # internal/types/msg.go:219-475

    for each record:                         # internal/bench/write_test.go:16-78
        w := spec.NewMessageWriterBuffer(buf)   # writer_msg.go:26-31
        w.Field(tag_f).<Kind_f>(v_f) ...        # internal/writer/msg.go:99-211
        w.Build()                               # internal/writer/msg.go:56-60

`decode_flat` / `encode_flat` run those loops for a whole batch held in HBM with one
launch sequence each.  Device memory and streams come from torch; the compute is the HIP
code in libspec_amd.so.  Nothing here falls back to a CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .schema import NP_DTYPE, VARLEN, Kind, Schema


def _stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _ptr(t: torch.Tensor | None):
    return C.c_void_p(t.data_ptr() if t is not None else 0)


def _check_dev(t: torch.Tensor, name: str, dtype=None):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")


@dataclass
class Columns:
    """Decoded SoA columns: one uint8 tensor [n, width] per schema field + status [n]."""
    schema: Schema
    cols: list
    status: torch.Tensor | None

    def numpy(self, f: int) -> np.ndarray:
        """Column f as a numpy array of its natural dtype (bins: [n, w] uint8; spans: [n, 2])."""
        kind = self.schema.fields[f].kind
        a = self.cols[f].cpu().numpy()
        if kind in (Kind.BIN64, Kind.BIN128, Kind.BIN256):
            return a
        v = a.view(NP_DTYPE[kind])
        return v.reshape(len(a), 2) if kind in VARLEN else v.reshape(len(a))


def alloc_columns(schema: Schema, n: int, device="cuda"):
    return [torch.empty((n, w), dtype=torch.uint8, device=device) for w in schema.widths]


def decode_flat(schema: Schema, stream: torch.Tensor, ends: torch.Tensor, *, cols=None,
                status: bool | torch.Tensor = True, cuda_stream=None) -> Columns:
    """spec_decode_flat: OpenMessageErr + one getter per field for every record.

    stream: uint8 [stream_len] device tensor (records back to back)
    ends:   int64 [n] device tensor, exclusive end offset of each record
    """
    _check_dev(stream, "stream", torch.uint8)
    _check_dev(ends, "ends", torch.int64)
    n = ends.numel()
    if cols is None:
        cols = alloc_columns(schema, n, stream.device)
    st = None
    if isinstance(status, torch.Tensor):
        st = status
    elif status:
        st = torch.empty(n, dtype=torch.uint8, device=stream.device)
    ptrs = (C.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
    rc = _lib.lib().spec_decode_flat(C.byref(schema.c), _ptr(stream), stream.numel(), _ptr(ends), n,
                                     ptrs, _ptr(st), _stream_handle(cuda_stream))
    _lib.check(rc, "spec_decode_flat")
    return Columns(schema, cols, st)


def decode_flat_errors(schema: Schema, stream: torch.Tensor, ends: torch.Tensor, cuda_stream=None):
    """spec_decode_flat_errors: decode_flat plus the per-record field error mask (bit f: field f's
    <Kind>Err getter errs, internal/types/msg.go:233-459) -> (Columns, errmask int64 [n]); a schema
    of more than 64 fields gets errmask int64 [ceil(nfields / 64), n] (row c: fields 64c..64c+63)."""
    _check_dev(stream, "stream", torch.uint8)
    _check_dev(ends, "ends", torch.int64)
    n = ends.numel()
    cols = alloc_columns(schema, n, stream.device)
    st = torch.empty(n, dtype=torch.uint8, device=stream.device)
    words = max(1, (len(schema) + 63) // 64)
    em = torch.empty((words, max(n, 1)), dtype=torch.int64, device=stream.device)
    ptrs = (C.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
    rc = _lib.lib().spec_decode_flat_errors(C.byref(schema.c), _ptr(stream), stream.numel(), _ptr(ends), n, ptrs,
                                             _ptr(st), _ptr(em), _stream_handle(cuda_stream))
    _lib.check(rc, "spec_decode_flat_errors")
    return Columns(schema, cols, st), (em[0, :n] if words == 1 else em[:, :n])


class Decoder:
    """Pre-bound spec_decode_flat call (arguments marshalled once) for repeated launches."""

    def __init__(self, schema: Schema, stream: torch.Tensor, ends: torch.Tensor, cols=None,
                 status: torch.Tensor | None = None, cuda_stream=None):
        _check_dev(stream, "stream", torch.uint8)
        _check_dev(ends, "ends", torch.int64)
        n = ends.numel()
        self.schema, self.stream, self.ends = schema, stream, ends
        self.cols = cols if cols is not None else alloc_columns(schema, n, stream.device)
        self.status = status if status is not None else torch.empty(n, dtype=torch.uint8, device=stream.device)
        self._ptrs = (C.c_void_p * max(1, len(self.cols)))(*[c.data_ptr() for c in self.cols])
        self._args = (C.byref(schema.c), _ptr(stream), stream.numel(), _ptr(ends), n, self._ptrs,
                      _ptr(self.status), _stream_handle(cuda_stream))
        self._fn = _lib.lib().spec_decode_flat

    def __call__(self):
        rc = self._fn(*self._args)
        if rc:
            _lib.check(rc, "spec_decode_flat")

    def result(self) -> Columns:
        return Columns(self.schema, self.cols, self.status)


class Encoder:
    """Reusable encode state (workspace + total) for one schema and batch size."""

    def __init__(self, schema: Schema, n: int, device="cuda"):
        self.schema = schema
        self.n = n
        ws = _lib.lib().spec_encode_flat_workspace_size(n)
        self.workspace = torch.empty((ws + 7) // 8, dtype=torch.int64, device=device)
        self.ws_bytes = ws
        self.total = torch.zeros(1, dtype=torch.int64, device=device)

    def _colptrs(self, cols):
        if len(cols) != len(self.schema):
            raise ValueError("one column per schema field")
        for i, c in enumerate(cols):
            _check_dev(c, f"column {i}")
            if c.numel() * c.element_size() < self.n * self.schema.fields[i].width:
                raise ValueError(f"column {i} too small")
        return (C.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])

    def size(self, cols, cuda_stream=None) -> torch.Tensor:
        """Sizing passes only; returns the device total (int64[1])."""
        rc = _lib.lib().spec_encode_flat_size(C.byref(self.schema.c), self._colptrs(cols), self.n,
                                              _ptr(self.workspace), self.ws_bytes, _ptr(self.total),
                                              _stream_handle(cuda_stream))
        _lib.check(rc, "spec_encode_flat_size")
        return self.total

    def encode_into(self, cols, heaps: dict, out: torch.Tensor, ends: torch.Tensor, cuda_stream=None):
        """All passes; writes out[:total], ends[n] and self.total (device)."""
        _check_dev(out, "out", torch.uint8)
        _check_dev(ends, "ends", torch.int64)
        nf = len(self.schema)
        hp = (C.c_void_p * max(1, nf))()
        hl = (C.c_uint64 * max(1, nf))()
        keep = []
        for f, fld in enumerate(self.schema.fields):
            if fld.kind in VARLEN:
                h = heaps[f]
                _check_dev(h, f"heap {f}", torch.uint8)
                keep.append(h)
                hp[f] = h.data_ptr()
                hl[f] = h.numel()
        rc = _lib.lib().spec_encode_flat(C.byref(self.schema.c), self._colptrs(cols), hp, hl, self.n,
                                         _ptr(out), out.numel(), _ptr(ends), _ptr(self.workspace),
                                         self.ws_bytes, _ptr(self.total), _stream_handle(cuda_stream))
        _lib.check(rc, "spec_encode_flat")


def encode_flat(schema: Schema, cols, heaps: dict, n: int | None = None, cuda_stream=None):
    """Encode a batch -> (stream uint8[total], ends int64[n]) on the device."""
    if n is None:
        n = cols[0].shape[0] if cols else 0
    dev = cols[0].device if cols else torch.device("cuda")
    enc = Encoder(schema, n, dev)
    total = int(enc.size(cols, cuda_stream).item())
    if total < 0:  # ~0: an encoder error (string/bytes span outside its heap or > MaxSize)
        raise _lib.SpecError(-1, "spec_encode_flat: encoder error")
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    ends = torch.empty(n, dtype=torch.int64, device=dev)
    enc.encode_into(cols, heaps, out, ends, cuda_stream)
    if int(enc.total.item()) != total:  # heap-range check failed in the full pass
        raise _lib.SpecError(-1, "spec_encode_flat: encoder error (span outside its heap)")
    return out[:total], ends


PARSE_MESSAGE, PARSE_LIST, PARSE_VALUE = 0, 1, 2  # include/spec_amd.h SPEC_PARSE_*


def parse_messages(stream: torch.Tensor, ends: torch.Tensor, head: int = 0, sizes: bool = True, cuda_stream=None,
                   root: int = PARSE_MESSAGE):
    """spec_parse_batch: spec.ParseMessage (root PARSE_MESSAGE), ParseList (PARSE_LIST) or
    ParseValue (PARSE_VALUE) — recursive validation — of every record.
    Returns (status uint8 [n], sizes int32 view of uint32 [n] or None)."""
    _check_dev(stream, "stream", torch.uint8)
    _check_dev(ends, "ends", torch.int64)
    n = ends.numel()
    st = torch.empty(n, dtype=torch.uint8, device=stream.device)
    sz = torch.empty(n, dtype=torch.int32, device=stream.device) if sizes else None
    rc = _lib.lib().spec_parse_batch(root, _ptr(stream), stream.numel(), _ptr(ends), n, head, _ptr(st), _ptr(sz),
                                     _stream_handle(cuda_stream))
    _lib.check(rc, "spec_parse_batch")
    return st, sz
